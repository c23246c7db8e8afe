#!/bin/bash
# GF(2^16) register encoder at k=512: timing by diagnostic mode (0 encode, 1 loads + stores only, 2 no loads,
# 3 no loads and no stores) and one SQ PMC pass of the encode mode.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/rs16d
mkdir -p "$OUT"
for m in 0 1 2 3; do
  echo "mode $m $(CDA_LIB=ab/libcda_rs16m$m.so timeout -k 10 120 python3 -u scripts/rs16_probe.py 20)" || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU --kernel-trace --output-format csv -d "$OUT/sq" -o run -- python3 $R/scripts/rs16_probe.py 5 > "$OUT/sq.log" 2>&1 || exit 1
python3 $R/scripts/pmc_table.py "$OUT/sq/run_counter_collection.csv" rs_encode16
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/lds" -o run -- python3 $R/scripts/rs16_probe.py 5 > "$OUT/lds.log" 2>&1 || exit 1
python3 $R/scripts/pmc_table.py "$OUT/lds/run_counter_collection.csv" rs_encode16

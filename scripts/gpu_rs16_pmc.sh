#!/bin/bash
# GF(2^16) register encoder at k=512: instruction-cache and SQ counters of the current build (scripts/rs16_probe.py).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/rs16p
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
P="python3 $R/scripts/rs16_probe.py 5"
step() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 $R/scripts/pmc_table.py "$OUT/$name/run_counter_collection.csv" rs_encode16
  return 0
}
step ic --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --kernel-trace --output-format csv -d "$OUT/ic" -o run -- $P
step sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/sq" -o run -- $P

#!/bin/bash
# Final GF(2^16) encoder at k=512: kernel trace + SQ / LDS / HBM counter passes of scripts/rs16_probe.py.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/rs16f
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
P="python3 $R/scripts/rs16_probe.py 5"
step() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc
  return 0
}
step trace --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $P
step sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/sq" -o run -- $P
step lds --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU --kernel-trace --output-format csv -d "$OUT/lds" -o run -- $P
step fetch --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o run -- $P
step write --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o run -- $P

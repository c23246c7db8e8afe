#!/bin/bash
# GF(2^16) register encoder at k=512: timing, then PMC passes that separate instruction-fetch stalls from
# dependency stalls (the kernel is ~75 KB of straight-line code).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/rs16ic
mkdir -p "$OUT"
timeout -k 10 120 python3 -u scripts/rs16_probe.py 20 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1
echo "list rc=$?"
step() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -ge 124 ] && exit $rc
  return 0
}
P="python3 $R/scripts/rs16_probe.py 5"
step pmc1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_IFETCH SQ_INSTS_SALU --kernel-trace --output-format csv -d "$OUT/pmc1" -o run -- $P
step pmc2 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --kernel-trace --output-format csv -d "$OUT/pmc2" -o run -- $P
step pmc3 --pmc SQ_IFETCH_LEVEL SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/pmc3" -o run -- $P

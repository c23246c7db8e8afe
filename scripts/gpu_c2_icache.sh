#!/bin/bash
# Config C2 (one k=128 block): latency probe, then instruction-cache and issue counters of its kernels.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/c2ic
mkdir -p "$OUT"
timeout -k 10 120 python3 -u scripts/c2_probe.py 2>/dev/null || exit $?
cd /tmp && export TMPDIR=/tmp
step() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 $R/scripts/pmc_table.py "$OUT/$name/run_counter_collection.csv" trees_lds leaf_hash rs_encode8 dah
  return 0
}
P="python3 $R/scripts/c2_probe.py"
step ic --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --kernel-trace --output-format csv -d "$OUT/ic" -o run -- $P
step sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/sq" -o run -- $P

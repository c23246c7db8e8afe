#!/bin/bash
# rocprofv3 evidence for the bench step: kernel trace + stats, then PMC passes
# (each counter group in its own run, no sys/runtime trace with --pmc).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof
TAG=${1:-r01}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras --no-k512-split ${BENCH_ARGS:-}"
step() {  # name timeout args...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" rocprofv3 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 5 "$OUT/$name.log"
  if [ $rc -ge 124 ]; then echo "ABORT"; exit $rc; fi
}
timeout -k 5 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
step trace 300 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $BENCH
step pmc_fetch 300 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 $BENCH
step pmc_write 300 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write" -o run -- python3 $BENCH
step pmc_valu 300 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/pmc_valu" -o run -- python3 $BENCH
step pmc_valu2 300 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/pmc_valu2" -o run -- python3 $BENCH
step pmc_lds 300 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM --kernel-trace --output-format csv -d "$OUT/pmc_lds" -o run -- python3 $BENCH
find "$OUT" -name "*.csv" | head -50

#!/bin/bash
# Round 3, GPU session B: the C-ABI split (replicas G = 1..8 on one GPU) and its k=512 timing.
set -u
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run split_tests 600 python -u -m pytest tests/test_split_capi_gpu.py tests/test_faults_gpu.py -x -v --timeout 300 --timeout-method thread
run k512 300 python -u scripts/k512_split_probe.py 5

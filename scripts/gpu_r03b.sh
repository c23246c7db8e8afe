#!/bin/bash
# Round 3, GPU session B: the C-ABI split (replicas G = 1..8 on one GPU), the register GF(2^16) encoder's parity,
# and config C5 timings (register encoder vs the LDS encoder, CDA_RS16=lds).
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
run ff16_tests 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "ff16 or matches_oracle or digests or repair_ff16"
run split_tests 600 python -u -m pytest tests/test_split_capi_gpu.py tests/test_faults_gpu.py -x -q --timeout 300 --timeout-method thread
run k512 300 python -u scripts/k512_split_probe.py 5
run k512_lds 300 env CDA_RS16=lds python -u scripts/k512_split_probe.py 5

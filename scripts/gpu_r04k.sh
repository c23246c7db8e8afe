#!/bin/bash
# Consensus path, fresh output: first touch by MADV_POPULATE_WRITE (default) vs touch loops (CDA_CONS_TOUCH=1);
# consensus GPU tests first.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_consensus_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04k_tests.log 2>&1
rc=$?; tail -n 2 gpurun_out/r04k_tests.log; [ $rc -ne 0 ] && exit $rc
for v in "CDA_CONS_TOUCH=0" "CDA_CONS_TOUCH=1" "CDA_CONS_TOUCH=0" "CDA_CONS_TOUCH=1"; do
  env $v timeout -k 10 300 python -u scripts/consensus_probe.py 20 > gpurun_out/r04k_probe.log 2>&1
  rc=$?; echo "== $v $(grep '^{' gpurun_out/r04k_probe.log)"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r04k_probe.log; exit $rc; }
done

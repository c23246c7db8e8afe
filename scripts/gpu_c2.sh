#!/bin/bash
# Small-batch tree path: full GPU parity suite, then C2 / small-batch latency with and without it.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 4 gpurun_out/c2_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 120 python -u scripts/c2_trees_probe.py 2>/dev/null || exit $?
  CDA_TREES_LDS=0 timeout -k 10 120 python -u scripts/c2_trees_probe.py 2>/dev/null || exit $?
done

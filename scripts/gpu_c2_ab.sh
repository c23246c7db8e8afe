#!/bin/bash
# Config C2 A/B: the whole GPU parity suite on the current libcda, then the C2 latency probe for each library given,
# in rotating order.  usage: scripts/gpu_c2_ab.sh <lib.so> [<lib.so> ...]
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c2ab_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/c2ab_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for lib in "$@"; do
    echo "$lib $(CDA_LIB=$lib timeout -k 10 120 python scripts/c2_probe.py 2>/dev/null)" || exit 1
  done
done

#!/bin/bash
# FF8 XCD-contiguous mapping (ab/libcda_c.so) vs HEAD (a): GPU parity on c, bench A/B; then C2 latency of the leaf
# prefetch build (ab/libcda_pf.so) vs a.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/combo2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 2 gpurun_out/combo2_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 bash scripts/ab_bench.sh 3 ab/libcda_a.so ab/libcda_c.so || exit $?
for i in 1 2; do
  for lib in ab/libcda_a.so ab/libcda_pf.so; do
    echo "$lib $(CDA_LIB=$lib timeout -k 10 120 python scripts/c2_probe.py 2>/dev/null | cut -c1-200)" || exit 1
  done
done

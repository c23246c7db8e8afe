#!/bin/bash
# round 4: level kernel holding the node's namespace words (no end re-read of the children): parity of both
# variants (v1: 4 waves/SIMD forced, 3 VGPRs spilled; v2: 133 VGPRs, 3 waves/SIMD) on the tree tests, then a
# rotating A/B bench against the previous build.
set -u
mkdir -p gpurun_out
for v in v1 v2; do
  CDA_LIB=ab/libcda_$v.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04u_tests_$v.log 2>&1
  rc=$?; echo "tests $v rc=$rc"; tail -n 1 gpurun_out/r04u_tests_$v.log; [ $rc -ne 0 ] && exit $rc
done
bash scripts/ab_bench.sh 3 ab/libcda_v1.so ab/libcda_v2.so ab/libcda_prev.so

#!/bin/bash
# Leaf-prefetch A/B (bench, rotating order) after the GPU parity suite, then the FF8 memory-only diagnostic.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/combo_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/combo_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 bash scripts/ab_bench.sh 3 ab/libcda_a.so ab/libcda_b.so || exit $?
bash scripts/gpu_rs8_diag.sh
bash scripts/gpu_rs16_pmc.sh

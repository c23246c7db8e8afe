#!/bin/bash
# Parity of the RS paths on the current libcda, then a rotating A/B of ab/libcda_a.so vs ab/libcda_b.so.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/parity.log 2>&1
rc=$?; tail -n 3 gpurun_out/parity.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 bash scripts/ab_bench.sh ${ROUNDS:-3} ab/libcda_a.so ab/libcda_b.so

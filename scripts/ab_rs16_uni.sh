#!/bin/bash
set -u
mkdir -p gpurun_out
CDA_LIB=$PWD/celestia-app_amd/cda/libcda_uni.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -k "ff16 or 512" --timeout 120 --timeout-method thread > gpurun_out/uni_tests.log 2>&1; rc=$?; tail -2 gpurun_out/uni_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  echo "base"; timeout -k 10 60 python3 -u scripts/rs16_probe.py 20 || exit $?
  echo "uni"; CDA_LIB=$PWD/celestia-app_amd/cda/libcda_uni.so timeout -k 10 60 python3 -u scripts/rs16_probe.py 20 || exit $?
done

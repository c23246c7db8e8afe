#!/bin/bash
# GF(2^16) half-slice encoder (two workgroups per CU): GPU suite, then same-box A/B of the RS passes at k=512 against
# the whole-codeword kernel (ab/libcda_h2off.so: make -C celestia-app_amd BUILD=build_h2off
# OUT=../ab/libcda_h2off.so EXTRA=-DCDA_RS16_H2=0).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04f_tests.log 2>&1
rc=$?; tail -n 5 gpurun_out/r04f_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for lib in celestia-app_amd/cda/libcda.so ab/libcda_h2off.so; do
    echo "$lib $(CDA_LIB=$lib timeout -k 10 120 python3 scripts/rs16_probe.py 20 2>/dev/null)" || exit 1
  done
done

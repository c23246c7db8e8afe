#!/bin/bash
# GF(2^16) half-slice encoder with the dynamic item queue: GPU suite; product vs whole-codeword (h2off),
# memory-only (h2m1), compute-only (h2m3); the phase trace (h2tr).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04g_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/r04g_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for lib in celestia-app_amd/cda/libcda.so ab/libcda_h2off.so ab/libcda_h2m1.so ab/libcda_h2m3.so; do
    echo "$lib $(CDA_LIB=$lib timeout -k 10 120 python3 scripts/rs16_probe.py 20 2>/dev/null)" || exit 1
  done
done
CDA_LIB=ab/libcda_h2tr.so timeout -k 10 120 python3 scripts/h2_trace_probe.py

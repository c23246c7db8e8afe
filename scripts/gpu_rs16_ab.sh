#!/bin/bash
# GF(2^16) encoder A/B: parity tests of the GF(2^16) paths on the current libcda, then the RS-only probe
# (scripts/rs16_probe.py) for each library given, in rotating order.
# usage: scripts/gpu_rs16_ab.sh <lib.so> [<lib.so> ...]
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "rs_ or codec or k512 or 256 or 512 or split or decode" > gpurun_out/rs16_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/rs16_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for lib in "$@"; do
    echo "$lib $(CDA_LIB=$lib timeout -k 10 120 python scripts/rs16_probe.py 20)" || exit 1
  done
done

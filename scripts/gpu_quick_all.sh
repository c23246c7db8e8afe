#!/bin/bash
# Whole GPU parity suite on the current libcda, then the C5 probe.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/quick_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 2 gpurun_out/quick_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/k512_probe.py 2>/dev/null | cut -c1-900

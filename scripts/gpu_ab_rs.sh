#!/bin/bash
# RS encoder variant check: parity tests of the extension/codec paths with the in-tree build, then an A/B of
# library builds (scripts/ab_bench.sh).  usage: scripts/gpu_ab_rs.sh <rounds> <lib.so>...
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "extend or rs_ or codec or mainnet or batch" > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/ab_tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_bench.sh "$@"

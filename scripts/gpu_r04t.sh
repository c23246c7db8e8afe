#!/bin/bash
# round 4: leaf shares read one 128-B line at a time.  GPU suite on the new library, rotating A/B bench against the
# previous build (ab/libcda_prev.so), then the read-request-size PMC pass on the new library.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04t_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 2 gpurun_out/r04t_tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_bench.sh 3 celestia-app_amd/cda/libcda.so ab/libcda_prev.so || exit 1
bash scripts/gpu_r04s.sh

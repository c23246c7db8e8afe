#!/bin/bash
# Quick GPU iteration: a test subset (pytest -k expression) and a short bench without extras.
set -u
mkdir -p gpurun_out
K=${1:-"extend or batch or rs_ or codec or repair"}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/quick_tests.log 2>&1
rc=$?; tail -n 5 gpurun_out/quick_tests.log; [ $rc -ge 124 ] && exit $rc
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/quick_bench.log 2>&1
rc=$?; python3 -c "
import json
for l in open('gpurun_out/quick_bench.log'):
    if l.startswith('{'):
        d=json.loads(l); print('value', d['value'], 'ms/step', d['ms_per_step'], 'kernels', d['kernels_ms'], 'frac', d['roofline']['frac'])
" ; exit $rc

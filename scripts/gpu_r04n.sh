#!/bin/bash
# Full-lane small tree levels / DAH fold: GPU suite, C2 probe, trees phase trace, short bench.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04n_tests.log 2>&1
rc=$?; tail -n 2 gpurun_out/r04n_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do echo "c2 $(timeout -k 10 120 python3 scripts/c2_probe.py 2>/dev/null)" || exit 1; done
CDA_LIB=ab/libcda_ttr.so timeout -k 10 120 python3 scripts/trees_trace_probe.py || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-extras --no-cpu-baseline --no-k512-split > gpurun_out/r04n_bench.log 2>&1
rc=$?; grep '^{' gpurun_out/r04n_bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["kernels_ms"])'; exit $rc

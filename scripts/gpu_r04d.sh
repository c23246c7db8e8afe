#!/bin/bash
# round 4 final pass (part 1): the GPU suite, smoke, then the default bench line (extras + cpu_baseline) as the driver
# runs it, and the consensus probe on the same box.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04d_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/r04d_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04d_smoke.log 2>&1
rc=$?; tail -n 3 gpurun_out/r04d_smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r04d_bench.log 2>&1
rc=$?; grep '^{' gpurun_out/r04d_bench.log | cut -c1-300; [ $rc -ne 0 ] && { tail -5 gpurun_out/r04d_bench.log; exit $rc; }
timeout -k 10 300 python -u scripts/consensus_probe.py 20 > gpurun_out/r04d_probe.log 2>&1
rc=$?; grep '^{' gpurun_out/r04d_probe.log; exit $rc

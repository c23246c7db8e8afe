#!/bin/bash
# Consensus path: part of a pageable bottom half staged through the pinned slab on the second stream
# (CDA_CONS_STG = MiB) vs all pageable; consensus GPU tests with the staged form first.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_consensus_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04l_tests.log 2>&1
rc=$?; tail -n 2 gpurun_out/r04l_tests.log; [ $rc -ne 0 ] && exit $rc
for v in "CDA_CONS_TRACE=" "CDA_CONS_STG=0" "CDA_CONS_TRACE=" "CDA_CONS_STG=0"; do
  env $v timeout -k 10 300 python -u scripts/consensus_probe.py 20 > gpurun_out/r04l_probe.log 2>&1
  rc=$?; echo "== $v $(grep '^{' gpurun_out/r04l_probe.log)"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r04l_probe.log; exit $rc; }
done

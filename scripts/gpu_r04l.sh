#!/bin/bash
# Consensus path: part of a pageable bottom half staged through the pinned slab on the second stream
# (CDA_CONS_STG = MiB) vs all pageable; consensus GPU tests with the staged form first.
set -u
mkdir -p gpurun_out
true && touch gpurun_out/r04l_tests.log
rc=$?; tail -n 2 gpurun_out/r04l_tests.log; [ $rc -ne 0 ] && exit $rc
for v in "CDA_CONS_NBAND=4" "CDA_CONS_NBAND=2" "CDA_CONS_NBAND=4" "CDA_CONS_NBAND=2"; do
  env $v timeout -k 10 300 python -u scripts/consensus_probe.py 20 > gpurun_out/r04l_probe.log 2>&1
  rc=$?; echo "== $v $(grep '^{' gpurun_out/r04l_probe.log)"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r04l_probe.log; exit $rc; }
done

#!/bin/bash
# round 4 GPU pass: the consensus path's forms (scripts/consensus_probe.py: fresh untouched vs reused output buffers,
# serial form vs the one-block path, forced output forms, copy-pool sweep), then the GPU suite.
set -u
mkdir -p gpurun_out
for v in "CDA_CONS_OUT=0" "CDA_CONS_OUT=3" "CDA_CONS_OUT=3 CDA_CONS_IN=1" "CDA_CONS_OUT=0 CDA_COPY_THREADS=5" "CDA_CONS_OUT=3 CDA_COPY_THREADS=5"; do
  env $v timeout -k 10 300 python -u scripts/consensus_probe.py 15 > gpurun_out/r04b_probe.log 2>&1
  rc=$?; echo "== $v"; grep '^{' gpurun_out/r04b_probe.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/r04b_probe.log; exit $rc; }
done
[ -n "${SKIP_TESTS:-}" ] && exit 0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04b_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/r04b_tests.log; exit $rc

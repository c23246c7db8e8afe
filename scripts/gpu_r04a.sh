#!/bin/bash
# round 4, first GPU pass: GF(2^16) tests after the compile-time diag-mode change, then the consensus-path probe.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "512 or rs16 or ff16 or codec or abi" > gpurun_out/r04a_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/r04a_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/consensus_probe.py 20 > gpurun_out/r04a_probe.log 2>&1
rc=$?; cat gpurun_out/r04a_probe.log | grep -v amdgpu.ids; exit $rc

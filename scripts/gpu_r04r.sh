#!/bin/bash
# round 4 final pass on the final code: GPU suite + smoke + rocprofv3 evidence (scripts/gpu_round.sh $TAG, default r04_v2), then
# the default bench line and the consensus probe.
set -u
mkdir -p gpurun_out
bash scripts/gpu_round.sh ${TAG:-r04_v2} > gpurun_out/r04r_round.log 2>&1
rc=$?; grep -E "^== |^rc=|passed|ABORT" gpurun_out/r04r_round.log; [ $rc -ne 0 ] && exit $rc
grep -q ABORT gpurun_out/r04r_round.log && exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r04r_bench.log 2>&1
rc=$?; grep '^{' gpurun_out/r04r_bench.log | cut -c1-300; [ $rc -ne 0 ] && { tail -5 gpurun_out/r04r_bench.log; exit $rc; }
timeout -k 10 300 python -u scripts/consensus_probe.py 20 > gpurun_out/r04r_probe.log 2>&1
rc=$?; grep '^{' gpurun_out/r04r_probe.log; exit $rc

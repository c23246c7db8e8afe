#!/bin/bash
# Round-3 verification session: GPU parity suite, smoke, rocprof evidence (profile.sh r03), default bench line.
set -u
./scripts/gpu_round.sh ${TAG:-r03} || exit $?
echo "== bench"; date
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; echo "rc=$rc"; tail -n 3 gpurun_out/bench_default.log
exit $rc

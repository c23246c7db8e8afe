#!/bin/bash
# Round-3 final verification: GPU parity suite, smoke, rocprof evidence (profile.sh r03_v3), C2 / C5 probes, default
# bench line.  Each GPU step has its own time limit; stop at the first crash/timeout.
set -u
mkdir -p gpurun_out
PROFILE=1 ./scripts/gpu_round.sh ${TAG:-r03_v4} || exit $?
echo "== c2"; timeout -k 10 120 python -u scripts/c2_probe.py > gpurun_out/c2_final.log 2>&1 || exit $?
tail -c 600 gpurun_out/c2_final.log
echo "== rs16"; timeout -k 10 120 python -u scripts/rs16_probe.py 20 > gpurun_out/rs16_final.log 2>&1 || exit $?
cat gpurun_out/rs16_final.log
echo "== bench"; date
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; echo "rc=$rc"; tail -n 3 gpurun_out/bench_default.log | cut -c1-600
exit $rc

#!/bin/bash
# Bench sweep over the two-stream software pipeline (CDA_PIPELINE chunks) at B=128.
set -u
mkdir -p gpurun_out
for P in ${*:-1 2 4 8 16}; do
  CDA_PIPELINE=$P timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_pipe$P.log 2>&1; rc=$?
  echo "pipeline=$P rc=$rc $(tail -1 gpurun_out/bench_pipe$P.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])' 2>/dev/null)"
  [ $rc -ge 124 ] && exit $rc
done
exit 0

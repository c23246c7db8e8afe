#!/bin/bash
# A/B of environment switches on one box, rotating order: scripts/env_ab.sh <rounds> "<ENV=..>" "<ENV=..>" ...
set -u
N=$1; shift
mkdir -p gpurun_out
for i in $(seq 1 "$N"); do
  for e in "$@"; do
    env $e timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/env_ab.log 2>&1 || exit 1
    echo "$e $(tail -1 gpurun_out/env_ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernels_ms"])')"
  done
done

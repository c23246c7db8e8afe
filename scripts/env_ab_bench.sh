#!/bin/bash
# A/B/... of environment settings on one library: short bench runs in rotating order.
# usage: scripts/env_ab_bench.sh <rounds> <lib.so> "VAR=a" "VAR=b" ...
set -u
N=$1; LIB=$2; shift 2
ENVS=("$@"); M=${#ENVS[@]}
mkdir -p gpurun_out
for i in $(seq 0 $((N - 1))); do
  for j in $(seq 0 $((M - 1))); do
    e=${ENVS[$(((i + j) % M))]}
    env $e CDA_LIB=$LIB timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/envab.log 2>&1 || { tail -3 gpurun_out/envab.log; exit 1; }
    echo "$e $(grep '^{' gpurun_out/envab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["kernels_ms"])')"
  done
done

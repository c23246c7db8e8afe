#!/bin/bash
# Bench sweep over sequential chunk sizes (CDA_CHUNK blocks) at B=128.
set -u
mkdir -p gpurun_out
for C in ${*:-0 4 8 16 32 64}; do
  CDA_CHUNK=$C timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_chunk$C.log 2>&1; rc=$?
  echo "chunk=$C rc=$rc $(tail -1 gpurun_out/bench_chunk$C.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernels_ms"])' 2>/dev/null)"
  [ $rc -ge 124 ] && exit $rc
done
exit 0

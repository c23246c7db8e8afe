#!/bin/bash
# A/B of two library builds on one box: alternating short bench runs (no extras), kernel times per run.
# usage: scripts/ab_bench.sh <lib_a.so> <lib_b.so> [rounds]
set -u
A=$1; B=$2; N=${3:-3}
mkdir -p gpurun_out
for i in $(seq 1 "$N"); do
  for v in A B; do
    lib=$A; [ "$v" = B ] && lib=$B
    CDA_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1 || exit 1
    python3 -c "
import json
for l in open('gpurun_out/ab_$v.log'):
    if l.startswith('{'):
        d=json.loads(l); k=d['kernels_ms']
        print('$v', d['value'], d['ms_per_step'], ' '.join(f'{n}={t}' for n, t in sorted(k.items())))
"
  done
done

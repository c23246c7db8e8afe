#!/bin/bash
# A/B/... of library builds on one box: short bench runs (no extras) in a rotating order so that run position
# (clock / thermal drift) does not favour one build; prints each run and the per-build means of the kernel times.
# usage: scripts/ab_bench.sh <rounds> <lib.so>[@VAR=value] [<lib.so>[@VAR=value] ...]
#   (lib.so@VAR=value: that build with VAR=value in the environment, for the knobs of the hooks build)
set -u
N=$1; shift
LIBS=("$@")
M=${#LIBS[@]}
mkdir -p gpurun_out
: > gpurun_out/ab_runs.jsonl
for i in $(seq 0 $((N - 1))); do
  for j in $(seq 0 $((M - 1))); do
    lib=${LIBS[$(((i + j) % M))]}
    path=${lib%%@*}; envs=(); [ "$path" != "$lib" ] && envs=("${lib#*@}")
    env "${envs[@]}" CDA_LIB=$path timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-k512-split > gpurun_out/ab_run.log 2>&1 || exit 1
    python3 -c "
import json
for l in open('gpurun_out/ab_run.log'):
    if l.startswith('{'):
        d=json.loads(l); print(json.dumps({'lib': '$lib', 'value': d['value'], 'kernels': d['kernels_ms']}))
" >> gpurun_out/ab_runs.jsonl
    tail -n 1 gpurun_out/ab_runs.jsonl
  done
done
python3 - <<'PY'
import json, collections
runs = [json.loads(l) for l in open('gpurun_out/ab_runs.jsonl')]
by = collections.defaultdict(list)
for r in runs: by[r['lib']].append(r)
for lib, rs in by.items():
    ks = sorted(rs[0]['kernels'])
    mean = {k: round(sum(r['kernels'][k] for r in rs) / len(rs), 4) for k in ks}
    print(lib, 'blocks/s', round(sum(r['value'] for r in rs) / len(rs)), mean)
PY

#!/bin/bash
# FF8 encoder at k=128, B=128: the product library vs a diagnostic build whose g2 kernel only loads and stores
# (ab/libcda_rs8mem.so, -DCDA_RS8_DIAG_NOCOMPUTE), per-kernel times from the bench's event pass.
set -u
mkdir -p gpurun_out
for i in 1 2; do
  for lib in ab/libcda_a.so ab/libcda_rs8mem.so; do
    CDA_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-extras --no-cpu-baseline > gpurun_out/rs8d.log 2>&1 || { tail -5 gpurun_out/rs8d.log; exit 1; }
    echo "$lib $(grep '^{' gpurun_out/rs8d.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernels_ms"])')"
  done
done

#!/bin/bash
# DAH fold with precomputed second-block schedules in dah_kernel: whole GPU suite on the current libcda, bench A/B
# (a = before, b = after), and the C5 probe of both.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/combo3_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 2 gpurun_out/combo3_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 bash scripts/ab_bench.sh 2 ab/libcda_a.so ab/libcda_b.so || exit $?
for lib in ab/libcda_a.so ab/libcda_b.so ab/libcda_a.so ab/libcda_b.so; do
  echo "$lib $(CDA_LIB=$lib timeout -k 10 200 python scripts/k512_probe.py 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_block"], d["kernels_ms"])')" || exit 1
done

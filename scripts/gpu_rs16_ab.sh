#!/bin/bash
# FF16 encoder variants: parity tests of the GF(2^16) paths, then the C5 probe per CDA_RS16_R4 / CDA_RS16_LDS_KB setting.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "rs_ or codec or k512 or 256 or 512 or split or decode" > gpurun_out/rs16_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/rs16_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for e in "$@"; do
    env $e timeout -k 10 300 python scripts/k512_probe.py > gpurun_out/rs16_probe.log 2>&1 || exit 1
    echo "$e $(tail -1 gpurun_out/rs16_probe.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_block"], d["kernels_ms"])')"
  done
done

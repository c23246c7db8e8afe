#!/bin/bash
# GF(2^16) encoder: parity at k=512 (codec, block path, split) and the probe timings by mode.
set -u
run() {
  local name=$1 t=$2; shift 2
  echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "rc=$rc"; tail -n 6 "gpurun_out/$name.log"; [ $rc -ge 124 ] && exit $rc; return 0
}
mkdir -p gpurun_out
run ff16_parity 300 python -u -m pytest tests/test_gpu_parity.py tests/test_split_capi_gpu.py -x -q --timeout 120 --timeout-method thread -k "ff16 or 512 or split"
for m in 0 3 4 5 6; do echo "mode $m"; CDA_LIB=ab/libcda_rs16m$m.so timeout -k 10 120 python3 -u scripts/rs16_probe.py 20 || exit $?; done

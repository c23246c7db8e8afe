#!/bin/bash
# Parity tests, then bench sweeps over stream count / batch (one GPU session).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/tests.log 2>&1; rc=$?
tail -3 gpurun_out/tests.log; [ $rc -ge 124 ] && exit $rc
CFGS=${*:-"1:32 2:32 4:32 8:32 4:64"}
for cfg in $CFGS; do
  S=${cfg%%:*}; B=${cfg##*:}
  CDA_STREAMS=$S timeout -k 10 300 python bench.py --steps 10 --warmup 3 --batch $B --no-cpu-baseline > gpurun_out/bench_s${S}_b${B}.log 2>&1; rc=$?
  echo "streams=$S batch=$B rc=$rc $(tail -1 gpurun_out/bench_s${S}_b${B}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])' 2>/dev/null)"
  [ $rc -ge 124 ] && exit $rc
done
exit 0

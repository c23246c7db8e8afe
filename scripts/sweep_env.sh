#!/bin/bash
# Bench sweep over engine environment knobs (one GPU session, no parity tests).
# Usage: scripts/sweep_env.sh "CDA_CU_SPLIT=0 CDA_STREAMS=1" "CDA_CU_SPLIT=64" ...   (BATCH env: blocks/step)
set -u
mkdir -p gpurun_out
B=${BATCH:-32}
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 python bench.py --steps 20 --warmup 3 --batch $B --no-cpu-baseline > gpurun_out/sweep_$i.log 2>&1; rc=$?
  echo "[$cfg] batch=$B rc=$rc $(tail -1 gpurun_out/sweep_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])' 2>/dev/null)"
  [ $rc -ge 124 ] && exit $rc
done
exit 0

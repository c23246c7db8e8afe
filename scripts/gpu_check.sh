#!/bin/bash
# One GPU session: parity tests, smoke, short bench.  Stops at the first step
# that crashed/timed out (exit >= 124); a plain test failure (1) continues.
set -u
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run tests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
run bench 400 python bench.py --steps 10 --warmup 2 --cpu-seconds 8

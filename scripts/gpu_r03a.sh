#!/bin/bash
# Round 3, GPU session A: parity tests, smoke, the full bench line, the copy ceilings, the C4 repair trace.
set -u
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 12 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
run copy_bw 120 ./tools/copy_bw 1024
run bench 600 python -u bench.py
run repair_trace 300 env CDA_REPAIR_TRACE=1 python -u scripts/repair_fresh_trace.py

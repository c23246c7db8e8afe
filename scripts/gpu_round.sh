#!/bin/bash
# One GPU session: parity tests, smoke, then the rocprofv3 evidence for the bench step.
# Each GPU step has its own time limit; stop at the first crash/timeout (exit >= 124).
set -u
TAG=${1:-r02}
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 15 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
if [ "${PROFILE:-1}" = 1 ]; then
  run profile 1100 ./scripts/profile.sh "$TAG"
fi

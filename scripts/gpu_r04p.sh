#!/bin/bash
# round 4: FF8 latency launches only for grids < 32 register-encoder workgroups (the consensus path's row bands):
# consensus probe A/B per CDA_RS8_LAT_U, rotating, plus C2 once each.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "consensus or single or extend" > gpurun_out/r04p_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 2 gpurun_out/r04p_tests.log; [ $rc -ne 0 ] && exit $rc
for u in 0 4; do echo "U=$u $(CDA_RS8_LAT_U=$u timeout -k 10 120 python scripts/c2_probe.py 2>/dev/null | cut -c1-200)" || exit 1; done
for i in 1 2 3; do
  for u in 0 4; do
    echo "U=$u $(CDA_RS8_LAT_U=$u timeout -k 10 300 python scripts/consensus_probe.py 20 2>/dev/null | cut -c1-420)" || exit 1
  done
done

#!/bin/bash
# round 4: latency launches of the FF8 encoder (LDS encoder over U-unit byte slices when the register encoder's grid
# is < 256 workgroups).  GPU suite on the default (U = 4), then C2 and the consensus probe per CDA_RS8_LAT_U.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04o_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/r04o_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for u in 0 2 4 8; do
    echo "U=$u $(CDA_RS8_LAT_U=$u timeout -k 10 120 python scripts/c2_probe.py 2>/dev/null)" || exit 1
  done
done
for u in 0 4; do
  echo "U=$u $(CDA_RS8_LAT_U=$u timeout -k 10 300 python scripts/consensus_probe.py 20 2>/dev/null)" || exit 1
done

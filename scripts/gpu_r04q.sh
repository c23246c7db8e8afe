#!/bin/bash
# round 4: consensus probe per CDA_RS8_LAT_U (row-band latency launches), rotating.
set -u
mkdir -p gpurun_out
for i in 1 2 3; do
  for u in 2 4 8; do
    echo "U=$u $(CDA_RS8_LAT_U=$u timeout -k 10 300 python scripts/consensus_probe.py 20 2>/dev/null | cut -c1-420)" || exit 1
  done
done

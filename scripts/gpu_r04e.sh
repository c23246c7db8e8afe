#!/bin/bash
# GF(2^16) encoder at k=512, round 4 build: product vs memory-only (mode 1) vs compute-only (mode 3) diag libraries
# (built beforehand: make -C celestia-app_amd BUILD=build_m$m OUT=../ab/libcda_rs16m$m.so EXTRA=-DCDA_RS16_DIAG_MODE=$m),
# then the PMC passes of the product build (scripts/gpu_rs16_final_pmc.sh).
set -u
for i in 1 2 3; do
  for lib in celestia-app_amd/cda/libcda.so ab/libcda_rs16m1.so ab/libcda_rs16m3.so; do
    echo "$lib $(CDA_LIB=$lib timeout -k 10 120 python3 scripts/rs16_probe.py 20 2>/dev/null)" || exit 1
  done
done
bash scripts/gpu_rs16_final_pmc.sh

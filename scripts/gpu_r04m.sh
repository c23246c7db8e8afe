#!/bin/bash
# GF(2^16) whole-codeword kernel: odd workgroups start ~4 / ~8 x s_sleep 127 later (ab/libcda_st4.so, st8.so)
set -u
for i in 1 2 3; do
  for lib in celestia-app_amd/cda/libcda.so ab/libcda_st4.so ab/libcda_st8.so; do
    echo "$lib $(CDA_LIB=$lib timeout -k 10 120 python3 scripts/rs16_probe.py 20 2>/dev/null)" || exit 1
  done
done

#!/bin/bash
# GF(2^16) half-slice encoder, static split by dispatch age (h2s4 / s5 / s6: the first workgroup of each CU takes
# 4 / 5 / 6 eighths of the items) against the whole-codeword kernel (h2off); phase trace of s5.
set -u
for i in 1 2 3; do
  for lib in ab/libcda_h2off.so ab/libcda_h2s4.so ab/libcda_h2s5.so ab/libcda_h2s6.so; do
    echo "$lib $(CDA_LIB=$lib timeout -k 10 120 python3 scripts/rs16_probe.py 20 2>/dev/null)" || exit 1
  done
done
CDA_LIB=ab/libcda_h2trs5.so timeout -k 10 120 python3 scripts/h2_trace_probe.py

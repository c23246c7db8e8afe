#!/bin/bash
# A/B of static issue priority (s_setprio 1) for the second half of the waves of the FF8 g2 encoder (CDA_RS8_PRIO) and
# of the GF(2^16) register encoder (CDA_RS16_PRIO): rotating bench runs and rs16_probe runs, one box.
set -u
bash scripts/ab_bench.sh 3 celestia-app_amd/cda/libcda.so ab/libcda_prio8.so > gpurun_out/prio8_ab.log 2>&1 || { tail -20 gpurun_out/prio8_ab.log; exit 1; }
tail -12 gpurun_out/prio8_ab.log
for i in 1 2 3; do
  for lib in celestia-app_amd/cda/libcda.so ab/libcda_prio16.so; do
    echo "$lib $(CDA_LIB=$lib timeout -k 10 120 python scripts/rs16_probe.py 20)" >> gpurun_out/prio16_ab.log || exit 1
  done
done
cat gpurun_out/prio16_ab.log

#!/bin/bash
# GF(2^16) register encoder diagnostics at k=512: timing by mode (encode / memory only / no loads / no memory), the
# LDS encoder for comparison, and rocprofv3 PMC passes of the encode mode.  The mode libraries are built beforehand
# on the CPU side: for m in 0 1 2 3; do make -C celestia-app_amd BUILD=build_m$m OUT=../ab/libcda_rs16m$m.so \
#   EXTRA=-DCDA_RS16_DIAG_MODE=$m; done
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/rs16
mkdir -p "$OUT"
for m in 0 1 2 3; do
  echo "mode $m"; CDA_LIB=ab/libcda_rs16m$m.so timeout -k 10 120 python3 -u scripts/rs16_probe.py 20 || exit $?
done
echo "lds"; CDA_RS16=lds timeout -k 10 120 python3 -u scripts/rs16_probe.py 20 || exit $?
cd /tmp && export TMPDIR=/tmp
step() {
  local name=$1; shift
  timeout -k 10 200 rocprofv3 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -ge 124 ] && exit $rc
  return 0
}
P="python3 $R/scripts/rs16_probe.py 5"
step trace --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $P
step pmc1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/pmc1" -o run -- $P
step pmc2 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM --kernel-trace --output-format csv -d "$OUT/pmc2" -o run -- $P
step pmc3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc3" -o run -- $P
step pmc4 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc4" -o run -- $P

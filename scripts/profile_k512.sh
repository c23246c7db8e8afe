#!/bin/bash
# rocprofv3 kernel trace + PMC passes of the C5 probe (k=512 block path, GF(2^16) encoder).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof512
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
step() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -ge 124 ] && exit $rc
  return 0
}
step trace --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $R/scripts/k512_probe.py
step pmc1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/pmc1" -o run -- python3 $R/scripts/k512_probe.py
step pmc2 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d "$OUT/pmc2" -o run -- python3 $R/scripts/k512_probe.py

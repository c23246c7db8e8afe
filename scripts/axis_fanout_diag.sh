#!/bin/bash
# Diagnosis of the per-axis queue under a 256-thread fan-out: per-rep phase times and process CPU time of the C
# driver's extension (one thread per axis), and the cgroup's CPU throttling counters around each run, for the given
# slot counts (test-hooks build, CDA_AXIS_SLOTS).  Output: gpurun_out/axis_diag/*.log
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=$R/gpurun_out/axis_diag
mkdir -p $D
python3 -c "
import sys; sys.path.insert(0,'tests'); import oracle_lib as O
O.gen_ods(128, 0xC0FFEE).tofile('$D/ods.bin')"
for slots in ${SLOTS:-4 1}; do
  for th in 256 8; do
    f=$D/s${slots}_t${th}.log
    { cat /sys/fs/cgroup/cpu.stat 2>/dev/null | sed 's/^/before /'; } > $f
    if [ "$slots" = oracle ]; then backend="oracle $R/oracle/liboracle.so"; else
      backend="cda $R/celestia-app_amd/cda/libcda_hooks.so"; fi
    CDA_AXIS_SLOTS=$slots RSMT2D_AXES_VERBOSE=1 timeout -k 5 300 tests/abi_client/rsmt2d_axes $backend \
      extend 128 $th 15 $D/ods.bin $D >> $f 2>&1
    echo "rc=$?" >> $f
    { cat /sys/fs/cgroup/cpu.stat 2>/dev/null | sed 's/^/after /'; } >> $f
    echo "== slots $slots threads $th"; grep -E "rep|throttl|rc=|total_ms" $f | tail -24
  done
done

#!/bin/bash
# Host AddressSanitizer on the GPU: the C-ABI client built with -fsanitize=address against the host-ASan build of
# libcda (make -C celestia-app_amd asan; make -C tests/abi_client asan -- both built on the CPU beforehand), driven
# by tests/test_abi_client.py: the one-block consensus path (copy pool, fresh / registered buffers, the in-place entry),
# batches, repair, codec, blob commitments, share proofs, node export and square construction, every host access of
# libcda checked.  Device code is not instrumented.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:protect_shadow_gap=0
CDA_ABI_CLIENT=$R/tests/abi_client/abi_host_client_asan timeout -k 10 600 python -u -m pytest tests/test_abi_client.py \
  -m gpu -x -v --timeout 300 --timeout-method thread > $R/gpurun_out/asan_tests.log 2>&1
rc=$?
tail -n 25 $R/gpurun_out/asan_tests.log
[ $rc -ne 0 ] && exit $rc
# the per-axis seams (csrc/axisq.cpp) from 16 and 64 concurrent callers, then a Repair axis by axis, under ASan
python3 - <<'PY' || exit 1
import numpy as np, os, subprocess, sys
sys.path.insert(0, "tests")
import oracle_lib as O
R = os.environ.get("GRAFT_REPO_ROOT", os.getcwd())
d = os.path.join(R, "gpurun_out", "asan_axes"); os.makedirs(d, exist_ok=True)
k = 32
ods = O.gen_ods(k, 5); ods.tofile(f"{d}/ods.bin")
drv = [f"{R}/tests/abi_client/rsmt2d_axes_asan", "cda", f"{R}/celestia-app_amd/cda/libcda_asan.so"]
log = open(f"{R}/gpurun_out/asan_axes.log", "w")
for threads in (16, 64):
    p = subprocess.run(drv + ["extend", str(k), str(threads), "2", f"{d}/ods.bin", d], capture_output=True, text=True,
                       timeout=300)
    log.write(p.stdout + p.stderr)
    assert p.returncode == 0, p.stderr[-2000:]
rc, eds, rr, cr, _ = O.extend_commit(ods)
assert np.array_equal(np.fromfile(f"{d}/eds.bin", np.uint8).reshape(eds.shape), eds)
eds.tofile(f"{d}/full.bin"); np.concatenate([rr, cr]).tofile(f"{d}/roots.bin")
(np.random.default_rng(2).random(eds.shape[0]) < 0.5).astype(np.uint8).tofile(f"{d}/pres.bin")
p = subprocess.run(drv + ["repair", str(k), "8", "1", f"{d}/full.bin", f"{d}/pres.bin", f"{d}/roots.bin", d],
                   capture_output=True, text=True, timeout=300)
log.write(p.stdout + p.stderr)
assert p.returncode == 0 and '"rc": 0' in p.stdout, p.stderr[-2000:]
assert np.array_equal(np.fromfile(f"{d}/repaired.bin", np.uint8).reshape(eds.shape), eds)
print("asan per-axis driver ok")
PY
exit 0

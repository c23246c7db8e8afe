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
exit $rc

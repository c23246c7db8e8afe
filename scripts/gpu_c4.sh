#!/bin/bash
# Repair (C4) session: repair parity tests, then the host-buffer repair spread with and without NUMA binding.
set -u
mkdir -p gpurun_out
[ "${SKIP_TESTS:-0}" = 1 ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_abi_client.py -m gpu -x -q -k "repair or abi" \
  --timeout 120 --timeout-method thread > gpurun_out/c4_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 5 gpurun_out/c4_tests.log; [ $rc -ne 0 ] && exit $rc
CDA_REPAIR_TRACE=1 timeout -k 10 200 python -u scripts/c4_numa_probe.py > gpurun_out/c4_bind.log 2>&1 || exit $?
grep mode gpurun_out/c4_bind.log
CDA_NUMA_BIND=0 timeout -k 10 200 python -u scripts/c4_numa_probe.py > gpurun_out/c4_nobind.log 2>&1 || exit $?
grep mode gpurun_out/c4_nobind.log
timeout -k 10 200 python -u -c "
import sys, json; sys.path.insert(0, 'celestia-app_amd')
import torch, bench, cda
torch.cuda.init()
ctx = cda.Context(0)
print(json.dumps(bench.repair_measure(ctx, reps=9)))" > gpurun_out/c4_bench.log 2>&1; rc=$?
tail -n 2 gpurun_out/c4_bench.log; exit $rc

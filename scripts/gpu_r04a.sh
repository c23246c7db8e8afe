#!/bin/bash
# round 4 GPU pass: the whole GPU suite on the current libcda; GF(2^16) encoder A/B (pipelined loop vs round 3's,
# ab/libcda_pipe0.so); C2 A/B (helper-expanded block-0 schedules vs ab/libcda_base.so); the consensus-path probe
# (serial form vs the one-block path); host first-touch rates; short N=1 / N=2 benches with config C5's split.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04a_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/r04a_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for lib in celestia-app_amd/cda/libcda.so ab/libcda_pipe0.so; do
    echo "rs16 $lib $(CDA_LIB=$lib timeout -k 10 120 python scripts/rs16_probe.py 20 2>/dev/null)" || exit 1
  done
done
for i in 1 2 3; do
  for lib in celestia-app_amd/cda/libcda.so ab/libcda_base.so; do
    echo "c2 $lib $(CDA_LIB=$lib timeout -k 10 120 python scripts/c2_probe.py 2>/dev/null)" || exit 1
  done
done
for i in 1 2; do
  for m in 0 4 8; do
    CDA_MIXED=$m timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-extras --no-cpu-baseline --no-k512-split > gpurun_out/r04a_mixed.log 2>&1 || { tail -5 gpurun_out/r04a_mixed.log; exit 1; }
    echo "mixed=$m $(grep '^{' gpurun_out/r04a_mixed.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["output_check"]["blocks_checked_vs_golden"], d["kernels_ms"])')"
  done
done
CDA_CONSENSUS=0 timeout -k 10 300 python -u scripts/consensus_probe.py 20 > gpurun_out/r04a_probe_serial.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04a_probe_serial.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/consensus_probe.py 20 > gpurun_out/r04a_probe.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04a_probe.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 ./tools/fault_probe > gpurun_out/r04a_fault.log 2>&1; cat gpurun_out/r04a_fault.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-extras --no-cpu-baseline > gpurun_out/r04a_bench1.log 2>&1
rc=$?; grep '^{' gpurun_out/r04a_bench1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("N1", d["value"], d["kernels_ms"], json.dumps(d.get("k512_split")))'; [ $rc -ne 0 ] && { tail -5 gpurun_out/r04a_bench1.log; exit $rc; }
timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 --no-extras --no-cpu-baseline > gpurun_out/r04a_bench2.log 2>&1
rc=$?; grep '^{' gpurun_out/r04a_bench2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("N2", d["value"], json.dumps(d.get("k512_split")))'; [ $rc -ne 0 ] && { tail -5 gpurun_out/r04a_bench2.log; exit $rc; }
exit 0

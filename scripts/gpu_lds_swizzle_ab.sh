set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "rs_ or codec or k512 or 256 or 512 or split or extend" > gpurun_out/sw_tests.log 2>&1
rc=$?; tail -n 2 gpurun_out/sw_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for lib in celestia-app_amd/ab/libcda_nosw.so celestia-app_amd/ab/libcda_sw.so; do
    CDA_LIB=$lib timeout -k 10 300 python scripts/k512_probe.py > gpurun_out/sw_probe.log 2>&1 || exit 1
    echo "$lib $(tail -1 gpurun_out/sw_probe.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_block"], d["kernels_ms"])')"
  done
done

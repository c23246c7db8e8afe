#!/bin/bash
# Round-6 GPU runner: stages given as arguments, each under its own timeout; stops at the first failure.
#   tests_axis  per-axis seams + codec / tree / consensus-form / fault tests
#   tests       the whole GPU suite
#   per_axis    same-box A/B of the per-axis seams: $AXIS_LIBS (default libcda.so) and the oracle
#   ab          rotating same-box A/B of $AB_LIBS (bench --no-extras), $AB_ROUNDS rounds
#   bench       the default bench line; profile: scripts/profile.sh $TAG; asan: scripts/gpu_asan.sh
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
T=${TAG:-r06}
for stage in "$@"; do
  echo "=== $stage"
  case $stage in
    tests_axis)
      timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_per_axis_gpu.py \
        tests/test_gpu_parity.py tests/test_consensus_gpu.py tests/test_faults_gpu.py -k "per_axis or rs_encode or \
rs_decode or codec or axis_root or wrapper or tree or push or empty_tree or concurrent or one_block or fault or upstream \
or driver or release" > gpurun_out/${T}_tests_axis.log 2>&1
      rc=$?; tail -3 gpurun_out/${T}_tests_axis.log ;;
    tests)
      timeout -k 10 1100 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
        > gpurun_out/${T}_tests.log 2>&1
      rc=$?; tail -3 gpurun_out/${T}_tests.log ;;
    per_axis)
      timeout -k 10 900 python -u scripts/per_axis_ab.py ${AXIS_LIBS:-celestia-app_amd/cda/libcda.so} \
        > gpurun_out/${T}_per_axis.json 2> gpurun_out/${T}_per_axis.err
      rc=$?; tail -c 600 gpurun_out/${T}_per_axis.err ;;
    ab)
      timeout -k 10 900 bash scripts/ab_bench.sh ${AB_ROUNDS:-3} ${AB_LIBS:-celestia-app_amd/cda/libcda.so} \
        > gpurun_out/${T}_ab.log 2>&1
      rc=$?; cp gpurun_out/ab_runs.jsonl gpurun_out/${T}_ab_runs.jsonl 2>/dev/null; tail -4 gpurun_out/${T}_ab.log ;;
    bench)
      timeout -k 10 900 python -u bench.py > gpurun_out/${T}_bench.log 2>&1
      rc=$?; tail -c 400 gpurun_out/${T}_bench.log ;;
    asan)
      timeout -k 10 900 bash scripts/gpu_asan.sh > gpurun_out/${T}_asan.log 2>&1
      rc=$?; tail -3 gpurun_out/${T}_asan.log ;;
    profile)
      timeout -k 10 1000 bash scripts/profile.sh ${T} > gpurun_out/${T}_profile.log 2>&1
      rc=$?; tail -5 gpurun_out/${T}_profile.log ;;
    *) echo "unknown stage $stage"; rc=2 ;;
  esac
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done

#!/bin/bash
# Round-5 GPU runs: each argument names a stage, run in order; every GPU step under its own time limit, the script
# stops at the first failure.  Outputs under gpurun_out/r05<tag>_*.
#   tests        the whole -m gpu suite
#   consensus    scripts/consensus_shapes.py (the one-block call in every go/cda shape), 3 rounds
#   rs16ab       GF(2^16) encoder probe over the libraries in $LIBS (default: release, ab/libcda_touch0.so,
#                ab/libcda_nt.so), 3 rotations
#   constrace    scripts/consensus_trace.py (phase trace of the page-locked one-block path, after a D2H warm-up)
#   bench        bench.py (default: N = 1, full extras + CPU baseline)
#   profile      scripts/profile.sh r05 (rocprofv3 kernel trace + PMC passes of bench.py --steps 5)
set -u
TAG=${TAG:-a}
mkdir -p gpurun_out
O=gpurun_out/r05${TAG}
for stage in "$@"; do
  case $stage in
    tests)
      timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > ${O}_tests.log 2>&1
      rc=$?; tail -n 3 ${O}_tests.log; [ $rc -ne 0 ] && exit $rc ;;
    consensus)
      timeout -k 10 400 python -u scripts/consensus_shapes.py 25 3 > ${O}_shapes.log 2>&1
      rc=$?; tail -c 2500 ${O}_shapes.log; [ $rc -ne 0 ] && exit $rc ;;
    duplex)
      for i in 1 2; do
        timeout -k 10 120 python -u scripts/pcie_duplex_probe.py >> ${O}_duplex.log 2>&1 || exit 1
        HSA_ENABLE_SDMA=0 timeout -k 10 120 python -u scripts/pcie_duplex_probe.py | sed 's/^{/{"sdma": 0, /' >> ${O}_duplex.log 2>&1 || exit 1
      done
      grep '^{' ${O}_duplex.log ;;
    consweep)  # one-block path forms (knobs read at cda_init), two rotations, plus the box's DMA duplex behaviour
      timeout -k 10 120 python -u scripts/pcie_duplex_probe.py > ${O}_consweep.log 2>&1 || exit 1
      for i in 1 2; do
        for v in ${CONS_FORMS:-"CDA_CONS_ORDER=0" "CDA_CONS_ORDER=1" "CDA_CONS_ORDER=1 CDA_CONS_IN=2" "CDA_CONS_ORDER=0 CDA_CONS_IN=2" "CDA_CONS_PUSH=1 CDA_CONS_ORDER=1"}; do
          echo "== $v $(env ${v//,/ } timeout -k 10 200 python -u scripts/consensus_trace.py | grep '^{')" >> ${O}_consweep.log || exit 1
        done
      done
      cat ${O}_consweep.log | cut -c 1-400 ;;
    constrace_prof)  # rocprofv3 kernel + memory-copy trace of pinned one-block calls (no PMC in this run)
      mkdir -p gpurun_out/prof_cons
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
        -d $GRAFT_REPO_ROOT/gpurun_out/prof_cons -o run -- python3 $GRAFT_REPO_ROOT/scripts/consensus_calls.py 40) \
        > ${O}_constrace_prof.log 2>&1
      rc=$?; tail -n 5 ${O}_constrace_prof.log; find gpurun_out/prof_cons -name "*.csv" | head; [ $rc -ne 0 ] && exit $rc ;;
    constrace_blit)
      HSA_ENABLE_SDMA=0 timeout -k 10 400 python -u scripts/consensus_trace.py > ${O}_constrace_blit.log 2>&1
      rc=$?; tail -c 2500 ${O}_constrace_blit.log; [ $rc -ne 0 ] && exit $rc ;;
    constrace)
      timeout -k 10 400 python -u scripts/consensus_trace.py > ${O}_constrace.log 2>&1
      rc=$?; tail -c 2500 ${O}_constrace.log; [ $rc -ne 0 ] && exit $rc ;;
    rs16ab)
      for i in 1 2 3; do
        for lib in ${LIBS:-celestia-app_amd/cda/libcda.so ab/libcda_touch0.so ab/libcda_nt.so}; do
          echo "$lib $(CDA_LIB=$lib timeout -k 10 120 python scripts/rs16_probe.py 20)" >> ${O}_rs16ab.log || exit 1
        done
      done
      cat ${O}_rs16ab.log ;;
    bench)
      timeout -k 10 900 python -u bench.py > ${O}_bench.log 2>&1
      rc=$?; tail -c 1500 ${O}_bench.log; [ $rc -ne 0 ] && exit $rc ;;
    profile)
      timeout -k 10 900 bash scripts/profile.sh r05${TAG} > ${O}_profile.log 2>&1
      rc=$?; tail -n 20 ${O}_profile.log; [ $rc -ne 0 ] && exit $rc ;;
    *) echo "unknown stage $stage"; exit 2 ;;
  esac
done
exit 0

#!/bin/bash
# A/B of the one-block path's forms (knobs since removed; results in profiles/r05_consensus_timeline.log) (CDA_CONS_PULL=1: a page-locked input read by the row pass across PCIe, against
# the DMA bands; CDA_CONS_BOT=0/1/2: where a pinned output's bottom half is copied): GPU tests of the consensus path in pull mode, then consensus_shapes and the device timeline per form.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/bot
mkdir -p $O
CDA_CONS_BOT=2 timeout -k 10 600 python -u -m pytest tests/test_consensus_gpu.py tests/test_abi_client.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  for v in 0 1 2; do
    echo "== bot=$v $(CDA_CONS_BOT=$v timeout -k 10 300 python -u scripts/consensus_shapes.py 25 1 | grep '^{')" >> $O/shapes.log || exit 1
  done
done
cut -c 1-1500 $O/shapes.log
for v in 0 1 2; do
  for m in inplace; do
    rm -rf $O/pc_${m}_$v
    (cd /tmp && export TMPDIR=/tmp && CDA_CONS_BOT=$v timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace \
      --output-format csv -d $O/pc_${m}_$v -o run -- python3 $R/scripts/consensus_calls.py 40 $m) > $O/pc_${m}_$v.log 2>&1 || exit 1
    f=$(find $O/pc_${m}_$v -name "run_kernel_trace.csv" | head -1)
    echo "== bot=$v $m $(grep median $O/pc_${m}_$v.log)" >> $O/timeline.log
    python3 $R/scripts/cons_timeline.py $(dirname $f) >> $O/timeline.log
  done
done
cat $O/timeline.log

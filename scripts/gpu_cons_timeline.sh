set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for m in pinned inplace; do
  rm -rf $R/gpurun_out/pc_$m
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
     -d $R/gpurun_out/pc_$m -o run -- python3 $R/scripts/consensus_calls.py 40 $m) > $R/gpurun_out/pc_$m.log 2>&1 || exit 1
  f=$(find $R/gpurun_out/pc_$m -name "run_kernel_trace.csv" | head -1)
  python3 $R/scripts/cons_timeline.py $(dirname $f) | tee -a $R/gpurun_out/pc_timeline.log
  grep median $R/gpurun_out/pc_$m.log
done

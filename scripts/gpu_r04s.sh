#!/bin/bash
# round 4: one rocprofv3 --pmc pass with the L2->fabric read-request size counters over the bench step (4 TCC
# counters, the per-pass limit), to calibrate the read traffic of each kernel (scripts/rdreq_sizes.py).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_rdreq
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-trace --output-format csv -d "$OUT/p" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-extras --no-k512-split > "$OUT/run.log" 2>&1
rc=$?; echo "rc=$rc"; grep -v "^[EW]2026" "$OUT/run.log" | tail -n 3 | cut -c1-200
exit $rc

#!/bin/bash
# round 4: level kernel with the children's first 64 B parked in LDS for the namespace range (no end re-read):
# GPU suite on it, rotating A/B against the previous build, request-size PMC pass.
set -u
mkdir -p gpurun_out
CDA_LIB=ab/libcda_v1.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04v_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 1 gpurun_out/r04v_tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_bench.sh 4 ab/libcda_v1.so ab/libcda_prev.so || exit 1
R=$(pwd); OUT=$R/gpurun_out/prof_rdreq_v1; mkdir -p $OUT
(cd /tmp && CDA_LIB=$R/ab/libcda_v1.so timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-trace --output-format csv -d "$OUT/p" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-extras --no-k512-split > "$OUT/run.log" 2>&1)
echo "pmc rc=$?"

#!/bin/bash
# GPU suite on the simplified consensus path (one results D2H, status set off the chain), its probe with the phase
# trace, then the GF(2^16) half-slice static-split A/B (scripts/gpu_r04h.sh).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04i_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/r04i_tests.log; [ $rc -ne 0 ] && exit $rc
CDA_CONS_TRACE=1 timeout -k 10 300 python -u scripts/consensus_probe.py 20 > gpurun_out/r04i_probe.log 2>&1
rc=$?; grep '^{' gpurun_out/r04i_probe.log; [ $rc -ne 0 ] && exit $rc
python3 - <<'PY'
import re, statistics as st
rows = {}
for l in open("gpurun_out/r04i_probe.log"):
    if l.startswith("cons_trace"):
        kv = dict(re.findall(r"(\w+)=([\d.]+)", l))
        rows.setdefault((kv["fresh"], kv["resident"]), []).append(kv)
for key, r in rows.items():
    print("fresh=%s resident=%s n=%d" % (key[0], key[1], len(r)),
          {f: round(st.median(float(x[f]) for x in r), 1) for f in r[0] if f not in ("fresh", "resident")})
PY
bash scripts/gpu_r04h.sh

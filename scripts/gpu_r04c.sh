#!/bin/bash
# consensus-path phase trace (CDA_CONS_TRACE=1: host timestamps per call, medians over the fresh with-EDS series)
set -u
mkdir -p gpurun_out
for v in "CDA_CONS_OUT=0 CDA_PROBE_SWEEP=1" "CDA_CONS_IN=1" "CDA_CONS_IN=1 CDA_COPY_THREADS=15" "CDA_CONS_OUT=0"; do
  env CDA_CONS_TRACE=1 $v timeout -k 10 300 python -u scripts/consensus_probe.py 15 > gpurun_out/r04c_probe.log 2>&1
  rc=$?; echo "== $v"; grep '^{' gpurun_out/r04c_probe.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/r04c_probe.log; exit $rc; }
  python - <<'PY'
import re, statistics as st
lines = [l for l in open("gpurun_out/r04c_probe.log") if l.startswith("cons_trace")]
groups = {}
for l in lines:
    kv = dict(re.findall(r"(\w+)=([\d.]+)", l))
    groups.setdefault((kv["fresh"], kv["resident"]), []).append(kv)
for key, rows in groups.items():
    print("fresh=%s resident=%s n=%d" % (key[0], key[1], len(rows)),
          {f: round(st.median(float(r[f]) for r in rows), 1) for f in rows[0] if f not in ("fresh", "resident")})
PY
done
[ -n "${SKIP_TESTS:-}" ] && exit 0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04c_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/r04c_tests.log; exit $rc

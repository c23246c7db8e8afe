#!/bin/bash
# Consensus path input forms: pageable (default) vs the caller's shares registered for the call (CDA_CONS_IN=3
# bands, 4 one copy), with the phase trace.
set -u
mkdir -p gpurun_out
for v in "CDA_CONS_IN=0" "CDA_CONS_IN=3" "CDA_CONS_IN=4" "CDA_CONS_IN=0"; do
  env CDA_CONS_TRACE=1 $v timeout -k 10 300 python -u scripts/consensus_probe.py 20 > gpurun_out/r04j_probe.log 2>&1
  rc=$?; echo "== $v"; grep '^{' gpurun_out/r04j_probe.log; [ $rc -ne 0 ] && { tail -5 gpurun_out/r04j_probe.log; exit $rc; }
  python3 - <<'PY'
import re, statistics as st
rows = {}
for l in open("gpurun_out/r04j_probe.log"):
    if l.startswith("cons_trace"):
        kv = dict(re.findall(r"(\w+)=([\d.]+)", l))
        rows.setdefault((kv["fresh"], kv["resident"]), []).append(kv)
for key, r in rows.items():
    print("fresh=%s resident=%s n=%d" % (key[0], key[1], len(r)),
          {f: round(st.median(float(x[f]) for x in r), 1) for f in r[0] if f not in ("fresh", "resident")})
PY
done

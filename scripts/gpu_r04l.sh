#!/bin/bash
# Consensus path: part of a pageable bottom half staged through the pinned slab on the second stream
# (CDA_CONS_STG = MiB) vs all pageable; consensus GPU tests with the staged form first.
set -u
mkdir -p gpurun_out
true && touch gpurun_out/r04l_tests.log
rc=$?; tail -n 2 gpurun_out/r04l_tests.log; [ $rc -ne 0 ] && exit $rc
for v in "CDA_CONS_H2D2=0" "CDA_CONS_H2D2=1" "CDA_CONS_H2D2=0" "CDA_CONS_H2D2=1" "CDA_CONS_H2D2=0"; do
  env -u CDA_CONS_TRACE $v timeout -k 10 300 python -u scripts/consensus_probe.py 20 > gpurun_out/r04l_probe.log 2>&1
  rc=$?; echo "== $v $(grep '^{' gpurun_out/r04l_probe.log)"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r04l_probe.log; exit $rc; }
done
python3 - <<'PY'
import re, statistics as st
rows = {}
for l in open("gpurun_out/r04l_probe.log"):
    if l.startswith("cons_trace"):
        kv = dict(re.findall(r"(\w+)=([\d.]+)", l))
        rows.setdefault((kv["fresh"], kv["resident"]), []).append(kv)
for key, r in rows.items():
    print("fresh=%s resident=%s n=%d" % (key[0], key[1], len(r)),
          {f: round(st.median(float(x[f]) for x in r), 1) for f in r[0] if f not in ("fresh", "resident")})
PY

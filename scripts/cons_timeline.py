"""One consensus call's device timeline from a rocprofv3 --kernel-trace --memory-copy-trace run
(scripts/gpu_r05.sh constrace_prof): kernels and copies merged, split into calls at idle gaps > GAP_US, and the
median-length call printed as `start end duration kind name queue`, us from its first event.
usage: cons_timeline.py <dir with run_kernel_trace.csv / run_memory_copy_trace.csv> [gap_us]"""
import csv
import os
import sys

d = sys.argv[1]
gap = float(sys.argv[2]) if len(sys.argv) > 2 else 150.0
ev = []
for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", r["Kernel_Name"].split("(")[0][:44],
               f"q{r.get('Queue_Id', '?')}"))
p = os.path.join(d, "run_memory_copy_trace.csv")
if os.path.exists(p):
    for r in csv.DictReader(open(p)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C",
                   r["Direction"].replace("MEMORY_COPY_", ""), f"s{r.get('Stream_Id', '?')}"))
ev.sort()
# a call starts with the status word's hipMemsetAsync (a fillBuffer kernel); otherwise split at idle gaps
starts = [i for i, e in enumerate(ev) if e[2] == "K" and "fillBuffer" in e[3]]
calls = []
if len(starts) >= 3:
    for a, b in zip(starts, starts[1:] + [len(ev)]):
        calls.append(ev[a:b])
else:
    cur, end = [], None
    for e in ev:
        if end is not None and e[0] - end > gap * 1e3:
            calls.append(cur)
            cur = []
        cur.append(e)
        end = e[1] if end is None else max(end, e[1])
    calls.append(cur)
calls = [c for c in calls[1:-1] if len(c) >= 6] or calls
spans = sorted((max(x[1] for x in c) - c[0][0], i) for i, c in enumerate(calls))
span, i = spans[len(spans) // 2]
c = calls[i]
print(f"# {len(calls)} calls; median span {span / 1e3:.1f} us (min {spans[0][0] / 1e3:.1f}, "
      f"max {spans[-1][0] / 1e3:.1f}); call {i}:")
t0 = c[0][0]
for s, e, kind, name, q in c:
    print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} {kind} {name:44s} {q}")

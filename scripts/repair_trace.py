"""Timeline of the last cda_repair call in a rocprofv3 kernel + memory-copy trace (gaps = host time)."""
import csv
import sys

d = sys.argv[1]
ev = []
for r in csv.DictReader(open(f"{d}/rp_kernel_trace.csv")):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:34]))
for r in csv.DictReader(open(f"{d}/rp_memory_copy_trace.csv")):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + r.get("Direction", "")[12:]))
ev.sort()
big = [i for i, e in enumerate(ev) if e[2].startswith("COPY") and e[1] - e[0] > 300000 and "HOST_TO_DEVICE" in e[2]]
which = int(sys.argv[2]) if len(sys.argv) > 2 else len(big) - 1
i0 = big[which]
i1 = big[which + 1] if which + 1 < len(big) else len(ev)
t0 = ev[i0][0]
prev = t0
idle = 0
for s, e, n in ev[i0:i1]:
    if s > prev:
        idle += s - prev
    print(f"{(s - t0) / 1e3:8.1f} +{(s - prev) / 1e3:6.1f} {(e - s) / 1e3:7.1f} {n}")
    prev = max(prev, e)
print(f"span {(prev - t0) / 1e3:.1f} us, device idle {idle / 1e3:.1f} us")

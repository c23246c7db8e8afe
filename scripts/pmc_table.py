"""Sum rocprofv3 PMC counters per dispatch and print one line per kernel (median over its dispatches).
usage: pmc_table.py <run_counter_collection.csv> [kernel-substring ...]"""
import collections
import csv
import statistics
import sys

path, pats = sys.argv[1], sys.argv[2:]
agg = collections.defaultdict(float)
names = {}
for r in csv.DictReader(open(path)):
    k = r["Kernel_Name"]
    if pats and not any(p in k for p in pats):
        continue
    agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    names[r["Dispatch_Id"]] = k
per = collections.defaultdict(lambda: collections.defaultdict(list))
for (d, c), v in agg.items():
    per[names[d].split("(")[0][:60]][c].append(v)
for k, cs in per.items():
    print(k, {c: int(statistics.median(v)) for c, v in sorted(cs.items())})

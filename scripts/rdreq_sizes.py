#!/usr/bin/env python3
"""Read bytes per kernel from the request-size counters (TCC_EA0_RDREQ_{32B,64B,128B}) of one rocprofv3 --pmc pass
(scripts/gpu_r04s.sh), against FETCH_SIZE's formula and the x2 correction of MI355X_MICROARCH.md: calibrates the
`traffic` of kernels whose loads are not 16-B-per-lane streaming reads (the leaf kernel: 16 B per lane at a 512-B
stride).  usage: rdreq_sizes.py <run_counter_collection.csv> [out.json]"""
import collections
import csv
import json
import re
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("cda::", "").replace("void ", "")
    key = f"{name}@grid={r['Grid_Size']}"
    acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[key].add(r["Dispatch_Id"])
out = {}
for key, c in sorted(acc.items()):
    n = len(disp[key])
    get = lambda s: c.get(f"TCC_EA0_RDREQ_{s}_sum", c.get(f"TCC_EA0_RDREQ_{s}", 0.0)) / n  # noqa: E731
    req = c.get("TCC_EA0_RDREQ_sum", c.get("TCC_EA0_RDREQ", 0.0)) / n
    n32, n64, n128 = get("32B"), get("64B"), get("128B")
    sized = 32 * n32 + 64 * n64 + 128 * n128
    fetch = 64 * (req - n32) + 32 * n32  # FETCH_SIZE's formula with no bubble counts
    out[key] = {"dispatches": n, "rdreq": req, "rdreq_32b": n32, "rdreq_64b": n64, "rdreq_128b": n128,
                "read_bytes_by_size": sized, "fetch_size_formula_bytes": fetch,
                "x2_corrected_bytes": 2 * fetch, "by_size_over_x2": sized / (2 * fetch) if fetch else None}
    print(f"{key:60s} n={n:3d} req={req:.4g} 32B={n32:.4g} 64B={n64:.4g} 128B={n128:.4g} "
          f"bytes={sized / 1e9:.4f} GB  x2={2 * fetch / 1e9:.4f} GB")
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)

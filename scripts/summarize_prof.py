#!/usr/bin/env python3
"""Summarize a scripts/profile.sh run (gpurun_out/prof) into profiles/<tag>_*.

Writes the rocprofv3 --stats kernel table verbatim and a per-kernel counter
summary (mean per dispatch).  FETCH_SIZE / WRITE_SIZE are in KB as reported;
the gfx950 correction (FETCH_SIZE x2 for wide streaming reads,
MI355X_MICROARCH.md §HBM) is applied in the 'hbm_bytes_corrected' column.
"""
import collections
import csv
import json
import os
import shutil
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
src = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/prof"
dst = "profiles"
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))

def short(n):
    n = n.replace("HIP_vector_type<unsigned int, 4u>", "uint4")
    return n.split("(")[0].replace("cda::", "").replace("void ", "")

def grid(r):
    """Total work-items of a dispatch (rocprofv3 writes Grid_Size, or Grid_Size_X/Y/Z)."""
    if r.get("Grid_Size"):
        return int(r["Grid_Size"])
    g = 1
    for a in "XYZ":
        g *= int(r.get(f"Grid_Size_{a}") or 1)
    return g


# per kernel name, and per (name, grid size) when one kernel is dispatched with several grid sizes (the NMT levels
# kernel: levels 1-2 over every tree, then the thinner upper levels) -- "<name>@grid=<n>"
counters = collections.defaultdict(lambda: collections.defaultdict(list))
durations = collections.defaultdict(list)
grids = collections.defaultdict(set)
for sub in sorted(os.listdir(src)):
    p = os.path.join(src, sub, "run_counter_collection.csv")
    if not os.path.exists(p):
        continue
    for r in csv.DictReader(open(p)):
        n = short(r["Kernel_Name"])
        counters[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
        counters[f"{n}@grid={grid(r)}"][r["Counter_Name"]].append(float(r["Counter_Value"]))
        grids[n].add(grid(r))
for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))):
    n = short(r["Kernel_Name"])
    durations[n].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    durations[f"{n}@grid={grid(r)}"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for n, gs in grids.items():  # single-grid kernels need no per-grid entries
    if len(gs) == 1:
        counters.pop(f"{n}@grid={next(iter(gs))}", None)

summary = {}
for k, cs in counters.items():
    if k.startswith("__amd"):
        continue
    row = {c: sum(v) / len(v) for c, v in cs.items()}
    row["bench_batch"] = int(os.environ.get("BENCH_BATCH", "128"))  # blocks per bench step when profiled
    if "FETCH_SIZE" in row and "WRITE_SIZE" in row:
        row["hbm_bytes_corrected"] = (2 * row["FETCH_SIZE"] + row["WRITE_SIZE"]) * 1024
    if k in durations:
        row["avg_duration_ns"] = sum(durations[k]) / len(durations[k])
        row["dispatches"] = len(durations[k])
    summary[k] = row
json.dump(summary, open(os.path.join(dst, f"{tag}_counters.json"), "w"), indent=1, sort_keys=True)
with open(os.path.join(dst, f"{tag}_summary.md"), "w") as f:
    f.write(f"# rocprofv3 summary ({tag})\n\nSource: scripts/profile.sh (bench.py --steps 5 --warmup 1), "
            "kernel trace + separate PMC passes.\n\n")
    f.write("| kernel | avg ns | dispatches | VALU instr/wave | issue-stall frac | waitcnt/barrier frac | FETCH KB | WRITE KB | eff. clock GHz | VALU issue frac (2-cycle) |\n|---|---|---|---|---|---|---|---|---|---|\n")
    for k, r in sorted(summary.items(), key=lambda kv: -kv[1].get("avg_duration_ns", 0) * kv[1].get("dispatches", 0)):
        vpw = r.get("SQ_INSTS_VALU", 0) / r["SQ_WAVES"] if r.get("SQ_WAVES") else 0
        stall = r.get("SQ_WAIT_INST_ANY", 0) / r["SQ_WAVE_CYCLES"] if r.get("SQ_WAVE_CYCLES") else 0
        wait = r.get("SQ_WAIT_ANY", 0) / r["SQ_WAVE_CYCLES"] if r.get("SQ_WAVE_CYCLES") else 0
        clk = r.get("GRBM_GUI_ACTIVE", 0) / 8 / r["avg_duration_ns"] if r.get("avg_duration_ns") else 0
        # wave64 VALU instructions x 2 cycles over the SIMD-cycles of the dispatch (1024 SIMDs, GRBM_GUI_ACTIVE counts
        # each of the 8 XCDs).  SQ_ACTIVE_INST_VALU is NOT a busy-cycle count on gfx950: it equals SQ_INSTS_VALU.
        busy = r.get("SQ_INSTS_VALU", 0) * 2 / (1024 * r["GRBM_GUI_ACTIVE"] / 8) if r.get("GRBM_GUI_ACTIVE") else 0
        f.write(f"| {k} | {r.get('avg_duration_ns', 0):.0f} | {r.get('dispatches', 0)} | {vpw:.0f} | {stall:.2f} | "
                f"{wait:.2f} | {r.get('FETCH_SIZE', 0):.0f} | {r.get('WRITE_SIZE', 0):.0f} | {clk:.2f} | {busy:.2f} |\n")
print(open(os.path.join(dst, f"{tag}_summary.md")).read())

#!/usr/bin/env python3
"""Static check of the counted vmcnt waits of the GF(2^16) register encoder (csrc/rs16_kernels.hip read_prefetch).

The encoder issues its LDS prefetch (8 x global_load_lds_dwordx4) from inline asm and reads it back behind an asm
`s_waitcnt vmcnt(N)` whose N is a hand count of the vector-memory instructions the wave issues between the prefetch
and the read (kAfterPrefetch = 24 in the loop, 8 after the prologue).  On gfx950 loads, stores and LDS-DMA retire from
vmcnt in issue order, so the wait covers the prefetch iff every path from the last DMA load to the wait issues at
least N vector-memory instructions; exactly N means no over-wait.  A compiler change that moves a store or a spill
across the prefetch would break the count silently -- this walks the disassembly's control-flow graph instead.

usage: vmcnt_check.py <libcda.so>   (exit 0 and one line per wait when every path count equals its N)
"""
import os
import re
import subprocess
import sys
import tempfile

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
KERNEL = "rs_encode16_reg_kernel"
LINE = re.compile(r"^\s+([a-z_0-9]+)(.*?)//\s*([0-9A-F]+):.*?(?:<(\S+)\+0x([0-9a-f]+)>)?\s*$")
SYM = re.compile(r"^([0-9a-f]+) <(\S+)>:")
VMEM = ("global_", "buffer_", "flat_", "scratch_")


def code_objects(lib, tmp):
    """Unbundle the gfx950 device code objects of a HIP shared library into tmp; returns their paths."""
    dst = os.path.join(tmp, os.path.basename(lib))
    with open(lib, "rb") as f, open(dst, "wb") as g:
        g.write(f.read())
    subprocess.run([OBJDUMP, "--offloading", dst], cwd=tmp, check=True, capture_output=True)
    return [os.path.join(tmp, n) for n in sorted(os.listdir(tmp)) if "gfx950" in n]


def parse(text):
    """The kernel's instructions as (addr, mnemonic, operands, branch target addr or None), in address order."""
    out, base, inside = [], None, False
    for ln in text.splitlines():
        m = SYM.match(ln)
        if m:
            inside = KERNEL in m.group(2)
            base = int(m.group(1), 16) if inside else None
            continue
        if not inside:
            continue
        m = LINE.match(ln)
        if not m:
            continue
        mn, ops, addr, sym, off = m.groups()
        tgt = base + int(off, 16) if (sym and mn.startswith(("s_branch", "s_cbranch"))) else None
        out.append((int(addr, 16), mn, ops.strip(), tgt))
    return out


def is_vmem(mn):
    return mn.startswith(VMEM)


def check(insts):
    """[(wait addr, N, min path count, max path count)] for every read_prefetch wait reachable from a prefetch."""
    idx = {a: i for i, (a, _, _, _) in enumerate(insts)}
    waits = {}
    for i, (a, mn, ops, _) in enumerate(insts):
        m = re.match(r"vmcnt\((\d+)\)$", ops)
        if mn == "s_waitcnt" and m and i + 1 < len(insts) and insts[i + 1][1] == "ds_read_b128":
            waits[i] = int(m.group(1))
    # the last DMA load of each group of prefetch loads
    starts = [i for i, (_, mn, _, _) in enumerate(insts)
              if mn.startswith("global_load_lds") and not insts[i + 1][1].startswith("global_load_lds")
              and not any(insts[j][1].startswith("global_load_lds") for j in range(i + 1, min(i + 4, len(insts))))]
    seen = {}
    for s in starts:
        stack, visited = [(s + 1, 0)], set()
        while stack:
            i, n = stack.pop()
            while i < len(insts):
                if (i, n) in visited:
                    break
                visited.add((i, n))
                a, mn, ops, tgt = insts[i]
                if i in waits:
                    lo, hi = seen.get(i, (n, n))
                    seen[i] = (min(lo, n), max(hi, n))
                    break
                if mn.startswith("global_load_lds"):
                    break  # another prefetch before any read-back: that one owns the next wait
                if is_vmem(mn):
                    n += 1
                if mn == "s_endpgm":
                    break
                if mn == "s_branch":
                    i = idx[tgt]
                    continue
                if mn.startswith("s_cbranch"):
                    stack.append((idx[tgt], n))
                i += 1
    return [(insts[i][0], waits[i], lo, hi) for i, (lo, hi) in sorted(seen.items())]


def main(lib):
    with tempfile.TemporaryDirectory() as tmp:
        for co in code_objects(lib, tmp):
            text = subprocess.run([OBJDUMP, "-d", co], capture_output=True, text=True, check=True).stdout
            if KERNEL not in text:
                continue
            insts = parse(text)
            res = check(insts)
            scratch = sum(1 for _, mn, _, _ in insts if mn.startswith("scratch_"))
            ok = bool(res) and all(lo == hi == n for _, n, lo, hi in res) and scratch == 0
            for a, n, lo, hi in res:
                print(f"wait @0x{a:x}: vmcnt({n}), vector-memory instructions after the prefetch on every path: "
                      f"{lo}..{hi}")
            print(f"scratch instructions: {scratch}")
            print("ok" if ok else "MISMATCH")
            return 0 if ok else 1
    print("no", KERNEL, "in", lib)
    return 2


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))

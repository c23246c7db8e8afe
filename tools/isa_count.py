#!/usr/bin/env python3
"""Static VALU mix of the kernels in a `hipcc --cuda-device-only -S` listing, priced with the issue costs measured
on MI355X (profiles/r02_valu_ubench.txt): 2 cycles per wave64 instruction for plain VOP2-class ops and v_bitop3 /
v_fma_f32, 4 cycles for the other VOP3-only ops (v_alignbit, v_add3, v_lshl_or, v_perm, v_bfi, ...) and for ANY
VALU instruction with an SGPR or literal source.  Loops are counted once (a static mix): for kernels whose loop bodies
repeat the straight-line work (SHA-256 compressions) the average cycles per instruction carries over.

    tools/isa_count.py <listing.s> [kernel-regex] [--json out.json]
"""
import collections
import json
import re
import sys

FULL_RATE = {
    "v_add_u32", "v_sub_u32", "v_subrev_u32", "v_xor_b32", "v_or_b32", "v_and_b32", "v_not_b32", "v_lshlrev_b32",
    "v_lshrrev_b32", "v_ashrrev_i32", "v_mov_b32", "v_cndmask_b32", "v_bitop3_b32", "v_bitop3_b16", "v_fma_f32",
    "v_add_co_u32", "v_addc_co_u32", "v_sub_co_u32", "v_subb_co_u32", "v_subrev_co_u32", "v_max_u32", "v_min_u32",
    "v_max_i32", "v_min_i32", "v_mul_f32", "v_add_f32", "v_sub_f32", "v_max_f32", "v_min_f32",
}
SGPR = re.compile(r"(?<![\w\[])s(\d+|\[\d+:\d+\])\b|\bvcc\b|\bexec\b|\b0x[0-9a-fA-F]{3,}\b|\b\d{3,}\b")


def base_op(op):
    return re.sub(r"_e(32|64)$|_sdwa$|_dpp$", "", op)


def kernels(path):
    name, body = None, []
    for line in open(path):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            name, body = m.group(1), []
            continue
        if name is None:
            continue
        if "s_endpgm" in line:
            yield name, body
            name = None
            continue
        body.append(line)


def analyse(body):
    c = collections.Counter()
    cycles = n = with_s = 0
    for line in body:
        t = line.split(";")[0].strip().split(None, 1)
        if not t or t[0].startswith(".") or t[0].endswith(":"):
            continue
        c[t[0]] += 1
        if not t[0].startswith("v_") or t[0].startswith(("v_readfirstlane", "v_readlane", "v_writelane")):
            continue
        srcs = t[1].split(",", 1)[1] if len(t) > 1 and "," in t[1] else ""
        has_s = bool(SGPR.search(srcs))
        full = base_op(t[0]) in FULL_RATE and not has_s
        with_s += has_s
        cycles += 2 if full else 4
        n += 1
    return c, n, cycles, with_s


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    out = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    if out in args:
        args.remove(out)
    res = {}
    for name, body in kernels(args[0]):
        if len(args) > 1 and not re.search(args[1], name):
            continue
        c, n, cyc, with_s = analyse(body)
        res[name] = {"valu_static": n, "valu_cycles_static": cyc, "avg_cycles_per_valu": round(cyc / max(1, n), 3),
                     "valu_with_sgpr_or_literal": with_s}
        print(f"{name}: VALU {n}, {cyc} cycles ({cyc / max(1, n):.2f}/instr), SGPR/literal operands {with_s} | "
              + ", ".join(f"{k}:{v}" for k, v in c.most_common(8)))
    if out:
        json.dump(res, open(out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()

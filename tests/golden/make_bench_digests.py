#!/usr/bin/env python3
"""DAHs of the blocks bench.py extends, so the bench can check its own output against committed data.

bench.py's default workload (k=128) extends 16 distinct synthetic squares per rank, seeds
0xC0FFEE + rank * B + b for b < 16 (B = 128 blocks per GPU per step, replicated 8 times to
fill the batch); ranks 0..7 are covered. Its config C5 probe extends k=512 squares with seeds
0xC0FFEE and 0xC0FFEE + 1. The DAHs come from the CPU oracle (oracle/, pinned by the
reference's fixtures, tests/test_oracle.py); the k=512 (GF(2^16)) ones inherit its
"parity unpinned" status.

Output: tests/golden/bench_digests.json. Run from the repo root (about a minute on 8 cores).
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as O  # noqa: E402

OUT = os.path.join(HERE, "bench_digests.json")
B, DISTINCT, RANKS = 128, 16, 8


def main():
    out = {"k128": {}, "k512": {}, "note": __doc__.strip().splitlines()[0]}
    for r in range(RANKS):
        for b in range(DISTINCT):
            seed = 0xC0FFEE + r * B + b
            rc, _, _, _, dah = O.extend_commit(O.gen_ods(128, seed), want_eds=False)
            assert rc == 0
            out["k128"][str(seed)] = dah.hex()
    for seed in (0xC0FFEE, 0xC0FFEE + 1):
        rc, _, _, _, dah = O.extend_commit(O.gen_ods(512, seed), want_eds=False)
        assert rc == 0
        out["k512"][str(seed)] = dah.hex()
        print("k512", seed, dah.hex())
    json.dump(out, open(OUT, "w"), indent=1)


if __name__ == "__main__":
    main()

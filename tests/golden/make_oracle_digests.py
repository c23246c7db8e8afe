#!/usr/bin/env python3
"""Digests of the oracle's outputs on the seeded synthetic squares (SURVEY.md §8c "golden fixtures").

For k in {1, 2, 4, ..., 256} and seed 0xC0FFEE + k (the generator of SURVEY.md §8d,
oracle/da.c ora_gen_ods): SHA-256 of the EDS bytes, SHA-256 of row roots ‖ column
roots, and the DAH. The oracle itself is pinned by the reference's fixtures
(tests/test_oracle.py); these digests freeze its outputs so a regression in either
the oracle or the device path shows up against committed data, and the GPU tests can
check k up to 256 without recomputing the CPU side.

Output: tests/golden/oracle_digests.json. Run from the repo root.
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as O  # noqa: E402

OUT = os.path.join(HERE, "oracle_digests.json")


def main():
    out = {}
    for k in [1, 2, 4, 8, 16, 32, 64, 128, 256]:
        ods = O.gen_ods(k, 0xC0FFEE + k)
        rc, eds, rr, cr, dah = O.extend_commit(ods)
        assert rc == 0
        out[str(k)] = {"seed": 0xC0FFEE + k, "eds_sha256": hashlib.sha256(eds.tobytes()).hexdigest(),
                       "roots_sha256": hashlib.sha256(rr.tobytes() + cr.tobytes()).hexdigest(), "dah": dah.hex()}
        print(k, out[str(k)]["dah"])
    json.dump(out, open(OUT, "w"), indent=1)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""The reference's own valid ShareProof / RowProof as JSON vectors for the proof verifiers.

Source: /root/reference/pkg/proof/row_proof_test.go:67-89 (root, validRowProof) and
share_proof_test.go:74-93 (validShareProof). Per the comments there, the data comes
from TestNewShareInclusionProof "1 transaction share" of a celestia-app version
whose namespaces were 33 bytes (1 version byte + 32-byte ID). The script only
extracts the byte literals. tests/test_inclusion.py checks the verifiers restated
in oracle/inclusion.c against them.

Output: tests/golden/share_proof_fixture.json. Run from the repo root.
"""
import json
import os
import re

REF = "/root/reference/pkg/proof"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "share_proof_fixture.json")
HEX = re.compile(r"\{\s*(0x[0-9a-fA-F]+(?:\s*,\s*0x[0-9a-fA-F]+)*)\s*,?\s*\}")


def literals(text):
    return [bytes(int(x, 16) for x in m.group(1).split(",")) for m in HEX.finditer(text)]


def func_body(src, name):
    i = src.index(f"func {name}()")
    j = src.find("\nfunc ", i + 1)
    return src[i:j if j > 0 else len(src)]


def main():
    rp = open(os.path.join(REF, "row_proof_test.go")).read()
    sp = open(os.path.join(REF, "share_proof_test.go")).read()
    root = literals(rp[rp.index("var root = "):].split("\n", 1)[0])[0]
    rbody = func_body(rp, "validRowProof")
    r = literals(rbody)  # row root, leaf hash, aunts...
    sbody = func_body(sp, "validShareProof")
    s = literals(sbody)  # data share, nodes...
    nid = bytes(int(x) for x in re.search(r"NamespaceId:\s*\[\]byte\{([^}]*)\}", sbody).group(1).split(","))
    fx = {
        "source": "pkg/proof/row_proof_test.go:67-89, pkg/proof/share_proof_test.go:74-93",
        "root": root.hex(),
        "row_roots": [r[0].hex()],
        "row_proof": {"total": int(re.search(r"Total:\s*(\d+)", rbody).group(1)),
                      "index": int(re.search(r"Index:\s*(\d+)", rbody).group(1)),
                      "leaf_hash": r[1].hex(), "aunts": [a.hex() for a in r[2:]]},
        "start_row": int(re.search(r"StartRow:\s*(\d+)", rbody).group(1)),
        "end_row": int(re.search(r"EndRow:\s*(\d+)", rbody).group(1)),
        "data": [s[0].hex()],
        "nmt": {"start": int(re.search(r"Start:\s*(\d+)", sbody).group(1)),
                "end": int(re.search(r"End:\s*(\d+)", sbody).group(1)), "nodes": [x.hex() for x in s[1:]]},
        "namespace_id": nid.hex(),
        "namespace_version": int(re.search(r"NamespaceVersion:\s*uint32\((\d+)\)", sbody).group(1)),
    }
    json.dump(fx, open(OUT, "w"), indent=1)
    print(f"row proof: {len(fx['row_proof']['aunts'])} aunts; nmt: {len(fx['nmt']['nodes'])} nodes, "
          f"{len(s[0])}-byte share, {len(nid)}-byte namespace id; wrote {os.path.relpath(OUT)}")


if __name__ == "__main__":
    main()

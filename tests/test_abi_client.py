"""The C-ABI client (tests/abi_client/abi_host_client.c) calls libcda exactly as the cgo shim (go/cda) does --
pageable host buffers, flattened shares, 90-byte root records -- in its own process without Python or torch in
between.  Its outputs must equal the committed golden digests (tests/golden/oracle_digests.json) and mainnet
block 408's data_hash (x/blob/test/testdata/block_response.json)."""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

import oracle_lib as O

HERE = os.path.dirname(os.path.abspath(__file__))
CLIENT = os.path.join(HERE, "abi_client", "abi_host_client")


def test_client_is_built():
    assert os.path.exists(CLIENT), "run __graft_entry__.build() (make -C tests/abi_client)"


def _run(tmp_path, ods, k):
    src = tmp_path / "ods.bin"
    src.write_bytes(np.ascontiguousarray(ods, np.uint8).tobytes())
    out = subprocess.run([CLIENT, str(src), str(k), str(tmp_path)], capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stderr
    assert "abi_host_client ok" in out.stdout
    rd = lambda n: (tmp_path / n).read_bytes()  # noqa: E731
    flat = np.ascontiguousarray(ods, np.uint8).tobytes()
    ns, tot = flat[:29], len(flat)
    b1 = min(tot // 2, 1000)
    b2 = min(b1 + 5000, tot)
    for i, (a, b) in enumerate(((0, b1), (b1, b2))):  # the client's two blobs, against oracle/inclusion.c
        rc, want = O.blob_commitment(ns, flat[a:b])
        assert rc == 0 and rd("commitments.bin")[32 * i:32 * (i + 1)] == want, i
    return rd("eds.bin"), rd("row_roots.bin"), rd("col_roots.bin"), rd("dah.bin"), rd("repaired.bin")


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 2, 8, 32, 128])
def test_abi_client_matches_golden_digests(tmp_path, k):
    fx = json.load(open(os.path.join(HERE, "golden", "oracle_digests.json")))[str(k)]
    eds, rr, cr, dah, repaired = _run(tmp_path, O.gen_ods(k, fx["seed"]), k)
    assert dah.hex() == fx["dah"]
    assert hashlib.sha256(eds).hexdigest() == fx["eds_sha256"]
    assert hashlib.sha256(rr + cr).hexdigest() == fx["roots_sha256"]
    assert repaired == eds


@pytest.mark.gpu
def test_abi_client_mainnet_block_408(tmp_path):
    z = np.load(os.path.join(HERE, "golden", "mainnet_h408.npz"))
    eds, rr, cr, dah, repaired = _run(tmp_path, z["ods"], 32)
    assert dah == z["data_hash"].tobytes()
    assert repaired == eds

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


def _run(tmp_path, ods, k, blobs=None):
    src = tmp_path / "ods.bin"
    src.write_bytes(np.ascontiguousarray(ods, np.uint8).tobytes())
    extra = []
    if blobs is not None:  # [(ns29, data)] -> blobs.bin ([u32 n][n x 29][(n + 1) x u64][data])
        offs = np.zeros(len(blobs) + 1, np.uint64)
        offs[1:] = np.cumsum([len(d) for _, d in blobs])
        (tmp_path / "blobs.bin").write_bytes(np.uint32(len(blobs)).tobytes() + b"".join(n for n, _ in blobs) +
                                             offs.tobytes() + b"".join(d for _, d in blobs))
        extra = [str(tmp_path / "blobs.bin")]
    out = subprocess.run([CLIENT, str(src), str(k), str(tmp_path)] + extra, capture_output=True, text=True,
                         timeout=180)
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
    """Block 408 through the C ABI: the DAH is the header's data_hash, and the proposal pre-pass (one
    cda_blob_commitments call over block 408's blob plus synthetic blobs, as ProcessProposal batches every BlobTx)
    reproduces the commitment the block's MsgPayForBlobs carries and the oracle's for the others."""
    z = np.load(os.path.join(HERE, "golden", "mainnet_h408.npz"))
    b = np.load(os.path.join(HERE, "golden", "mainnet_h408_blobs.npz"))
    rng = np.random.default_rng(408)
    blobs = [(b["namespaces"][0].tobytes(), b["data"].tobytes())]
    for n in (1, 511, 4000, 70000):
        blobs.append((bytes(19) + bytes([n % 251 + 1]) + bytes(rng.integers(0, 256, 9, dtype=np.uint8)),
                      bytes(rng.integers(0, 256, n, dtype=np.uint8))))
    eds, rr, cr, dah, repaired = _run(tmp_path, z["ods"], 32, blobs)
    assert dah == z["data_hash"].tobytes()
    assert repaired == eds
    got = (tmp_path / "proposal_commitments.bin").read_bytes()
    assert got[:32] == b["commitments"][0].tobytes()  # the PFB's share commitment in mainnet block 408
    for i, (ns, d) in enumerate(blobs):
        assert got[32 * i:32 * (i + 1)] == O.blob_commitment(ns, d)[1], i

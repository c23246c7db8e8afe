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
# CDA_ABI_CLIENT: another build of the client (scripts/gpu_asan.sh runs these tests with the AddressSanitizer one)
CLIENT = os.environ.get("CDA_ABI_CLIENT") or os.path.join(HERE, "abi_client", "abi_host_client")


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


def _parse_proof(buf, k):
    """proof.bin of the C client (cda_share_inclusion_proof's outputs, rows in order)."""
    info = np.frombuffer(buf[:24], np.uint32)
    start_row, end_row, nrows, total, naunts, max_nodes = (int(x) for x in info)
    at = 24

    def take(n):
        nonlocal at
        out = buf[at:at + n]
        at += n
        return out
    roots = [take(90) for _ in range(nrows)]
    leafs = [take(32) for _ in range(nrows)]
    aunts = [[take(32) for _ in range(naunts)] for _ in range(nrows)]
    s = np.frombuffer(take(4 * nrows), np.int32)
    e = np.frombuffer(take(4 * nrows), np.int32)
    c = np.frombuffer(take(4 * nrows), np.int32)
    nodes = [[take(90) for _ in range(int(c[i]))] for i in range(nrows)]
    root = take(32)
    assert at == len(buf)
    return {"start_row": start_row, "end_row": end_row, "total": total, "data_root": root,
            "rows": [{"row_root": roots[i], "leaf_hash": leafs[i], "aunts": aunts[i], "start": int(s[i]),
                      "end": int(e[i]), "nodes": nodes[i]} for i in range(nrows)]}


@pytest.mark.gpu
def test_abi_client_block_408_proofs_nodes_and_square(tmp_path, ctx):
    """the calls go/cda's f1 / f3 bindings make (go/cda/proof.go, go/cda/square.go, go/patches/0005),
    from the C client on mainnet block 408:
    * NewShareInclusionProof of the block's PFB blob (cda_share_inclusion_proof): equal to the Python binding's
      proof, every row proof verifies against the header's data_hash and every NMT range proof against its row root;
    * the subtree cacher's nodes (cda_extend_commit_nodes): GetCommitment walked over the C client's row nodes gives
      the commitment the block's MsgPayForBlobs carries;
    * square.Construct from the host layout plan of the block's 274 txs (cda_construct_extend_commit): the shares
      equal the block's ODS and the DAH is the data_hash."""
    from cda import inclusion as I
    from cda import square as S
    from cda.da import DataAvailabilityHeader
    from test_inclusion import mainnet_blobs
    from test_proposal import mainnet_txs
    z = np.load(os.path.join(HERE, "golden", "mainnet_h408.npz"))
    data_hash = z["data_hash"].tobytes()
    b = mainnet_blobs()[0]
    start, end = b["start"], b["start"] + b["n"]
    ss, segs, _ = S.plan(mainnet_txs(), 128, 64)
    assert ss == 32
    recs, data, reserved = S.device_plan(segs)
    (tmp_path / "segs.bin").write_bytes(np.uint32(len(recs)).tobytes() + bytes(recs) +
                                        np.uint64(sum(r.data_len for r in recs)).tobytes() + data.tobytes() +
                                        np.uint32(len(reserved)).tobytes() + reserved.tobytes())
    src = tmp_path / "ods.bin"
    src.write_bytes(z["ods"].tobytes())
    out = subprocess.run([CLIENT, str(src), "32", str(tmp_path), "--proof", str(start), str(end), "--nodes",
                          "--segments", str(tmp_path / "segs.bin")], capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stderr
    # f1: share inclusion proof
    got = _parse_proof((tmp_path / "proof.bin").read_bytes(), 32)
    want = ctx.share_inclusion_proof(z["ods"], start, end)
    assert got == want
    assert got["data_root"] == data_hash
    shares = [bytes(s) for s in z["ods"]]
    ns = shares[start][:29]
    cursor = 0
    for i, row in enumerate(got["rows"]):
        r = got["start_row"] + i
        assert O.merkle_verify(got["total"], r, row["leaf_hash"], row["aunts"], data_hash, row["row_root"])
        used = row["end"] - row["start"]
        assert O.nmt_verify_inclusion(ns, shares[start + cursor:start + cursor + used], row["start"], row["end"],
                                      row["nodes"], row["row_root"])
        cursor += used
    assert cursor == end - start
    # f1: node export -> GetCommitment over the exported row trees
    w = 64
    row_nodes = np.frombuffer((tmp_path / "row_nodes.bin").read_bytes(), np.uint8).reshape(w, 2 * w - 1, 90)
    rr = np.frombuffer((tmp_path / "row_roots.bin").read_bytes(), np.uint8).reshape(w, 90)
    cr = np.frombuffer((tmp_path / "col_roots.bin").read_bytes(), np.uint8).reshape(w, 90)
    dah = DataAvailabilityHeader(list(rr), list(cr), ctx=ctx)
    assert dah.hash() == data_hash
    cacher = I.EDSSubTreeRootCacher(32, row_nodes)
    assert I.get_commitment(cacher, dah, b["start"], b["n"], 64, ctx=ctx) == b["commitment"]
    eds = O.extend(z["ods"])
    for t in (0, 17, 63):
        assert np.array_equal(row_nodes[t], O.tree_levels(O.axis_leaf_nodes(eds, 0, t))), t
    # f3: square construction on the device
    assert (tmp_path / "construct_ods.bin").read_bytes() == z["ods"].tobytes()
    assert (tmp_path / "construct_dah.bin").read_bytes() == data_hash

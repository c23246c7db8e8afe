"""One square split over ranks (cda.split).

CPU tests run world-size 2 and 4 `gloo` ranks with the oracle test double
(tests/split_worker.py). They pin the distributed logic: row/column ownership,
the all-to-all layout, the bottom-row subtree fold and the order in which push
errors are reported. The GPU test runs 2 gloo ranks on the one GPU of the box
through libcda (DeviceOps). Every case is checked bit-exact against the
single-process oracle.
"""
import os
import socket

import numpy as np
import pytest

import oracle_lib as O


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(world, k, seed, use_gpu, tmp_path, unsorted=False):
    import torch.multiprocessing as mp
    import split_worker
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=split_worker.run_rank, args=(r, world, port, k, seed, use_gpu, str(tmp_path), unsorted))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(600)
        assert p.exitcode == 0, f"rank exited with {p.exitcode}"
    return [dict(np.load(os.path.join(tmp_path, f"rank{r}.npz"))) for r in range(world)]


def _check(res, k, seed, world):
    from cda import split
    import hashlib
    ods = O.gen_ods(k, seed)
    rc, eds, rr, cr, dah = O.extend_commit(ods)
    assert rc == 0
    w = 2 * k
    E = eds.reshape(w, w, 512)
    for r, out in enumerate(res):
        assert int(out["rc"]) == 0
        assert np.array_equal(out["row_roots"], rr)
        assert np.array_equal(out["col_roots"], cr)
        assert out["dah"].tobytes() == dah
        (a, b), (c, d) = split.plan(k, world, r)
        assert out["rows_sha"].tobytes() == hashlib.sha256(E[a:b].tobytes()).digest()
        assert out["cols_sha"].tobytes() == hashlib.sha256(np.ascontiguousarray(E[:, c:d]).tobytes()).digest()


def test_plan():
    from cda import split
    assert split.plan(512, 8, 3) == ((192, 256), (384, 512))
    assert split.plan(4, 1, 0) == ((0, 4), (0, 8))
    with pytest.raises(ValueError):
        split.plan(4, 3, 0)
    with pytest.raises(ValueError):
        split.plan(2, 4, 0)


@pytest.mark.parametrize("world,k", [(2, 4), (2, 8), (4, 8)])
def test_split_gloo_cpu(tmp_path, world, k):
    _check(_run(world, k, 77 + k, False, tmp_path), k, 77 + k, world)


def test_split_gloo_cpu_push_error(tmp_path):
    k, world = 8, 2
    res = _run(world, k, 5, False, tmp_path, unsorted=True)
    ods = O.gen_ods(k, 5).reshape(k, k, 512).copy()
    ods[1, [2, 3]] = ods[1, [3, 2]]
    eds = O.extend(ods.reshape(k * k, 512))
    rc, _, _, axis, index = O.roots(eds)
    assert rc == O.E_NS_ORDER
    for out in res:
        assert int(out["rc"]) == -5
        assert (int(out["axis"]), int(out["index"])) == (axis, index)
        assert int(out["leaf"]) == 3


@pytest.mark.gpu
@pytest.mark.parametrize("k", [16, 128, 512])
def test_split_gloo_gpu(tmp_path, k):
    """2 ranks on the box's one GPU: HIP kernels via libcda, gloo host-staged exchange."""
    _check(_run(2, k, 900 + k, True, tmp_path), k, 900 + k, 2)

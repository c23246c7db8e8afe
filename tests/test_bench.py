"""bench.py plumbing on CPU: --gpus N spawns N ranks itself (no torchrun), the ranks form a process group and
the max-over-ranks timing collective runs; the CPU baseline sampler counts independent blocks."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_bench(*args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, capture_output=True,
                         text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 prints exactly one JSON line
    return json.loads(lines[0])


def _check_ranks(r, n):
    """The N > 1 line's self-verification: ranks_seen from an all_reduce over the run's group, one
    report per rank (its own step time, host, pid), distinct ranks 0..n-1."""
    rep = r["ranks"]
    assert rep["ranks_seen"] == n and len(rep["per_rank"]) == n
    assert sorted(p["rank"] for p in rep["per_rank"]) == list(range(n))
    assert len({p["pid"] for p in rep["per_rank"]}) == n
    assert [p["ms_per_step"] for p in sorted(rep["per_rank"], key=lambda p: p["rank"])] == [float(i) for i in range(n)]


def test_bench_spawns_two_ranks():
    r = _run_bench("--gpus", "2", "--dry-run")
    assert r["n_gpus"] == 2 and r["ranks_seen"] == 2 and r["max_rank"] == 1
    _check_ranks(r, 2)
    # config C5's split helper (started before the GPU is touched, run between two CPU barriers) answered
    assert r["k512_split"] == {"dry_run": True, "G": 2, "helper_wall_s": r["k512_split"]["helper_wall_s"]}


def test_bench_spawns_four_ranks():
    r = _run_bench("--gpus", "4", "--dry-run")
    assert r["n_gpus"] == 4 and r["ranks_seen"] == 4
    _check_ranks(r, 4)
    assert r["k512_split"]["G"] == 4


def test_bench_spawns_eight_ranks():
    """The driver's N = 8 line: 8 gloo ranks, every rank reports, and config C5's split helper
    answers for G = 8 with its fields (an error field when it fails, never the exit code)."""
    r = _run_bench("--gpus", "8", "--dry-run")
    assert r["n_gpus"] == 8 and r["ranks_seen"] == 8 and r["max_rank"] == 7
    _check_ranks(r, 8)
    split = r["k512_split"]
    assert split.get("G") == 8 or "error" in split
    assert set(split) <= {"dry_run", "G", "helper_wall_s", "error"}


def test_bench_split_helper_failure_is_a_field():
    """A helper that cannot run becomes an error field, not the bench's exit code."""
    sys.path.insert(0, ROOT)
    import bench
    h = bench.SplitHelper(2, dry_run=False)
    h.p.stdin.write("quit\n")  # the helper leaves without answering
    h.p.stdin.flush()
    h.p.wait(timeout=60)
    r = h.run(timeout=5)
    assert "error" in r


def test_cpu_throughput_sampler():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    ods = O.gen_ods(8, 0xC0FFEE)
    n, el = O.extend_commit_throughput(ods, 2, 0.2)
    assert n >= 2 and el > 0.0


def test_bench_workload_helpers():
    sys.path.insert(0, ROOT)
    import bench
    import oracle_lib as O
    # bench's generator is the oracle's ora_gen_ods (same SplitMix64 stream, sorted)
    assert np.array_equal(bench.gen_ods(8, 0xC0FFEE + 3), O.gen_ods(8, 0xC0FFEE + 3))
    assert bench.block_bytes(128) == 41989152
    assert bench.block_compressions_ref(128) == 1573374

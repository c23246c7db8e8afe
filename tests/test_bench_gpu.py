"""bench.py's output contract on the GPU, at a small batch: one JSON line with the BASELINE metric, a whole-job value
consistent with its own step time, the roofline object of the dominant kernel and every block's DAH checked against
the committed digests (the timed steps' output, tests/golden/bench_digests.json)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_line_contract():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1", "--batch", "8",
           "--no-extras", "--no-cpu-baseline", "--no-k512-split"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert d["metric"] == base["metric"]
    for key in ("value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
                "vs_baseline", "dtype", "data", "config", "roofline"):
        assert key in d, key
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1
    assert d["higher_is_better"] is True and d["scaling"] == "weak" and d["vs_baseline"] is None
    # value = blocks of all ranks / elapsed, ms_per_step = elapsed / steps
    assert d["value"] == pytest.approx(8 * 1000.0 / d["ms_per_step"], rel=1e-3)
    r = d["roofline"]
    for key in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert key in r, key
    assert r["peak"] > 0 and 0 < r["frac"] <= 1 and r["frac"] == pytest.approx(r["achieved"] / r["peak"], rel=1e-2)
    assert d["output_check"]["blocks_checked_vs_golden"] == 8

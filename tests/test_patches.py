"""go/patches/000{1..5} apply, in order and without fuzz, to the reference's own files (the integration a maintainer
performs).  CPU only; skipped where /root/reference is absent (the GPU box)."""
import os
import re
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
PATCHES = os.path.join(os.path.dirname(HERE), "go", "patches")
REF = "/root/reference"

pytestmark = pytest.mark.skipif(not os.path.isdir(REF) or shutil.which("patch") is None,
                                reason="needs the reference tree and patch(1)")


def _patches():
    return sorted(os.path.join(PATCHES, f) for f in os.listdir(PATCHES) if f.endswith(".patch"))


def _touched(p):
    out = set()
    for line in open(p, encoding="utf-8"):
        m = re.match(r"^(?:\+\+\+|---) (?:[ab]/)?(\S+)", line)
        if m and m.group(1) != "/dev/null":
            out.add(m.group(1))
    return out


def test_five_patches():
    assert [os.path.basename(p)[:4] for p in _patches()] == ["0001", "0002", "0003", "0004", "0005"]


def test_patches_apply_in_order_to_the_reference(tmp_path):
    files = set().union(*(_touched(p) for p in _patches()))
    for f in files:
        src = os.path.join(REF, f)
        if os.path.exists(src):  # new files (e.g. x/blob/types/commitments_batch.go) are created by their patch
            os.makedirs(os.path.dirname(tmp_path / f), exist_ok=True)
            shutil.copy(src, tmp_path / f)
    for p in _patches():
        r = subprocess.run(["patch", "-p1", "--fuzz=0", "-i", p], cwd=tmp_path, capture_output=True, text=True)
        assert r.returncode == 0, (os.path.basename(p), r.stdout, r.stderr)
        assert "FAILED" not in r.stdout and "fuzz" not in r.stdout, (os.path.basename(p), r.stdout)
    # the seams the Go side hooks exist after patching
    da_go = (tmp_path / "pkg/da/data_availability_header.go").read_text()
    assert "func NewDataAvailabilityHeaderFromShares" in da_go
    assert "da.NewDataAvailabilityHeaderFromShares" in (tmp_path / "app/prepare_proposal.go").read_text()
    assert "da.NewDataAvailabilityHeaderFromShares" in (tmp_path / "app/process_proposal.go").read_text()
    assert "NewSubtreeCacherFromShares" in (tmp_path / "pkg/inclusion/nmt_caching.go").read_text()

"""Static check of the GF(2^16) encoder's hand-counted vmcnt waits (rs16_kernels.hip kAfterPrefetch).

tools/vmcnt_check.py disassembles the gfx950 code object inside the built libcda.so and walks every control-flow path
from each LDS prefetch (8 x global_load_lds_dwordx4, issued by inline asm) to its read-back wait (read_prefetch's
`s_waitcnt vmcnt(N)`), counting the vector-memory instructions issued in between.  CPU only: no kernel runs."""
import os
import shutil
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import vmcnt_check as V  # noqa: E402

LIB = os.path.join(ROOT, "celestia-app_amd", "cda", "libcda.so")

pytestmark = pytest.mark.skipif(not (os.path.exists(V.OBJDUMP) and os.path.exists(LIB)),
                                reason="needs llvm-objdump and the built libcda.so")


@pytest.fixture(scope="module")
def insts(tmp_path_factory):
    import subprocess
    tmp = str(tmp_path_factory.mktemp("co"))
    for co in V.code_objects(LIB, tmp):
        text = subprocess.run([V.OBJDUMP, "-d", co], capture_output=True, text=True, check=True).stdout
        if V.KERNEL in text:
            return V.parse(text)
    pytest.fail("no rs_encode16_reg_kernel in libcda.so")


def test_every_prefetch_wait_equals_its_path_count(insts):
    res = V.check(insts)
    # 8 wave-pair bodies (one per OM), each with the prologue's read-back (vmcnt(8)) and the loop's (vmcnt(24))
    assert sorted(n for _, n, _, _ in res) == [8] * 8 + [24] * 8
    for a, n, lo, hi in res:
        assert lo == hi == n, (hex(a), n, lo, hi)


def test_no_scratch_traffic(insts):
    """A spill is a vector-memory instruction too: it would shift every count."""
    assert not [i for i in insts if i[1].startswith("scratch_")]


def test_check_detects_an_extra_store(insts):
    """A store moved between a loop prefetch and its wait makes that path's count 25 > 24: reported, not hidden."""
    res = V.check(insts)
    wait = next(a for a, n, _, _ in res if n == 24)
    i = next(j for j, x in enumerate(insts) if x[0] == wait)
    bad = insts[:i] + [(insts[i][0] - 2, "global_store_dwordx4", "v[0:1], v[2:5], off", None)] + insts[i:]
    got = {a: (n, lo, hi) for a, n, lo, hi in V.check(bad)}
    assert got[wait] == (24, 25, 25)


def test_cli_reports_ok(capsys):
    assert V.main(LIB) == 0
    assert capsys.readouterr().out.rstrip().endswith("ok")


def test_objdump_present():
    assert shutil.which(V.OBJDUMP) or os.path.exists(V.OBJDUMP)

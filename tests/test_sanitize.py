"""libcda's host planners (celestia-app_amd/csrc/plan.cpp) under AddressSanitizer + UndefinedBehaviorSanitizer,
checked against the naive restatements in tests/san/plan_check.cpp (CPU only; scripts/sanitize.sh adds the
sanitized oracle under the whole CPU suite and keeps the log under profiles/)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_planners_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "plan_check")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                           "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-o", exe,
                           os.path.join(ROOT, "tests", "san", "plan_check.cpp"),
                           os.path.join(ROOT, "celestia-app_amd", "csrc", "plan.cpp")])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="halt_on_error=1")
    out = subprocess.run([exe], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "plan_check: all passed" in out.stdout

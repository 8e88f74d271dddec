"""Host C++ of the GBDT engine under AddressSanitizer + UndefinedBehaviorSanitizer; the TSan
pass runs with `tools/sanitize.sh` (SKIP_TSAN=0)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_gbdt_host_engine_asan_ubsan_clean():
    env = dict(os.environ, SKIP_TSAN="1")
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize.sh")], env=env, capture_output=True, text=True,
                       timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "all native host tests passed" in r.stdout

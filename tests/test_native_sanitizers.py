"""Host C++ under sanitizers, via tools/sanitize.sh:

* ASan + UBSan: the GBDT engine (CPU backend, concurrent pushes / predictions, validation sets, malformed
  models), the VW learner core (every reduction, truncated models, malformed command lines and examples)
  and the image kernels (odd shapes, kernels wider than the image, every colour conversion).
* TSan: the GBDT engine with 4 OpenMP threads (LLVM libomp + Archer, so OpenMP synchronisation is visible
  to TSan) plus 4 std::threads pushing disjoint row blocks and predicting concurrently.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(part: str, marker: str):
    env = dict(os.environ, ONLY=part)
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize.sh")], env=env, capture_output=True, text=True,
                       timeout=1200)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-6000:]
    assert marker in r.stdout and "sanitizers clean" in r.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("part,marker", [("gbdt", "all native host tests passed"),
                                         ("vw", "all native vw host tests passed"),
                                         ("image", "all native image host tests passed")])
def test_host_code_asan_ubsan_clean(part, marker):
    _run(part, marker)


@pytest.mark.skipif(not os.path.exists("/opt/rocm/llvm/bin/clang++") or
                    not os.path.exists("/opt/rocm/llvm/lib/libarcher.so"), reason="needs clang + Archer")
def test_gbdt_engine_tsan_clean_with_threads():
    _run("tsan", "all native host tests passed")

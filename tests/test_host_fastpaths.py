"""The product's exact fast paths (sng_math.h) equal the general expressions bit for bit (host build, CPU only)."""
import json
import os
import shutil
import subprocess
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_fast_division_linear_marcher_and_slab_are_exact():
    d = tempfile.mkdtemp()
    try:
        exe = os.path.join(d, "march_check")
        subprocess.run([HIPCC, "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-I", os.path.join(REPO, "synerfgine_amd", "csrc"),
                        os.path.join(REPO, "tests", "native", "march_check.cpp"), "-o", exe], check=True, capture_output=True)
        out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
        r = json.loads(out.stdout)
        assert r["div"][0] > 7_000_000 and r["div"][1] == 0
        assert r["march"][1] > 100_000 and r["march"][2] == 0
        assert r["slab"][0] > 1_000_000 and r["slab"][1] == 0
        assert r["stepdiv"][0] > 1_000_000 and r["stepdiv"][1] == 0
        assert out.returncode == 0
    finally:
        shutil.rmtree(d, ignore_errors=True)

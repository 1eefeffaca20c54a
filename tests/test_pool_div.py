"""The avg-pool's exact fast division (jr_pool.hip pool_div: reciprocal
multiply + one fma correction, guarded) is bitwise IEEE x / d for every tap
count d of a 3x3 window.  The full proof is the exhaustive run of
tools/verify_pool_div.c over all 2^32 inputs (profiles/r02d_pool_div_exhaustive.txt);
this test compiles the same checker and runs a sample (every 65,537th bit
pattern plus every input around the 2^-100 guard) on the CPU."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_pool_div_matches_ieee_division(tmp_path):
    exe = tmp_path / "verify_pool_div"
    subprocess.run(["gcc", "-O3", "-mfma", "-fopenmp", os.path.join(ROOT, "tools", "verify_pool_div.c"), "-o",
                    str(exe), "-lm"], check=True)
    out = subprocess.run([str(exe), "65537"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "OK" in out.stdout and out.stdout.count("0 mismatches") == 6

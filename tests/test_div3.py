"""The V-cycle kernels' division-free mean of three residual components (pamg_device.h div3):
RN(x * RN(1/3)) corrected by one fma with the exact remainder is RN(x / 3) (Markstein's theorem).
This host check runs the same operation sequence (IEEE fma, as v_fma_f64) against true division
on 10^8 doubles of every exponent in the fast path's range plus structured values, bit for bit."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
SRC = os.path.join(ROOT, "scripts", "micro", "div3_check.c")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_div3_is_correctly_rounded(tmp_path):
    exe = str(tmp_path / "div3_check")
    subprocess.run(["gcc", "-O2", "-mfma", "-ffp-contract=off", "-fopenmp", SRC, "-lm", "-o", exe], check=True)
    r = subprocess.run([exe, "100000000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 mismatches" in r.stdout, r.stdout

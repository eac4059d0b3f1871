"""Checker::value (texture.rs:69-81) decides on sinf(f x) * sinf(f y) * sinf(f z) < 0 with the
platform libm (glibc).  The kernel decides by sign parity (Checker); this runs
the exhaustive proof oracle/tools/sin_sign_check.cpp over EVERY finite float: the double fast
path and the exact integer reduction rtw::pi_parity (csrc/rtw_checker.h, the kernel's code) agree
with glibc's sinf sign, sinf x == x below 2^-12, and |sinf x| >= 3.2e-9 above it."""
import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_sin_sign_proof_exhaustive(tmp_path):
    exe = tmp_path / "sin_sign_check"
    subprocess.run(["g++", "-O2", "-fopenmp", "-ffp-contract=off", str(ROOT / "oracle/tools/sin_sign_check.cpp"),
                    "-o", str(exe)], check=True)
    r = subprocess.run([str(exe), "1"], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout + r.stderr
    m = re.search(r"min\|sinf\| \(\|x\| >= 2\^-12\) ([0-9.e+-]+)", r.stdout)
    assert m and float(m.group(1)) >= 3.2e-9, r.stdout

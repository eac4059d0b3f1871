"""a build cannot carry a parity-breaking or removed compile-time switch.

rtw_kernel.hip refuses (#error) RTW_DIAG_ONE_TRIP (a timing diagnostic that samples the cube, not the
reference's unit ball) and RTW_DIAG_NO_STORE (one that drops the sample stores) unless RTW_ALLOW_NON_REFERENCE is set too, and every switch round 4 removed (the
xoroshiro64+ output RTW_RNG_PLUS, the dropped reciprocal rect test RTW_RECT_RCP, the folded equivalence
switches).  Preprocessing is enough to see the #error, so no device compile runs here."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
SRC = ROOT / "raytracer-weekend_amd" / "csrc" / "rtw_kernel.hip"


def _preprocess(*defs):
    cmd = [HIPCC, "-E", "-x", "hip", "--offload-arch=gfx950", "--cuda-device-only", "-std=c++17",
           "-o", "/dev/null", str(SRC)] + [f"-D{d}" for d in defs]
    return subprocess.run(cmd, capture_output=True, text=True, timeout=300)


pytestmark = pytest.mark.skipif(not Path(HIPCC).exists(), reason="hipcc not installed")


def test_product_build_preprocesses():
    r = _preprocess()
    assert r.returncode == 0, r.stderr[-2000:]


@pytest.mark.parametrize("macro", ["RTW_DIAG_ONE_TRIP", "RTW_DIAG_NO_STORE", "RTW_RNG_PLUS", "RTW_RECT_RCP=1", "RTW_SPH_RCP=0",
                                   "RTW_FAST_RCP=0", "RTW_DIEL_PRE=0", "RTW_START_LDS=0", "RTW_RECT_SELECT=0"])
def test_parity_breaking_or_removed_switch_fails_the_build(macro):
    r = _preprocess(macro)
    assert r.returncode != 0
    assert "#error" in r.stderr or "error:" in r.stderr


@pytest.mark.parametrize("macro", ["RTW_DIAG_ONE_TRIP", "RTW_DIAG_NO_STORE"])
def test_diagnostic_build_needs_explicit_opt_in(macro):
    assert _preprocess(macro, "RTW_ALLOW_NON_REFERENCE").returncode == 0

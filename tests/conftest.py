"""pytest setup: markers, and the two libraries under test.

`rtw` is the product's Python host mirror (raytracer-weekend_amd/, loaded by path because
the directory name is not an identifier); `orc` is the CPU oracle binding (test infra).
"""
import importlib.util
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
REF = Path("/root/reference")


def load_rtw():
    if "rtw_amd" in sys.modules:
        return sys.modules["rtw_amd"]
    pkg = ROOT / "raytracer-weekend_amd"
    spec = importlib.util.spec_from_file_location("rtw_amd", pkg / "__init__.py",
                                                  submodule_search_locations=[str(pkg)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["rtw_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def load_oracle():
    if "rtw_oracle_py" in sys.modules:
        return sys.modules["rtw_oracle_py"]
    spec = importlib.util.spec_from_file_location("rtw_oracle_py", ROOT / "oracle" / "oracle.py")
    mod = importlib.util.module_from_spec(spec)
    sys.modules["rtw_oracle_py"] = mod
    spec.loader.exec_module(mod)
    return mod


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def rtw():
    return load_rtw()


@pytest.fixture(scope="session")
def orc():
    return load_oracle()


@pytest.fixture(scope="session")
def gpu(rtw):
    # -m gpu runs on the MI355X box: a missing device is a failure, never a silent skip
    assert rtw.device_count() >= 1, "no HIP device visible for a gpu-marked test"
    return rtw


@pytest.fixture
def knobs(monkeypatch):
    """monkeypatch with the tuning gate open: the product library reads its RTW_* tuning knobs (kernel
    variants, scheduling parameters, SAH build knobs) only when RTW_TUNING=1."""
    monkeypatch.setenv("RTW_TUNING", "1")
    return monkeypatch

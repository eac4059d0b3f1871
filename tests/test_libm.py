"""The render path's f32 transcendentals (rtw_oracle.c §libm).

Rust's f32::log10 / sin / acos / atan2 call the platform libm; this build defines them as the
correctly rounded values (double evaluation, one rounding).  Pinned here against
(float)(f64 libm) over every input the medium draw can produce (log10 of rand Standard<f32>)
and over dense samples of the other domains; the GPU functions are pinned to these in
tests/test_gpu_parity.py.  glibc 2.35's f32 versions are not correctly rounded: sinf / acosf /
atan2f differ by at most 1 ulp, log10f by at most 2 (checked too)."""
import ctypes
import math

import numpy as np
import pytest

_libm = ctypes.CDLL("libm.so.6")
for _n in ("log10f", "sinf", "acosf"):
    getattr(_libm, _n).restype = ctypes.c_float
    getattr(_libm, _n).argtypes = [ctypes.c_float]
_libm.atan2f.restype = ctypes.c_float
_libm.atan2f.argtypes = [ctypes.c_float, ctypes.c_float]


def cr(fn, a, b=None):
    """Correctly rounded reference: numpy f64 ufunc, rounded once to f32."""
    with np.errstate(all="ignore"):
        a64 = a.astype(np.float64)
        if fn == 0:
            return np.log10(a64).astype(np.float32)
        if fn == 1:
            return np.sin(a64).astype(np.float32)
        if fn == 2:
            return np.arccos(a64).astype(np.float32)
        return np.arctan2(a64, b.astype(np.float64)).astype(np.float32)


def same(x, y):
    return (x.view(np.uint32) == y.view(np.uint32)) | (np.isnan(x) & np.isnan(y))


def test_log10_every_standard_f32(orc):
    """Every value rand's Standard<f32> yields, k * 2^-24 (ConstantMedium's log10 argument)."""
    a = (np.arange(1, 1 << 24, dtype=np.float64) * 2.0 ** -24).astype(np.float32)
    got = orc.libm(0, a)
    assert same(got, cr(0, a)).all()
    assert orc.libm(0, np.array([0.0], np.float32))[0] == -np.inf


@pytest.mark.parametrize("fn,lo,hi,stride", [(1, 0, 0x47000000, 97), (2, 0, 0x3F800001, 37)])
def test_sin_acos_dense(orc, fn, lo, hi, stride):
    """sin over |x| < 32768 (Noise's argument scale z + 10 turb), acos over [-1, 1] (sphere uv)."""
    b = np.arange(lo, hi, stride, dtype=np.uint32)
    a = np.concatenate([b, b | np.uint32(0x80000000)]).view(np.float32)
    got = orc.libm(fn, a)
    assert same(got, cr(fn, a)).all()


def test_atan2_random_and_special(orc):
    rng = np.random.default_rng(3)
    e = rng.integers(100, 150, (2, 1 << 20))
    m = rng.integers(0, 1 << 23, (2, 1 << 20))
    s = rng.integers(0, 2, (2, 1 << 20))
    ab = ((s << 31) | (e << 23) | m).astype(np.uint32).view(np.float32)
    got = orc.libm(3, ab[0], ab[1])
    assert same(got, cr(3, ab[0], ab[1])).all()
    sp = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 1e-45, -1e-45, 3e38], np.float32)
    y, x = np.meshgrid(sp, sp)
    y, x = y.ravel(), x.ravel()
    got = orc.libm(3, y, x)
    want = np.array([_libm.atan2f(float(p), float(q)) for p, q in zip(y, x)], np.float32)
    ulp = np.abs(got.view(np.int32).astype(np.int64) - want.view(np.int32).astype(np.int64))
    assert (same(got, want) | (ulp <= 1)).all()  # C99 Annex F cases as glibc, values within 1 ulp


def test_within_ulps_of_glibc(orc):
    """The correctly rounded value is within 1 ulp of glibc's sinf / acosf, 2 of its log10f."""
    rng = np.random.default_rng(5)
    a = rng.uniform(-1, 1, 20000).astype(np.float32)
    for fn, f in ((1, _libm.sinf), (2, _libm.acosf)):
        got = orc.libm(fn, a)
        want = np.array([f(float(x)) for x in a], np.float32)
        assert (np.abs(got.view(np.int32).astype(np.int64) - want.view(np.int32).astype(np.int64)) <= 1).all()
    u = (rng.integers(1, 1 << 24, 20000) * 2.0 ** -24).astype(np.float32)
    got = orc.libm(0, u)
    want = np.array([_libm.log10f(float(x)) for x in u], np.float32)
    assert (np.abs(got.view(np.int32).astype(np.int64) - want.view(np.int32).astype(np.int64)) <= 2).all()
    assert math.isclose(float(orc.libm(2, np.array([-1.0], np.float32))[0]), math.pi, rel_tol=1e-7)

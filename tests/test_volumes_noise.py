"""ConstantMedium / Isotropic (volumes.rs, material.rs:148-165) and Perlin Noise (perlin.rs,
texture.rs:83-95): the oracle against the independent numpy restatement's golden vectors
(tests/golden/make_golden.py), plus the host-side Perlin::new and scene-builder checks."""
import ctypes as C
from pathlib import Path

import numpy as np
import pytest

G = np.load(Path(__file__).parent / "golden" / "golden.npz")


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


def test_perlin_noise_and_turbulence(orc):
    grad, perm = G["perlin_grad"], G["perlin_perm"]
    for p, want_n, want_t in zip(G["perlin_pts"], G["perlin_noise"], G["perlin_turb"]):
        assert bits(orc.noise(grad, perm, p, 0)) == bits(want_n), p
        assert bits(orc.noise(grad, perm, p, 7)) == bits(want_t), p


def test_noise_lattice_points_are_zero(orc):
    """perlin.rs: at lattice points every corner's weight vector or blend vanishes."""
    grad, perm = G["perlin_grad"], G["perlin_perm"]
    for p in ([0, 0, 0], [3, -7, 250], [-1, -1, -1]):
        assert orc.noise(grad, perm, np.array(p, np.float32), 0) == 0.0


def test_perlin_new_matches_restatement(rtw):
    """Perlin::new(rng) (perlin.rs:14-48) on the build's seeded scene stream."""
    g, p = rtw.perlin_generate(7)
    assert np.array_equal(bits(g), bits(G["perlin_new_grad"]))
    assert np.array_equal(p, G["perlin_new_perm"])
    for a in range(3):
        assert sorted(p[a].tolist()) == list(range(256))
    assert np.allclose(np.linalg.norm(g, axis=1), 1.0, atol=1e-6)


def test_medium_hits(orc):
    """volumes.rs:37-78 in the build's order-independent form (sub-stream draw, unclipped rec2)."""
    for row, want in zip(G["medium_in"], G["medium_out"]):
        kind, dens = int(row[0]), np.float32(row[1])
        par = np.asarray(row[2:8], np.float32)
        ray = np.asarray(row[8:15], np.float32)
        seg = int(row[15]) | (int(row[16]) << 32)
        key = int(row[17])
        t = (C.c_float * 1)()
        hit = orc.lib().oracle_medium_hit(kind, orc.fp(par), dens, orc.fp(ray), 0.001, np.inf, seg, key, t)
        assert hit == int(want[0]), row
        if hit:
            assert bits(t[0]) == bits(want[1]), row


def test_medium_density_limits(orc):
    """A vanishing density never scatters (hit_distance > distance inside); a huge one scatters at
    the entry point (t -> rec1_t, volumes.rs:56-64)."""
    ray = np.array([-3, 0.1, 0.2, 1, 0, 0, 0.5], np.float32)
    sph = np.array([0, 0, 0, 1, 0, 0], np.float32)
    t = (C.c_float * 1)()
    for seg in range(50):
        assert orc.lib().oracle_medium_hit(0, orc.fp(sph), 1e-30, orc.fp(ray), 0.001, np.inf, seg, 3, t) == 0
        assert orc.lib().oracle_medium_hit(0, orc.fp(sph), 1e30, orc.fp(ray), 0.001, np.inf, seg, 3, t) == 1
        entry = np.float32(-(-3.0) - np.sqrt(np.float32(1 - 0.1 ** 2 - 0.2 ** 2)))
        assert abs(t[0] - entry) < 1e-5
    # t_max below the scattering point: no hit (the closest-hit comparison)
    assert orc.lib().oracle_medium_hit(0, orc.fp(sph), 1e30, orc.fp(ray), 0.001, 1.0, 0, 3, t) == 0


def test_constant_medium_builder(rtw):
    s = rtw.Scene()
    white = s.solid_rgb(1, 1, 1)
    m = s.lambertian(white)
    with s.constant_medium(0.5, white):
        with s.translate((1, 0, 0)), s.rotate_y(30):
            s.cuboid((0, 0, 0), (1, 2, 1), m)
    text = s.dump()
    assert "begin medium" in text and "isotropic" in text
    assert s.info(0) == 1  # the medium is one world leaf; its boundary is not
    bad = rtw.Scene()
    w2 = bad.solid_rgb(1, 1, 1)
    m2 = bad.lambertian(w2)
    with pytest.raises(rtw.RtwError):
        with bad.constant_medium(0.5, w2):
            bad.sphere((0, 0, 0), 1, m2)
            bad.sphere((0, 0, 2), 1, m2)  # two boundary objects: ConstantMedium wraps one Hittable


def test_noise_texture_validates_permutations(rtw):
    s = rtw.Scene()
    g, p = rtw.perlin_generate(1)
    p = p.copy()
    p[1, 5] = p[1, 6]
    with pytest.raises(rtw.RtwError):
        s.noise(4.0, (g, p))

"""The far-origin bound of DESIGN.md §2 against the reference's f32 sphere test itself (CPU, numpy float32).

spherical.rs:26-44 evaluates, in f32 and in this order, oc = o - c, a = |d|², half_b = oc·d, c = |oc|² - r²,
disc = half_b² - a·c, then the nearer root in (t_min, t_max), else the farther one, and the hit point o + t·d.  For
distant origins the subtraction cancels and rays that miss the sphere by a little "hit" it.  rtw_flatten.cpp
(sphere_reach, far_bound) claims such a reported point lies within r + reach(D, r) of the centre, D = |oc|:
reach = min(x / 2r, sqrt x) + u·D with x = 40u(D² + r²), u = 2^-24 (37u derived to first order, 40u kept).
Here random rays aimed just outside spheres of many radii from many distances are put through the reference's
arithmetic (each numpy float32 operation rounds once, as Rust's f32 does, no fused multiply-add), and every
reported hit point must lie inside that bound -- while spurious hits must exist (the bound is not vacuous).
"""
import numpy as np

U = 2.0 ** -24


def _reach(D, r):
    x = 40.0 * U * (D * D + r * r)
    return np.minimum(x / (2.0 * r), np.sqrt(x)) + U * D


def _dot(a, b):
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]


def _reference_hit(o, d, c, r, t_min=np.float32(0.001), t_max=np.float32(np.inf)):
    """spherical.rs:26-44 in f32: (hit, t) per ray."""
    oc = [o[k] - c[k] for k in range(3)]
    a = _dot(d, d)
    half_b = _dot(oc, d)
    cc = _dot(oc, oc) - r * r
    disc = half_b * half_b - a * cc
    with np.errstate(invalid="ignore"):
        sq = np.sqrt(disc)
        root = (-half_b - sq) / a
        bad = (root < t_min) | (t_max < root)
        root = np.where(bad, (-half_b + sq) / a, root)
        bad2 = (root < t_min) | (t_max < root)
    hit = (disc >= 0) & ~bad2
    return hit, root


def test_far_origin_hits_stay_inside_the_bound():
    rng = np.random.default_rng(20260618)
    n = 400_000
    worst, spurious = 0.0, 0
    for _ in range(6):
        D = 10.0 ** rng.uniform(1.0, 3.7, n)            # origin distance 10 .. 5,000
        r = 10.0 ** rng.uniform(-1.3, 0.5, n)           # radius 0.05 .. 3
        c = rng.uniform(-20.0, 20.0, (3, n))            # sphere centre
        u1 = rng.normal(size=(3, n))
        u1 /= np.linalg.norm(u1, axis=0)
        o = c + u1 * D                                  # origin D from the centre
        # aim past the centre at a miss distance rho in [0.9 r, r + 1.5 reach]: grazing and near-miss rays
        rho = r * 0.9 + rng.uniform(0.0, 1.0, n) * (0.1 * r + 1.5 * _reach(D, r))
        w = rng.normal(size=(3, n))
        w -= u1 * (w * u1).sum(axis=0)
        w /= np.linalg.norm(w, axis=0)
        target = c + w * rho
        d = (target - o) * rng.uniform(0.3, 3.0, n)     # unnormalised directions, as the reference's bounces
        f = np.float32
        o32, d32, c32, r32 = [o[k].astype(f) for k in range(3)], [d[k].astype(f) for k in range(3)], \
            [c[k].astype(f) for k in range(3)], r.astype(f)
        hit, t = _reference_hit(o32, d32, c32, r32)
        p = [o32[k] + t * d32[k] for k in range(3)]     # the hit point as the reference forms it (f32)
        dist = np.sqrt(sum((p[k].astype(np.float64) - c32[k].astype(np.float64)) ** 2 for k in range(3)))
        Dx = np.sqrt(sum((o32[k].astype(np.float64) - c32[k].astype(np.float64)) ** 2 for k in range(3)))
        r64 = r32.astype(np.float64)
        # the bound of the sphere test plus the linear roundings of the hit point (16u (D + M), M = the scene's size)
        M = np.maximum.reduce([np.abs(x.astype(np.float64)) for x in c32]) + r64
        bound = r64 + _reach(Dx, r64) + 16.0 * U * (Dx + M)
        h = hit & np.isfinite(t)
        over = (dist - r64)[h] / (bound - r64)[h]
        worst = max(worst, float(over.max()))
        spurious += int(((dist - r64)[h] > 1e-6 * Dx[h]).sum())
        assert (dist[h] <= bound[h]).all(), (dist[h][dist[h] > bound[h]][:4], bound[h][dist[h] > bound[h]][:4])
    assert spurious > 1000, spurious  # far-origin spurious hits are common: the bound is exercised
    assert worst > 0.05, worst        # and some come within reach of it (it is not loose by orders of magnitude)

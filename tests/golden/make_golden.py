"""Independent numpy-float32 restatement of the reference hot path -> golden vectors.

Written separately from oracle/rtw_oracle.c (not a translation of it) straight from the
reference lines cited below, to pin the C oracle: tests/test_golden.py checks the oracle
bit-for-bit against the vectors this script writes to tests/golden/golden.npz.
tanf/sinf/cosf (camera and YRotation set-up, host side) call the C library through ctypes —
the libm functions Rust's f32 methods call in the reference build.  acosf/atan2f (sphere uv, on
the render path) are the correctly rounded values, (float) of the f64 result: glibc's f32
versions are only faithfully rounded and other platforms differ, so this build defines the
render path's transcendentals as correctly rounded (rtw_oracle.c §libm).

    python tests/golden/make_golden.py        # rewrites tests/golden/golden.npz
"""
from __future__ import annotations

import ctypes
import math
from pathlib import Path

import numpy as np

F = np.float32
M64 = (1 << 64) - 1
_libm = ctypes.CDLL("libm.so.6")
for _n in ("tanf", "sinf", "cosf", "acosf"):
    getattr(_libm, _n).restype = ctypes.c_float
    getattr(_libm, _n).argtypes = [ctypes.c_float]
_libm.atan2f.restype = ctypes.c_float
_libm.atan2f.argtypes = [ctypes.c_float, ctypes.c_float]


def tanf(x): return F(_libm.tanf(float(x)))
def sinf(x): return F(_libm.sinf(float(x)))
def cosf(x): return F(_libm.cosf(float(x)))
def acosf(x): return F(math.acos(float(x)))                 # correctly rounded (see docstring)
def atan2f(y, x): return F(math.atan2(float(y), float(x)))


# ------------------------------------------------------------------ bit sources (this build's RNG)
def splitmix64(z: int) -> int:
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


class Pcg32:
    def __init__(self, state: int):
        self.s = state & M64

    def next_u32(self) -> int:
        old = self.s
        self.s = (old * 6364136223846793005 + 1442695040888963407) & M64
        xs = (((old >> 18) ^ old) >> 27) & 0xFFFFFFFF
        rot = old >> 59
        return ((xs >> rot) | (xs << ((32 - rot) & 31))) & 0xFFFFFFFF


class Xoro64:
    """xoroshiro64* (Blackman & Vigna 2018): this build's per-path stream (DESIGN.md §Parity RNG)."""

    def __init__(self, state: int):
        self.s0, self.s1 = state & 0xFFFFFFFF, (state >> 32) & 0xFFFFFFFF

    @staticmethod
    def rotl(x, k):
        return ((x << k) | (x >> (32 - k))) & 0xFFFFFFFF

    def next_u32(self) -> int:
        s0, s1 = self.s0, self.s1
        result = (s0 * 0x9E3779BB) & 0xFFFFFFFF
        s1 ^= s0
        self.s0 = self.rotl(s0, 26) ^ s1 ^ ((s1 << 9) & 0xFFFFFFFF)
        self.s1 = self.rotl(s1, 13)
        return result

    @property
    def state(self) -> int:
        return self.s0 | (self.s1 << 32)


def xoro_seed(h: int) -> int:
    return h if h else 0x9E3779B97F4A7C15


class Draws:
    """Explicit u32 stream (unit vectors) with rand 0.9's float conversions."""

    def __init__(self, src):
        self.src = src
        self.used = 0

    def u32(self) -> int:
        self.used += 1
        if isinstance(self.src, (Pcg32, Xoro64)):
            return self.src.next_u32()
        return int(self.src[self.used - 1]) if self.used - 1 < len(self.src) else 0x80000000

    def gen_f32(self) -> np.float32:  # Standard<f32>: 24 high bits
        return F(self.u32() >> 8) * F(1.0 / 16777216.0)

    def gen_range(self, lo, hi) -> np.float32:  # UniformFloat::sample_single
        lo, hi = F(lo), F(hi)
        scale = F(hi - lo)
        while True:
            v12 = np.array([(self.u32() >> 9) | 0x3F800000], np.uint32).view(np.float32)[0]
            res = F(F(v12 - F(1.0)) * scale) + lo
            res = F(res)
            if res < hi:
                return res
            scale = np.array([scale], np.float32).view(np.uint32)
            scale = (scale - np.uint32(1)).view(np.float32)[0]


def path_state(seed, j, i, s):
    return xoro_seed(splitmix64(splitmix64(seed) ^ ((j << 48) | (i << 32) | s)))


# ------------------------------------------------------------------ vec3.rs
def v(x, y, z): return np.array([x, y, z], np.float32)
def dot(a, b): return F(F(F(a[0] * b[0]) + F(a[1] * b[1])) + F(a[2] * b[2]))
def len2(a): return dot(a, a)
def cross(a, b):
    return np.array([F(a[1] * b[2]) - F(a[2] * b[1]), F(a[2] * b[0]) - F(a[0] * b[2]),
                     F(a[0] * b[1]) - F(a[1] * b[0])], np.float32)
def unit(a): return (a / np.sqrt(len2(a))).astype(np.float32)
def reflect(a, n): return (a - n * F(F(2.0) * dot(a, n))).astype(np.float32)


def refract(uv, n, eta):  # vec3.rs:144-151
    cos_t = min(dot(-uv, n), F(1.0))
    perp = ((uv + n * cos_t) * F(eta)).astype(np.float32)
    k = -np.sqrt(F(abs(F(F(1.0) - len2(perp)))))
    return (perp + n * F(k)).astype(np.float32)


def in_unit_sphere(d):  # vec3.rs:101-108
    while True:
        p = v(d.gen_range(-1, 1), d.gen_range(-1, 1), d.gen_range(-1, 1))
        if len2(p) < F(1.0):
            return p


def in_unit_disk(d):  # vec3.rs:124-131
    while True:
        p = v(d.gen_range(-1, 1), d.gen_range(-1, 1), 0.0)
        if len2(p) < F(1.0):
            return p


# ------------------------------------------------------------------ camera.rs
def camera_new(lf, la, up, vfov, aspect, aperture, focus, t0=0.0, t1=1.0):
    theta = F(F(vfov) * F(F(math.pi) / F(180.0)))
    h = tanf(F(theta / F(2.0)))
    vh = F(F(2.0) * h)
    vw = F(F(aspect) * vh)
    lf, la, up = v(*lf), v(*la), v(*up)
    w = unit((lf - la).astype(np.float32))
    u = unit(cross(up, w))
    vv = cross(w, u)
    hor = (u * F(F(focus) * vw)).astype(np.float32)
    ver = (vv * F(F(focus) * vh)).astype(np.float32)
    llc = (((lf - hor / F(2.0)) - ver / F(2.0)) - w * F(focus)).astype(np.float32)
    return dict(origin=lf, lower_left_corner=llc, horizontal=hor, vertical=ver, u=u, v=vv, w=w,
                lens_radius=F(F(aperture) / F(2.0)), time0=F(t0), time1=F(t1))


def get_ray(c, s, t, d):  # camera.rs:66-74
    rd = (in_unit_disk(d) * c["lens_radius"]).astype(np.float32)
    off = (c["u"] * rd[0] + c["v"] * rd[1]).astype(np.float32)
    o = (c["origin"] + off).astype(np.float32)
    dirn = ((((c["lower_left_corner"] + c["horizontal"] * F(s)) + c["vertical"] * F(t)) - c["origin"]) - off)
    return o, dirn.astype(np.float32), d.gen_range(c["time0"], c["time1"])


# ------------------------------------------------------------------ hittables
def face(d, outward):  # hittable/mod.rs:32-48
    front = dot(d, outward) < F(0.0)
    return (outward if front else -outward).astype(np.float32), front


def sphere_uv(p):  # spherical.rs:62-77
    pi = F(math.pi)
    theta = acosf(-p[1])
    phi = F(atan2f(-p[2], p[0]) + pi)
    return F(phi / F(F(2.0) * pi)), F(theta / pi)


def hit_sphere(o, d, tmin, tmax, c, r):  # spherical.rs:18-60
    oc = (o - c).astype(np.float32)
    a = len2(d)
    hb = dot(oc, d)
    cc = F(len2(oc) - F(F(r) * F(r)))
    disc = F(F(hb * hb) - F(a * cc))
    if disc < F(0.0):
        return None
    sq = np.sqrt(disc)
    root = F(F(-hb - sq) / a)
    if root < tmin or tmax < root:
        root = F(F(-hb + sq) / a)
        if root < tmin or tmax < root:
            return None
    p = (o + d * root).astype(np.float32)
    outward = ((p - c) / F(r)).astype(np.float32)
    uvu, uvv = sphere_uv(outward)
    n, front = face(d, outward)
    return root, p, n, uvu, uvv, front


def center_at(c0, t0, c1, t1, time):  # spherical.rs:117-123
    return (c0 + (c1 - c0) * F(F(F(time) - F(t0)) / F(F(t1) - F(t0)))).astype(np.float32)


def hit_rect(o, d, tmin, tmax, axis, a0, a1, b0, b1, k):  # rectangular.rs:27-159
    kx, ax, bx = [(2, 0, 1), (1, 0, 2), (0, 1, 2)][axis]
    t = F(F(F(k) - o[kx]) / d[kx])
    if t < tmin or t > tmax:
        return None
    x = F(o[ax] + F(t * d[ax]))
    y = F(o[bx] + F(t * d[bx]))
    if x < a0 or x > a1 or y < b0 or y > b1:
        return None
    uu = F(F(x - F(a0)) / F(F(a1) - F(a0)))
    vv = F(F(y - F(b0)) / F(F(b1) - F(b0)))
    outward = np.zeros(3, np.float32)
    outward[kx] = 1.0
    p = (o + d * t).astype(np.float32)
    n, front = face(d, outward)
    return t, p, n, uu, vv, front


def hit_tri(o, d, tmin, tmax, verts):  # triangular.rs:97-138 (default normals / uvs)
    a, b, c = verts
    ab, ac = (b - a).astype(np.float32), (c - a).astype(np.float32)
    n = cross(ab, ac)
    det = -dot(d, n)
    inv = F(F(1.0) / det)
    ao = (o - a).astype(np.float32)
    x = cross(ao, d)
    u = F(dot(ac, x) * inv)
    vv = F(-dot(ab, x) * inv)
    t = F(dot(ao, n) * inv)
    if t < tmin or t > tmax:
        return None
    if not (t >= 0 and u >= 0 and vv >= 0 and F(u + vv) <= 1):
        return None
    p = (o + d * t).astype(np.float32)
    w = F(F(F(1.0) - u) - vv)
    hn = ((n * w + n * u) + n * vv).astype(np.float32)
    uvs = [(0, 0), (1, 0), (0, 1)]
    huu = F(F(F(w * F(uvs[0][0])) + F(u * F(uvs[1][0]))) + F(vv * F(uvs[2][0])))
    hvv = F(F(F(w * F(uvs[0][1])) + F(u * F(uvs[1][1]))) + F(vv * F(uvs[2][1])))
    nn, front = face(d, hn)
    return t, p, nn, huu, hvv, front


def aabb_hit(mn, mx, o, d, tmin, tmax):  # aabb.rs:23-48
    tmin, tmax = F(tmin), F(tmax)
    with np.errstate(all="ignore"):
        for a in range(3):
            inv = F(F(1.0) / d[a])
            t0 = F(F(mn[a] - o[a]) * inv)
            t1 = F(F(mx[a] - o[a]) * inv)
            if inv < 0:
                t0, t1 = t1, t0
            tmin = F(np.fmax(t0, tmin))
            tmax = F(np.fmin(t1, tmax))
            if tmax <= tmin:
                return False
    return True


# ------------------------------------------------------------------ material.rs
def reflectance(cos, ri):  # material.rs:108-112, powi(5) = x * ((x*x)*(x*x))
    r0 = F(F(F(1.0) - F(ri)) / F(F(1.0) + F(ri)))
    r0 = F(r0 * r0)
    x = F(F(1.0) - cos)
    x2 = F(x * x)
    return F(r0 + F(F(F(1.0) - r0) * F(x * F(x2 * x2))))


def scatter(kind, params, d_in, p, n, front, draws):
    """-> (scattered?, direction, attenuation)"""
    if kind == 0:  # Lambertian material.rs:42-56
        dirn = (n + unit(in_unit_sphere(draws))).astype(np.float32)
        if all(abs(dirn) < F(1e-8)):
            dirn = n
        return True, dirn, v(*params[:3])
    if kind == 1:  # Metal :78-95
        refl = reflect(unit(d_in), n)
        dirn = (refl + in_unit_sphere(draws) * F(params[3])).astype(np.float32)
        return bool(dot(dirn, n) > F(0.0)), dirn, v(*params[:3])
    ir = F(params[3])  # Dielectric :116-142
    ratio = F(F(1.0) / ir) if front else ir
    ud = unit(d_in)
    cos_t = min(dot(-ud, n), F(1.0))
    sin_t = np.sqrt(F(F(1.0) - F(cos_t * cos_t)))
    cannot = F(ratio * sin_t) > F(1.0)
    if cannot or reflectance(cos_t, ratio) > draws.gen_f32():
        dirn = reflect(ud, n)
    else:
        dirn = refract(ud, n, ratio)
    return True, dirn, v(1, 1, 1)


def tonemap(s, spp):  # console_app/src/main.rs:78-88
    with np.errstate(invalid="ignore"):
        c = np.sqrt(F(F(F(1.0) / F(spp)) * F(s)))
    if np.isnan(c):
        return 0
    c = min(max(c, F(0.0)), F(0.999))
    x = F(F(255.999) * c)
    return int(min(255, max(0, math.floor(x))))


# ------------------------------------------------------------------ jumpy-balls (scenes.rs:63-162)
def scene_rng(seed):
    return Pcg32(splitmix64(splitmix64(seed) ^ 0x5343454E45))


def jumpy_balls(seed):
    """-> list of spheres (c0[3], t0, c1[3], t1, r, mat) and materials list."""
    r = Pcg32(0)
    r = scene_rng(seed)
    d = Draws(r)
    mats = [("checker",), (0, (0.4, 0.2, 0.1)), (2, 1.5), (1, (0.7, 0.6, 0.5), 0.0)]
    sph = [((0, -1000, 0), 1000.0, 0), ((-4, 0.2, 0.1), 1.0, 1), ((0, 1, 0), 1.0, 2), ((0, 1, 0), -0.95, 2),
           ((4, 1, 0), 1.0, 3)]
    out = [(v(*c), F(0), v(*c), F(1), F(rad), m, False) for c, rad, m in sph]
    for a in range(-11, 11):
        for b in range(-11, 11):
            cx = F(F(a) + F(F(0.9) * d.gen_f32()))
            cy = F(0.2)
            cz = F(F(b) + F(F(0.9) * d.gen_f32()))
            dd = v(cx - F(4.0), cy - F(0.2), cz - F(0.0))
            if np.sqrt(len2(dd)) <= F(0.9):
                continue
            lo, hi = d.u32(), d.u32()
            choose = ((hi << 32 | lo) >> 11) * (1.0 / 9007199254740992.0)
            if choose < 0.8:
                r1 = [d.gen_range(0, 1) for _ in range(3)]
                r2 = [d.gen_range(0, 1) for _ in range(3)]
                mats.append((0, tuple(F(x * y) for x, y in zip(r1, r2))))
            elif choose < 0.95:
                al = tuple(d.gen_range(0.5, 1.0) for _ in range(3))
                mats.append((1, al, d.gen_range(0.0, 0.5)))
            else:
                mats.append((2, 1.5))
            c2y = F(cy + d.gen_range(0.0, 0.5))
            out.append((v(cx, cy, cz), F(0), v(cx, c2y, cz), F(1), F(0.2), len(mats) - 1, True))
    return out, mats


def render_jumpy(w, h, spp, scene_seed, seed, aspect):
    sph, mats = jumpy_balls(scene_seed)
    cam = camera_new((13, 2, 3), (0, 0, 0), (0, 1, 0), 20.0, aspect, 0.1, 10.0)
    C0 = np.stack([s[0] for s in sph]); C1 = np.stack([s[2] for s in sph])
    T0 = np.array([s[1] for s in sph], np.float32); T1 = np.array([s[3] for s in sph], np.float32)
    R = np.array([s[4] for s in sph], np.float32)
    moving = np.array([s[6] for s in sph])
    bg = v(0.7, 0.8, 1.0)
    img = np.zeros((h, w, 3), np.float32)
    rays = 0
    for j in range(h - 1, -1, -1):
        for i in range(w):
            tot = v(0, 0, 0)
            for s in range(spp):
                d = Draws(Xoro64(path_state(seed, j, i, s)))
                uu = F(F(F(i) + d.gen_f32()) / F(w - 1))
                vv = F(F(F(j) + d.gen_f32()) / F(h - 1))
                o, dirn, time = get_ray(cam, uu, vv, d)
                T = v(1, 1, 1)
                col = v(0, 0, 0)
                for _depth in range(50):
                    rays += 1
                    # all spheres at once (element-wise float32 ops in the reference's order)
                    frac = ((F(time) - T0) / (T1 - T0)).astype(np.float32)
                    cen = np.where(moving[:, None], (C0 + (C1 - C0) * frac[:, None]).astype(np.float32), C0)
                    oc = (o[None, :] - cen).astype(np.float32)
                    a = len2(dirn)
                    hb = ((oc[:, 0] * dirn[0] + oc[:, 1] * dirn[1]) + oc[:, 2] * dirn[2]).astype(np.float32)
                    cc = (((oc[:, 0] * oc[:, 0] + oc[:, 1] * oc[:, 1]) + oc[:, 2] * oc[:, 2]) - R * R)
                    disc = (hb * hb - a * cc.astype(np.float32)).astype(np.float32)
                    with np.errstate(invalid="ignore"):
                        sq = np.sqrt(disc)
                        r1 = ((-hb - sq) / a).astype(np.float32)
                        r2 = ((-hb + sq) / a).astype(np.float32)
                    root = np.where(r1 < F(0.001), r2, r1)
                    ok = (disc >= 0) & (root >= F(0.001))
                    if not ok.any():
                        col = (T * bg).astype(np.float32)
                        break
                    tmin_all = root[ok].min()
                    k = int(np.nonzero(ok & (root == tmin_all))[0].max())  # later object wins ties
                    t = root[k]
                    p = (o + dirn * t).astype(np.float32)
                    outward = ((p - cen[k]) / R[k]).astype(np.float32)
                    n, front = face(dirn, outward)
                    m = mats[sph[k][5]]
                    if m[0] == "checker":
                        sines = F(F(sinf(F(10.0) * p[0]) * sinf(F(10.0) * p[1])) * sinf(F(10.0) * p[2]))
                        alb = (0.2, 0.3, 0.1) if sines < 0 else (0.9, 0.9, 0.9)
                        ok2, nd, att = scatter(0, alb, dirn, p, n, front, d)
                    elif m[0] == 0:
                        ok2, nd, att = scatter(0, m[1], dirn, p, n, front, d)
                    elif m[0] == 1:
                        ok2, nd, att = scatter(1, tuple(m[1]) + (m[2],), dirn, p, n, front, d)
                    else:
                        ok2, nd, att = scatter(2, (1, 1, 1, m[1]), dirn, p, n, front, d)
                    if not ok2:
                        col = v(0, 0, 0)
                        break
                    T = (T * att).astype(np.float32)
                    o, dirn = p, nd
                tot = (tot + col).astype(np.float32)
            img[h - 1 - j, i] = tot
    return img, rays, cam


# ------------------------------------------------------------------ Perlin (perlin.rs), Noise (texture.rs:89-95)
def log10f(x): return F(-np.inf) if x == 0 else F(math.log10(float(x)))   # correctly rounded
def sinf_cr(x): return F(math.sin(float(x)))


def perlin_noise(grad, perm, p):  # perlin.rs:50-76, interp :93-117 (filtered point for both uses)
    fl = np.floor(p).astype(np.float32)
    base = [int(x) for x in fl]
    w = (p - fl).astype(np.float32)
    f = ((w * w).astype(np.float32) * (F(3.0) - F(2.0) * w).astype(np.float32)).astype(np.float32)
    acc = F(0.0)
    one = v(1, 1, 1)
    for i in range(2):
        for j in range(2):
            for k in range(2):
                hsh = perm[0][(base[0] + i) & 255] ^ perm[1][(base[1] + j) & 255] ^ perm[2][(base[2] + k) & 255]
                c = v(i, j, k)
                wv = (f - c).astype(np.float32)
                bl = ((c * f).astype(np.float32) + ((one - c) * (one - f)).astype(np.float32)).astype(np.float32)
                bf = F(F(bl[0] * bl[1]) * bl[2])
                acc = F(acc + F(bf * dot(grad[hsh], wv)))
    return acc


def turbulence(grad, perm, p, depth=7):  # perlin.rs:78-91
    acc, weight, tp = F(0.0), F(1.0), p.astype(np.float32)
    for _ in range(depth):
        acc = F(acc + F(weight * perlin_noise(grad, perm, tp)))
        weight = F(weight * F(0.5))
        tp = (tp * F(2.0)).astype(np.float32)
    return F(abs(acc))


def perlin_new(d):  # perlin.rs:14-48 with the scene stream; usize gen_range(0..i) as a widening multiply
    grad = np.array([unit(v(d.gen_range(-1, 1), d.gen_range(-1, 1), d.gen_range(-1, 1))) for _ in range(256)],
                    np.float32)
    perms = []
    for _ in range(3):
        p = list(range(256))
        for i in range(255, 0, -1):
            t = (d.u32() * i) >> 32
            p[i], p[t] = p[t], p[i]
        perms.append(p)
    return grad, np.array(perms, np.uint32)


# ------------------------------------------------------------------ ConstantMedium (volumes.rs:37-78)
def medium_hit(kind, par, o, d, tmin, tmax, density, seg, key):
    """The build's order-independent form: rec2 unclipped, draw from the (segment, key) sub-stream."""
    neg_inv = F(F(-1.0) / F(density))
    def boundary(lo):
        if kind == 0:
            h = hit_sphere(o, d, F(lo), F(np.inf), par[:3], par[3])
            return None if h is None else h[0]
        p0, p1 = par[:3], par[3:6]
        sides = [(0, p0[0], p1[0], p0[1], p1[1], p1[2]), (0, p0[0], p1[0], p0[1], p1[1], p0[2]),
                 (1, p0[0], p1[0], p0[2], p1[2], p1[1]), (1, p0[0], p1[0], p0[2], p1[2], p0[1]),
                 (2, p0[1], p1[1], p0[2], p1[2], p1[0]), (2, p0[1], p1[1], p0[2], p1[2], p0[0])]
        closest, found = F(np.inf), None
        for sd in sides:  # Cuboid::hit = the six rects as a closest-hit list (rectangular.rs:238-240)
            h = hit_rect(o, d, F(lo), closest, *sd)
            if h is not None:
                closest, found = h[0], h[0]
        return found
    r1 = boundary(-np.inf)
    if r1 is None:
        return None
    r2 = boundary(F(r1 + F(0.0001)))
    if r2 is None:
        return None
    t1 = F(max(r1, F(tmin)))
    if t1 >= r2:
        return None
    t1 = F(max(t1, F(0.0)))
    ln = F(np.sqrt(len2(d)))
    dist = F(F(r2 - t1) * ln)
    u = Xoro64(xoro_seed(splitmix64(seg ^ splitmix64(key)))).next_u32()
    hd = F(neg_inv * log10f(F(u >> 8) * F(1.0 / 16777216.0)))
    if hd > dist:
        return None
    t = F(t1 + F(hd / ln))
    return None if t > tmax else t


def main():
    rng = np.random.default_rng(20240807)
    g = {}
    # RNG
    g["pcg_state"] = np.array([0x853C49E6748FEA9B, 12345, 2 ** 63 + 7], np.uint64)
    g["pcg_out"] = np.array([[Pcg32(int(s)).next_u32() for _ in range(1)] for s in g["pcg_state"]], np.uint32)
    streams = []
    for s in g["pcg_state"]:
        p = Pcg32(int(s))
        streams.append([p.next_u32() for _ in range(8)])
    g["pcg_stream"] = np.array(streams, np.uint32)
    g["xoro_state"] = np.array([0x853C49E6748FEA9B, 1, 2 ** 63 + 7, 0xFFFFFFFF00000000], np.uint64)
    xs = []
    for st in g["xoro_state"]:
        x = Xoro64(int(st))
        xs.append([x.next_u32() for _ in range(8)])
    g["xoro_stream"] = np.array(xs, np.uint32)
    keys = np.array([[0, 0, 0, 0], [7, 3, 5, 1], [2024, 1079, 1919, 511], [2 ** 40 + 3, 17, 9, 100]], np.uint64)
    g["path_keys"] = keys
    g["path_state"] = np.array([path_state(int(a), int(b), int(c), int(d)) for a, b, c, d in keys], np.uint64)
    u = rng.integers(0, 2 ** 32, 64, dtype=np.uint64).astype(np.uint32)
    u[:4] = [0, 0xFFFFFFFF, 0x80000000, 0x000001FF]
    g["u32"] = u
    g["u32_f32"] = np.array([Draws([x]).gen_f32() for x in u], np.float32)
    g["u32_m11"] = np.array([Draws([x]).gen_range(-1, 1) for x in u], np.float32)
    g["u32_05"] = np.array([Draws([x]).gen_range(0.0, 0.5) for x in u], np.float32)
    # sphere uv KAT table (spherical.rs:66-68) + random points
    pts = np.array([[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]], np.float32)
    g["uv_pts"] = pts
    g["uv_out"] = np.array([sphere_uv(p) for p in pts], np.float32)
    # primitive hits over random rays
    rays = []
    for _ in range(256):
        o = rng.uniform(-3, 3, 3).astype(np.float32)
        tgt = rng.uniform(-1, 1, 3).astype(np.float32)
        d = (tgt - o + rng.normal(0, 0.3, 3)).astype(np.float32)
        rays.append(np.concatenate([o, d, [rng.uniform(0, 1)]]).astype(np.float32))
    rays = np.array(rays, np.float32)
    g["rays"] = rays
    prims = {
        "sphere": (0, np.array([0.1, -0.2, 0.3, 1.1], np.float32)),
        "hollow": (0, np.array([0.0, 0.0, 0.0, -0.95], np.float32)),
        "msphere": (1, np.array([0.0, 0.2, 0.1, 0.0, 0.3, 0.7, 0.1, 1.0, 0.6], np.float32)),
        "rect_xy": (2, np.array([0, -1, 1, -0.5, 0.8, 0.25], np.float32)),
        "rect_xz": (2, np.array([1, -1, 1, -0.5, 0.8, -0.1], np.float32)),
        "rect_yz": (2, np.array([2, -1, 1, -0.5, 0.8, 0.4], np.float32)),
        "tri": (3, np.array([-1, -1, 0.2, 1, -0.8, 0.1, 0.1, 1.2, -0.3], np.float32)),
    }
    for name, (kind, par) in prims.items():
        out = np.full((len(rays), 11), np.nan, np.float32)
        for q, r in enumerate(rays):
            o, d, time = r[:3], r[3:6], r[6]
            if kind == 0:
                hit = hit_sphere(o, d, F(0.001), F(np.inf), par[:3], par[3])
            elif kind == 1:
                c = center_at(par[:3], par[3], par[4:7], par[7], time)
                hit = hit_sphere(o, d, F(0.001), F(np.inf), c, par[8])
            elif kind == 2:
                hit = hit_rect(o, d, F(0.001), F(np.inf), int(par[0]), *par[1:6])
            else:
                hit = hit_tri(o, d, F(0.001), F(np.inf), (par[:3], par[3:6], par[6:9]))
            if hit is not None:
                t, p, n, uu, vv, front = hit
                out[q] = [1, t, *p, *n, uu, vv, float(front)]
            else:
                out[q, 0] = 0
        g[f"prim_{name}_kind"] = np.array([kind])
        g[f"prim_{name}_par"] = par
        g[f"prim_{name}_out"] = out
    # aabb
    boxes = rng.uniform(-1, 1, (256, 6)).astype(np.float32)
    boxes[:, 3:] = np.maximum(boxes[:, :3], boxes[:, 3:]) + 0.05
    boxes[:, :3] = np.minimum(boxes[:, :3], boxes[:, 3:] - 0.1)
    rays_ax = rays.copy()
    rays_ax[::7, 3] = 0.0  # parallel to a slab: inf / NaN handling (Rust max/min ignore NaN)
    g["aabb_boxes"] = boxes
    g["aabb_rays"] = rays_ax
    g["aabb_out"] = np.array([aabb_hit(b[:3], b[3:], r[:3], r[3:6], 0.001, np.inf) for b, r in zip(boxes, rays_ax)])
    # scatter with fixed draws
    sc_in = []
    sc_out = []
    sc_draws = []
    for q in range(96):
        kind = q % 3
        d_in = rng.normal(0, 1, 3).astype(np.float32)
        n = unit(rng.normal(0, 1, 3).astype(np.float32))
        if dot(d_in, n) > 0:
            n = -n
        front = bool(q % 2)
        p = rng.uniform(-1, 1, 3).astype(np.float32)
        params = np.array([*rng.uniform(0, 1, 3), [0.0, 0.3, 1.0][q % 3] if kind == 1 else 1.5], np.float32)
        draws = rng.integers(0, 2 ** 32, 24, dtype=np.uint64).astype(np.uint32)
        dr = Draws(draws)
        ok, dirn, att = scatter(kind, params, d_in, p, n, front, dr)
        sc_in.append(np.concatenate([[kind, front], params, d_in, p, n]))
        sc_draws.append(draws)
        sc_out.append(np.concatenate([[ok, dr.used], dirn, att]))
    g["scatter_in"] = np.array(sc_in, np.float32)
    g["scatter_out"] = np.array(sc_out, np.float32)
    g["scatter_draws"] = np.array(sc_draws, np.uint32)
    # camera + get_ray
    cams = [((13, 2, 3), (0, 0, 0), (0, 1, 0), 20.0, 16 / 9, 0.1, 10.0),
            ((278, 278, -800), (278, 278, 0), (0, 1, 0), 40.0, 1.0, 0.0, 10.0),
            ((-5, -30, 25), (0, 0, 5), (1, 0, 0), 40.0, 16 / 9, 0.0, 10.0)]
    cam_f, gr, gr_draws = [], [], []
    for ci, cargs in enumerate(cams):
        c = camera_new(*cargs)
        cam_f.append(np.concatenate([c[k] for k in ("origin", "lower_left_corner", "horizontal", "vertical", "u",
                                                     "v", "w")] + [[c["lens_radius"], c["time0"], c["time1"]]]))
        for q in range(16):
            s_, t_ = F(rng.uniform()), F(rng.uniform())
            draws = rng.integers(0, 2 ** 32, 12, dtype=np.uint64).astype(np.uint32)
            dr = Draws(draws)
            o, d, time = get_ray(c, s_, t_, dr)
            gr.append(np.concatenate([[ci, s_, t_], o, d, [time, dr.used]]))
            gr_draws.append(draws)
    g["cam_args"] = np.array([[*a[0], *a[1], *a[2], a[3], a[4], a[5], a[6]] for a in cams], np.float32)
    g["cam_fields"] = np.array(cam_f, np.float32)
    g["get_ray"] = np.array(gr, np.float32)
    g["get_ray_draws"] = np.array(gr_draws, np.uint32)
    # tonemap
    sums = np.concatenate([rng.uniform(0, 80, 60), [0, -1, np.inf, np.nan, 1e-30, 50.0, 49.9]]).astype(np.float32)
    g["tm_sum"] = sums
    g["tm_out"] = np.array([tonemap(x, 50) for x in sums], np.uint8)
    # a whole image: jumpy-balls 16x9x2 spp (scene seed 5, render seed 9)
    img, nrays, _ = render_jumpy(16, 9, 2, 5, 9, 16 / 9)
    g["jumpy_img"] = img
    g["jumpy_rays"] = np.array([nrays])
    sph, mats = jumpy_balls(5)
    g["jumpy_spheres"] = np.array([[*s[0], s[1], *s[2], s[3], s[4], s[5], s[6]] for s in sph], np.float32)
    # Perlin noise / turbulence over random tables (perlin.rs:50-122) and Perlin::new (perlin.rs:14-48)
    pg = np.array([unit(x) for x in rng.normal(0, 1, (256, 3)).astype(np.float32)], np.float32)
    pp = np.stack([rng.permutation(256) for _ in range(3)]).astype(np.uint32)
    pts = rng.uniform(-20, 20, (96, 3)).astype(np.float32)
    pts[:8] = np.floor(pts[:8])  # lattice points
    pts[8:16] *= np.float32(40.0)  # beyond one period of the 256-wide lattice
    g["perlin_grad"], g["perlin_perm"], g["perlin_pts"] = pg, pp, pts
    g["perlin_noise"] = np.array([perlin_noise(pg, pp, p) for p in pts], np.float32)
    g["perlin_turb"] = np.array([turbulence(pg, pp, p, 7) for p in pts], np.float32)
    g["noise_value"] = np.array([F(F(0.5) * F(F(1.0) + sinf_cr(F(F(F(4.0) * p[2]) + F(F(10.0) * t)))))
                                 for p, t in zip(pts, g["perlin_turb"])], np.float32)
    ng, npm = perlin_new(Draws(scene_rng(7)))
    g["perlin_new_grad"], g["perlin_new_perm"] = ng, npm
    # ConstantMedium hits (sphere and cuboid boundaries)
    med_in, med_out = [], []
    for q in range(160):
        kind = q % 2
        par = (np.array([0.2, -0.1, 0.3, 1.3, 0, 0], np.float32) if kind == 0
               else np.array([-1.0, -0.7, -1.2, 0.9, 1.1, 0.8], np.float32))
        dens = [0.05, 0.5, 5.0, 50.0][q % 4]
        o = rng.uniform(-3, 3, 3).astype(np.float32)
        if q % 5 == 0:
            o = rng.uniform(-0.5, 0.5, 3).astype(np.float32)  # starting inside
        d = (rng.uniform(-0.5, 0.5, 3) - o).astype(np.float32)
        seg = int(rng.integers(0, 2 ** 63))
        key = int(rng.integers(0, 4000))
        t = medium_hit(kind, par, o, d, 0.001, np.inf, dens, seg, key)
        med_in.append([kind, dens, *par, *o, *d, 0.5, seg & 0xFFFFFFFF, seg >> 32, key])
        med_out.append([0.0, 0.0] if t is None else [1.0, t])
    g["medium_in"] = np.array(med_in, np.float64)
    g["medium_out"] = np.array(med_out, np.float32)
    out = Path(__file__).resolve().parent / "golden.npz"
    np.savez_compressed(out, **g)
    print("wrote", out, "keys", len(g), "jumpy rays", nrays)


if __name__ == "__main__":
    main()

"""Far-origin sphere hits (round 6).

The reference's f32 sphere test (spherical.rs:26-44) cancels in hb² - a·c: a ray whose origin is D away from a
sphere "hits" it up to ~sqrt(3u)·D outside its surface, and the flat list (hittable/mod.rs:57-69) finds every such
hit.  The GPU's BVH pads its sphere leaves for origins within D0 of the BVH and sends farther rays through the
far-origin walk (rtw_kernel.hip trace_begin / trace_far).  These tests put the origin where the bound matters:
inside the r = 1000 ground sphere, under a field of small balls, bit for bit against the oracle with equal ray
counts; and the three random worlds of round 5's 3,000-seed run at 64x36x4 that the padded boxes alone missed."""
import numpy as np
import pytest

from test_gpu_fuzz import _random_world

pytestmark = pytest.mark.gpu


def _ball_field(rtw, s, rng, n=14, moving=True, rotated=False):
    """jumpy-balls' shape in miniature: a checkered r = 1000 ground (always-tested) and an n x n grid of 0.2 balls
    (a BVH), some moving, optionally inside a YRotation + Translation."""
    ground = s.lambertian(s.checker(s.solid_rgb(0.2, 0.3, 0.1), s.solid_rgb(0.9, 0.9, 0.9), 10.0))
    s.sphere((0, -1000, 0), 1000, ground)
    mats = [s.lambertian_solid(tuple(rng.uniform(0.1, 0.9, 3))) for _ in range(3)]
    mats += [s.metal(tuple(rng.uniform(0.5, 1.0, 3)), 0.2), s.dielectric(1.5)]
    xs = np.arange(n, dtype=np.float32) - n / 2
    c = np.array([(a + 0.9 * rng.uniform(), 0.2, b + 0.9 * rng.uniform()) for a in xs for b in xs], np.float32)
    m = [int(rng.choice(mats)) for _ in range(len(c))]

    def add():
        k = len(c) // 2 if moving else len(c)
        s.spheres(c[:k], np.full(k, 0.2, np.float32), m[:k])
        if moving:
            c1 = c[k:] + np.array([0, 0.25, 0], np.float32) * rng.uniform(0, 1, (len(c) - k, 1)).astype(np.float32)
            s.moving_spheres(c[k:], np.zeros(len(c) - k), c1, np.ones(len(c) - k), np.full(len(c) - k, 0.2), m[k:])
    if rotated:
        with s.translate((0.3, 0.0, -0.2)):
            with s.rotate_y(17.0):
                add()
    else:
        add()


@pytest.mark.parametrize("variant", ["static", "moving", "rotated"])
def test_far_origin_camera_bit_exact(gpu, orc, variant):
    """A camera inside the ground sphere, ~1,200 units below the ball field, looking up through it: every camera
    ray is a far-origin ray that reaches the field's grown box, and the ones that graze a ball within the sphere
    test's cancellation band hit it in the reference's list.  GPU == oracle bit for bit, equal ray counts."""
    rtw = gpu
    rng = np.random.default_rng({"static": 1, "moving": 2, "rotated": 3}[variant])
    s = rtw.Scene()
    _ball_field(rtw, s, rng, moving=variant != "static", rotated=variant == "rotated")
    text, imgs = s.dump(), s.images()
    s.commit()
    assert s.info(14) == 1 and s.info(3) > 0  # a BVH with sphere tests: the far-origin bound is on
    cam = rtw.Camera.new((0.35, -1200.0, 0.15), (0.0, 0.2, 0.0), (1, 0, 0), 0.8, 1.0, 0.0, 1200.0)
    w = h = 48
    g, st = rtw.Raytracer(s, cam, (0.7, 0.8, 1.0), w, h, 2, seed=11).render()
    r, rays = orc.OracleScene(text, imgs).render(orc.camera_from_fields(cam.as_dict()), (0.7, 0.8, 1.0), w, h, 2,
                                                seed=11)
    assert st["rays"] == rays, f"ray count {st['rays']} vs oracle {rays}"
    bad = np.argwhere((g.view(np.uint32) != r.view(np.uint32)).any(axis=2))
    assert bad.size == 0, f"{len(bad)} mismatching pixels, first {bad[:4].tolist()}"


@pytest.mark.parametrize("seed", [863, 1981, 2503])
def test_far_origin_fuzz_regressions(gpu, orc, seed):
    """The random worlds whose 64x36x4 frames differed in round 5 (profiles/r05/r05fin_fuzz3000x4.log), each by one
    path bouncing inside the r = 1000 ground with a spurious small-sphere hit 1.9-2.8 r from its centre."""
    _random_world(gpu, orc, seed, 64, 36, 4)

"""Scene presets (console_app/src/scenes.rs restated in C++) vs an independent Python
restatement (tests/golden/make_golden.py) and the reference's literal constants."""
import importlib.util
from pathlib import Path

import numpy as np
import pytest

spec = importlib.util.spec_from_file_location("make_golden", Path(__file__).parent / "golden" / "make_golden.py")
mg = importlib.util.module_from_spec(spec)
spec.loader.exec_module(mg)


def parse_dump(text):
    mats, prims, tex = [], [], []
    for line in text.splitlines():
        t = line.split()
        if not t:
            continue
        if t[0] == "mat":
            mats.append(t[2:])
        elif t[0] == "tex":
            tex.append(t[2:])
        elif t[0] in ("sphere", "msphere", "rect", "cuboid", "tri", "begin", "end"):
            prims.append(t)
    return tex, mats, prims


def f(x):
    return np.float32(float.fromhex(x) if "0x" in x else float(x))


@pytest.mark.parametrize("seed", [0, 5, 42])
def test_jumpy_balls_layout(rtw, seed):
    """scenes.rs:63-162 with the seeded draws: sphere list, order and materials."""
    s = rtw.Scene()
    cam, bg = s.preset("jumpy-balls", 16 / 9, seed=seed)
    tex, mats, prims = parse_dump(s.dump())
    want, wmats = mg.jumpy_balls(seed)
    assert len(prims) == len(want)
    for p, w in zip(prims, want):
        c0, t0, c1, t1, r, mi, moving = w
        if moving:
            assert p[0] == "msphere"
            vals = [f(x) for x in p[1:10]]
            assert np.array_equal(np.array(vals, np.float32), np.array([*c0, t0, *c1, t1, r], np.float32))
        else:
            assert p[0] == "sphere"
            assert np.array_equal(np.array([f(x) for x in p[1:5]], np.float32), np.array([*c0, r], np.float32))
        m = mats[int(p[-1])]
        wm = wmats[mi]
        if wm[0] == "checker":
            assert m[0] == "lambertian" and tex[int(m[1])][0] == "checker"
        elif wm[0] == 0:
            assert m[0] == "lambertian"
            assert np.array_equal(np.array([f(x) for x in tex[int(m[1])][1:4]], np.float32),
                                  np.array(wm[1], np.float32))
        elif wm[0] == 1:
            assert m[0] == "metal"
            assert np.array_equal(np.array([f(x) for x in m[1:5]], np.float32), np.array([*wm[1], wm[2]], np.float32))
        else:
            assert m[0] == "dielectric" and f(m[1]) == np.float32(1.5)
    assert bg == pytest.approx((0.7, 0.8, 1.0))
    n_moving = sum(1 for w in want if w[6])
    assert 470 <= n_moving <= 484  # 22x22 grid minus the cells near (4, 0.2, 0) (scenes.rs:109)


def test_cornell_box_structure(rtw):
    """scenes.rs:350-414: 6 world rects, then Translation(YRotation(Cuboid)) x2."""
    s = rtw.Scene()
    cam, bg = s.preset("cornell-box", 1.0)
    tex, mats, prims = parse_dump(s.dump())
    kinds = [p[0] + (p[1] if p[0] in ("rect", "begin") else "") for p in prims]
    assert kinds == ["rectyz", "rectyz", "rectxz", "rectxz", "rectxz", "rectxy",
                     "begintranslate", "beginrotate_y", "cuboid", "end", "end",
                     "begintranslate", "beginrotate_y", "cuboid", "end", "end"]
    light = mats[int(prims[2][-1])]
    assert light[0] == "light" and [f(x) for x in tex[int(light[1])][1:4]] == [15, 15, 15]
    assert f(prims[7][2]) == 15 and f(prims[12][2]) == -18
    assert bg == (0.0, 0.0, 0.0)
    assert cam.as_dict()["lens_radius"] == 0.0


def test_cow_and_monument(rtw):
    s = rtw.Scene()
    s.preset("wavefront-cow-obj", 16 / 9)
    tex, mats, prims = parse_dump(s.dump())
    tris = [p for p in prims if p[0] == "tri"]
    assert len(tris) == 5804
    m = mats[int(tris[0][-1])]
    assert m[0] == "light" and [f(x) for x in tex[int(m[1])][1:4]] == [1, 0, 1]  # triangular.rs:177-182
    assert [p[0] for p in prims[:4]] == ["sphere", "rect", "begin", "begin"]  # translate(bvh(tris))
    s2 = rtw.Scene()
    s2.preset("textured-monument", 16 / 9)
    tex, mats, prims = parse_dump(s2.dump())
    tris = [p for p in prims if p[0] == "tri"]
    assert len(tris) == 7798
    m = mats[int(tris[0][-1])]
    assert m[0] == "lambertian" and tex[int(m[1])][:3] == ["image", "2048", "2048"]
    img = s2.images()[0].reshape(2048, 2048, 3)
    assert img[0, 0].tolist() == [176 - 32, 176, 176 - 32] or img[0, 0, 1] in (96, 176)
    assert all(int(t[-8]) == 7 for t in tris[:50])  # uv mask: every vertex has vt

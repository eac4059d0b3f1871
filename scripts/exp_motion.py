"""Experiment: how much of the jumpy-balls trace cost is the moving spheres' motion-swept boxes?

Renders a jumpy-balls-like world (scenes.rs:96-135 layout, numpy-seeded, not the preset's stream) with the
balls' vertical travel scaled by m in {1, 0.5, 0.25, 0}: m = 0.5 has the boxes a 2-way time-split tree would
give each half of the shutter.  Prints Mrays/s and traversal counts per m (1920x1080, --spp samples).
Usage: python scripts/exp_motion.py [--spp 64]
"""
import argparse
import importlib.util
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
PKG = ROOT / "raytracer-weekend_amd"


def load():
    spec = importlib.util.spec_from_file_location("rtw_amd", PKG / "__init__.py",
                                                  submodule_search_locations=[str(PKG)])
    m = importlib.util.module_from_spec(spec)
    sys.modules["rtw_amd"] = m
    spec.loader.exec_module(m)
    return m


def world(rtw, m_scale, seed=7):
    rng = np.random.default_rng(seed)
    s = rtw.Scene()
    g = s.checker(s.solid_rgb(0.2, 0.3, 0.1), s.solid_rgb(0.9, 0.9, 0.9), 10.0)
    s.sphere((0, -1000, 0), 1000, s.lambertian(g))
    s.sphere((-4, 1, 0), 1.0, s.lambertian_solid((0.4, 0.2, 0.1)))
    glass = s.dielectric(1.5)
    s.sphere((0, 1, 0), 1.0, glass)
    s.sphere((4, 1, 0), 1.0, s.metal((0.7, 0.6, 0.5), 0.0))
    c0, c1, mats = [], [], []
    for a in range(-11, 11):
        for b in range(-11, 11):
            c = np.array([a + 0.9 * rng.random(), 0.2, b + 0.9 * rng.random()], np.float32)
            if np.linalg.norm(c - np.array([4, 0.2, 0], np.float32)) <= 0.9:
                continue
            u = rng.random()
            if u < 0.8:
                mat = s.lambertian_solid(tuple(rng.random(3) * rng.random(3)))
            elif u < 0.95:
                mat = s.metal(tuple(0.5 + 0.5 * rng.random(3)), 0.5 * rng.random())
            else:
                mat = glass
            d = 0.5 * rng.random()
            c0.append(c)
            c1.append(c + np.array([0, m_scale * d, 0], np.float32))
            mats.append(mat)
    n = len(mats)
    s.moving_spheres(c0, np.zeros(n), c1, np.ones(n), np.full(n, 0.2), mats)
    return s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--frames", type=int, default=3)
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    rtw = load()
    w, h = 1920, 1080
    out = torch.zeros((h, w, 3), dtype=torch.float32, device=0)
    stream = torch.cuda.current_stream()
    for m_scale in (1.0, 0.5, 0.25, 0.0):
        s = world(rtw, m_scale)
        cam = rtw.Camera.new((13, 2, 3), (0, 0, 0), (0, 1, 0), 20.0, rtw.camera_aspect(w, h), 0.1, 10.0)
        s.commit(device=0)
        rt = rtw.Raytracer(s, cam, (0.7, 0.8, 1.0), w, h, args.spp, seed=1)
        st = rt.render_device(out.data_ptr(), 0, 0, 0, stream.cuda_stream, flags=rtw.FLAG_COUNT_TRAVERSAL,
                              want_stats=True)
        rays = st["rays"]
        for _ in range(args.frames + 1):
            rt.render_device(out.data_ptr(), 0, 0, 0, stream.cuda_stream)
        torch.cuda.synchronize()
        ms = s.path_kernel_times(0)[-args.frames:]
        kms = float(np.mean(ms))
        print(json.dumps({"motion_scale": m_scale, "nodes": len(s.nodes()), "kernel_ms": round(kms, 3),
                          "Mrays_s": round(rays / kms / 1e3, 1), "node4_per_ray": round(st["node_visits"] / rays, 3),
                          "boxes_per_ray": round(st["boxes_tested"] / rays, 3),
                          "prims_per_ray": [round(x / rays, 3) for x in st["prim_tests_by_type"][:2]]}), flush=True)
        del rt, s


if __name__ == "__main__":
    main()

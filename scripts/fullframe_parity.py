"""Whole-frame GPU vs oracle comparison at reduced spp (counts mismatching pixels): a bound on how often the BVH's
culling and the reference's flat list disagree on the benchmark frames themselves.
   usage: python scripts/fullframe_parity.py <preset> <w> <h> <spp> [threads]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import importlib

rtw = importlib.import_module("raytracer-weekend_amd")
import oracle as orc  # noqa: E402

name, w, h, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
threads = int(sys.argv[5]) if len(sys.argv) > 5 else 16
s = rtw.Scene()
cam, bg = s.preset(name, w / h, seed=42)  # bench.py's scene seed
text, imgs = s.dump(), s.images()
s.commit()
g, st = rtw.Raytracer(s, cam, bg, w, h, spp, seed=2024).render()  # bench.py's render seed
t0 = time.time()
r, rays = orc.OracleScene(text, imgs).render(orc.camera_from_fields(cam.as_dict()), bg, w, h, spp, seed=2024,
                                            threads=threads)
bad = np.argwhere((g.view(np.uint32) != r.view(np.uint32)).any(axis=2))
out = {"scene": name, "w": w, "h": h, "spp": spp, "gpu_rays": int(st["rays"]), "oracle_rays": int(rays),
       "mismatching_pixels": int(len(bad)), "first": bad[:10].tolist(), "oracle_s": round(time.time() - t0, 1)}
if len(bad):
    d = np.abs(g / spp - r / spp)
    out["max_abs_diff_mean"] = float(d.max())
    out["rmse"] = float(np.sqrt(np.mean((g / spp - r / spp) ** 2)))
print(json.dumps(out), flush=True)

"""Diagnose one fuzz seed (tests/test_gpu_fuzz.py): differing pixels, the first differing sample, the scene text."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import importlib

rtw = importlib.import_module("raytracer-weekend_amd")
import oracle as orc  # noqa: E402
import test_gpu_fuzz as T  # noqa: E402

seed = int(sys.argv[1])
W, H = int(sys.argv[2]), int(sys.argv[3])
out = sys.argv[4]
rng = np.random.default_rng(1000 + seed)
s = rtw.Scene()
T._build(rtw, s, rng)
eye = rng.uniform(-1, 1, 3) * np.array([8, 2, 8]) + np.array([0, 3, 0])
cam = rtw.Camera.new(tuple(eye), tuple(rng.uniform(-1, 1, 3)), (0, 1, 0), float(rng.uniform(30, 70)), W / H,
                     float(rng.choice([0.0, 0.1])), float(np.linalg.norm(eye)))
bg = tuple(rng.uniform(0, 0.8, 3))
text, imgs = s.dump(), s.images()
s.commit()
open(os.path.join(out, f"scene_{seed}.txt"), "w").write(text)
json.dump({"cam": cam.as_dict(), "bg": bg, "w": W, "h": H, "seed": seed,
           "images": [np.asarray(i).tolist() for i in imgs]}, open(os.path.join(out, f"setup_{seed}.json"), "w"))
o = orc.OracleScene(text, imgs)
res = {}
for spp in (1, 2, 3):
    g, st = rtw.Raytracer(s, cam, bg, W, H, spp, seed=seed).render()
    r, rays = o.render(orc.camera_from_fields(cam.as_dict()), bg, W, H, spp, seed=seed)
    bad = np.argwhere((g.view(np.uint32) != r.view(np.uint32)).any(axis=2))
    res[spp] = {"gpu_rays": int(st["rays"]), "oracle_rays": int(rays), "bad_pixels": bad.tolist()[:20]}
    for (y, x) in bad[:5]:
        res[spp].setdefault("values", []).append({"row": int(y), "col": int(x), "gpu": g[y, x].tolist(), "oracle": r[y, x].tolist()})
print(json.dumps(res, indent=1))
json.dump(res, open(os.path.join(out, f"diag_{seed}.json"), "w"), indent=1)

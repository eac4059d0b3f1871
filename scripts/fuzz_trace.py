"""Render one fuzz seed's frame (tests/test_gpu_fuzz.py) once, for a library built with -DRTW_DIAG_TRACE_PID."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import importlib

rtw = importlib.import_module("raytracer-weekend_amd")
import test_gpu_fuzz as T  # noqa: E402

seed, W, H, spp = (int(x) for x in sys.argv[1:5])
rng = np.random.default_rng(1000 + seed)
s = rtw.Scene()
T._build(rtw, s, rng)
eye = rng.uniform(-1, 1, 3) * np.array([8, 2, 8]) + np.array([0, 3, 0])
cam = rtw.Camera.new(tuple(eye), tuple(rng.uniform(-1, 1, 3)), (0, 1, 0), float(rng.uniform(30, 70)), W / H,
                     float(rng.choice([0.0, 0.1])), float(np.linalg.norm(eye)))
bg = tuple(rng.uniform(0, 0.8, 3))
s.commit()
g, st = rtw.Raytracer(s, cam, bg, W, H, spp, seed=seed).render()
print("rays", st["rays"], "pixel", g[int(sys.argv[5]), int(sys.argv[6])].tolist(), flush=True)

"""Find the first path whose segments differ between the GPU and the oracle on one fuzz seed (debugging aid).
   on the GPU box (RTW_LIB_PATH = a -DRTW_DIAG_TRACE_PID=-1 build):
       python scripts/fuzz_compare.py gpu <seed> <w> <h> <spp> > trace.txt
   here:
       python scripts/fuzz_compare.py compare <seed> <w> <h> <spp> trace.txt"""
import collections
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import importlib

rtw = importlib.import_module("raytracer-weekend_amd")
import test_gpu_fuzz as T  # noqa: E402

mode, seed, W, H, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])


def world():
    rng = np.random.default_rng(1000 + seed)
    s = rtw.Scene()
    T._build(rtw, s, rng)
    eye = rng.uniform(-1, 1, 3) * np.array([8, 2, 8]) + np.array([0, 3, 0])
    cam = rtw.Camera.new(tuple(eye), tuple(rng.uniform(-1, 1, 3)), (0, 1, 0), float(rng.uniform(30, 70)), W / H,
                         float(rng.choice([0.0, 0.1])), float(np.linalg.norm(eye)))
    return s, cam, tuple(rng.uniform(0, 0.8, 3))


s, cam, bg = world()
if mode == "gpu":
    s.commit()
    rtw.Raytracer(s, cam, bg, W, H, spp, seed=seed).render()
    sys.exit(0)
if mode == "oracle1":  # child: one path's oracle trace (ORACLE_TRACE in the environment) to stderr
    import oracle as orc
    j = int(os.environ["ORACLE_TRACE"].split(",")[0])
    orc.OracleScene(s.dump(), s.images()).render(orc.camera_from_fields(cam.as_dict()), bg, W, H, spp, seed=seed,
                                                 rows=[j], threads=1)
    sys.exit(0)
import oracle as orc  # noqa: E402
tx = (W + 7) // 8
gpu = collections.defaultdict(list)
for l in open(sys.argv[6]):
    t = l.split()
    if not t or t[0] != "rtwtrace":
        continue
    pid = int(t[2])
    hi, lane = pid >> 6, pid & 63
    slot, smp = divmod(hi, spp)
    ty, tcol = divmod(slot, tx)
    gpu[(ty * 8 + (lane >> 3), tcol * 8 + (lane & 7), smp)].append(l.rstrip())
_, rays, pr = orc.OracleScene(s.dump(), s.images()).render(orc.camera_from_fields(cam.as_dict()), bg, W, H, spp,
                                                           seed=seed, pixel_rays=True)
print("rays: gpu", sum(len(v) for v in gpu.values()), "oracle", rays)
for row in range(H):
    for col in range(W):
        g = sum(len(gpu.get((row, col, k), [])) for k in range(spp))
        if g == int(pr[row, col]):
            continue
        print(f"pixel row {row} col {col}: gpu {g} oracle {int(pr[row, col])}")
        j = H - 1 - row
        for k in range(spp):
            p = subprocess.run([sys.executable, __file__, "oracle1", str(seed), str(W), str(H), str(spp)],
                               env=dict(os.environ, ORACLE_TRACE=f"{j},{col},{k}"), capture_output=True, text=True)
            ol = [x for x in p.stderr.splitlines() if x.startswith("depth")]
            gl = gpu.get((row, col, k), [])
            if len(ol) != len(gl):
                print(f" sample {k}: oracle {len(ol)} segments, gpu {len(gl)}")
                for q in range(max(len(ol), len(gl))):
                    print("  O", ol[q][:330] if q < len(ol) else "-")
                    print("  G", gl[q][:330] if q < len(gl) else "-")
                sys.exit(0)

"""Locate paths whose segment counts differ between the GPU and the oracle on a preset frame (debugging aid):
per tile row, then per tile, then the first sample index, from ray counts (GPU stats per render, oracle per pixel).
   usage: python scripts/count_bisect.py <preset> <w> <h> <spp>"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import importlib

import torch

rtw = importlib.import_module("raytracer-weekend_amd")
import oracle as orc  # noqa: E402

name, w, h, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
s = rtw.Scene()
cam, bg = s.preset(name, w / h, seed=42)
text, imgs = s.dump(), s.images()
s.commit()
o = orc.OracleScene(text, imgs)
ocam = orc.camera_from_fields(cam.as_dict())
rt = rtw.Raytracer(s, cam, bg, w, h, spp, seed=2024)
tx, ty = (w + 7) // 8, (h + 7) // 8
dev = torch.device("cuda:0")
stream = torch.cuda.current_stream().cuda_stream


def gpu_rays(tiles, rt_=rt):
    ids = torch.tensor(tiles, dtype=torch.int32, device=dev)
    packed = torch.zeros((len(tiles), 64, 3), dtype=torch.float32, device=dev)
    st = rt_.render_device(packed.data_ptr(), 0, ids.data_ptr(), len(tiles), stream, want_stats=True)
    torch.cuda.synchronize()
    return int(st["rays"])


_, _, pr = o.render(ocam, bg, w, h, spp, seed=2024, pixel_rays=True)  # pr[row, i] (row 0 = top)
res = {"tile_rows": []}
for r in range(ty):
    g = gpu_rays([r * tx + c for c in range(tx)])
    ref = int(pr[r * 8:(r + 1) * 8].sum())
    if g != ref:
        res["tile_rows"].append((r, g, ref))
print("tile rows", res["tile_rows"], flush=True)
found = []
for r, _, _ in res["tile_rows"][:3]:
    for c in range(tx):
        t = r * tx + c
        g = gpu_rays([t])
        ref = int(pr[r * 8:(r + 1) * 8, c * 8:(c + 1) * 8].sum())
        if g != ref:
            found.append((t, g, ref))
print("tiles", found, flush=True)
for t, _, _ in found[:2]:
    r, c = divmod(t, tx)
    rows = [h - 1 - (r * 8 + k) for k in range(8) if r * 8 + k < h]
    for k in range(1, spp + 1):
        rtk = rtw.Raytracer(s, cam, bg, w, h, k, seed=2024)
        g = gpu_rays([t], rtk)
        _, _, pk = o.render(ocam, bg, w, h, k, seed=2024, rows=rows, pixel_rays=True)
        ref = int(pk[r * 8:(r + 1) * 8, c * 8:(c + 1) * 8].sum())
        if g != ref:
            _, _, pk1 = o.render(ocam, bg, w, h, k - 1, seed=2024, rows=rows, pixel_rays=True) if k > 1 else (0, 0, np.zeros_like(pk))
            per = (pk - pk1)[r * 8:(r + 1) * 8, c * 8:(c + 1) * 8]
            print(json.dumps({"tile": t, "sample": k - 1, "gpu_rays_k": g, "oracle_rays_k": ref,
                              "oracle_sample_segments": per.tolist()}), flush=True)
            break

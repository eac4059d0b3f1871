"""One rank's share of an N-GPU frame, rendered on this one GPU: the projected strong-scaling efficiency.

bench.py --gpus N gives rank r the tiles r, r + N, r + 2N, ... (rtw_render_device_strided); their path-kernel time on
one GPU, against the whole frame's / N, is the efficiency the N-GPU run can reach before its all-gather.

    python scripts/r06/share8.py [--n 8] [--configs jumpy-1080p,cornell-800,cow-1080p,monument-4k]
"""
import argparse
import importlib
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from bench import CONFIGS, RENDER_SEED, SCENE_SEED  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--configs", default="jumpy-1080p,cornell-800,cow-1080p,monument-4k")
    a = ap.parse_args()
    import torch
    rtw = importlib.import_module("raytracer-weekend_amd")
    for cfg in a.configs.split(","):
        name, w, h, spp, _ = CONFIGS[cfg]
        s = rtw.Scene()
        cam, bg = s.preset(name, rtw.camera_aspect(w, h), seed=SCENE_SEED)
        s.commit(device=0)
        rt = rtw.Raytracer(s, cam, bg, w, h, spp, seed=RENDER_SEED)
        nt = rtw.n_tiles(w, h)
        stream = torch.cuda.current_stream().cuda_stream

        def run(ids):
            d_ids = torch.tensor(ids, dtype=torch.int32, device="cuda:0")
            packed = torch.zeros((len(ids), 64, 3), dtype=torch.float32, device="cuda:0")
            rt.render_device(packed.data_ptr(), 0, d_ids.data_ptr(), len(ids), stream)  # warm-up
            torch.cuda.synchronize()
            s.path_kernel_times(0)
            t0 = time.time()
            for _ in range(a.steps):
                rt.render_device(packed.data_ptr(), 0, d_ids.data_ptr(), len(ids), stream)
            torch.cuda.synchronize()
            wall = (time.time() - t0) / a.steps * 1e3
            return sum(s.path_kernel_times(0)) / a.steps, wall

        full_k, full_w = run(list(range(nt)))
        share_k, share_w = run(list(range(0, nt, a.n)))
        print(json.dumps({"config": cfg, "n": a.n, "tiles": nt, "full_kernel_ms": round(full_k, 3),
                          "share_kernel_ms": round(share_k, 3), "full_step_ms": round(full_w, 3),
                          "share_step_ms": round(share_w, 3),
                          "projected_efficiency_kernel": round(full_k / (a.n * share_k), 4),
                          "projected_efficiency_step": round(full_w / (a.n * share_w), 4)}), flush=True)


if __name__ == "__main__":
    main()

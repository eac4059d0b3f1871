"""Trace every path of one tile-sample on the GPU and in the oracle, and print the first pixel whose segment
sequences differ (debugging aid).
   on the GPU box (a library built with -DRTW_DIAG_TRACE_PID=-1 via RTW_LIB_PATH; device printf to stdout):
       python scripts/tile_trace.py gpu <preset> <w> <h> <tile> <sample>  > trace.txt
   here (the oracle, ORACLE_TRACE):
       python scripts/tile_trace.py compare <preset> <w> <h> <tile> <sample> trace.txt"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import importlib

mode, name, w, h, tile, sample = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), \
    int(sys.argv[6])
rtw = importlib.import_module("raytracer-weekend_amd")
if mode == "gpu":
    import torch
    s = rtw.Scene()
    cam, bg = s.preset(name, w / h, seed=42)
    s.commit()
    rt = rtw.Raytracer(s, cam, bg, w, h, sample + 1, seed=2024)
    ids = torch.tensor([tile], dtype=torch.int32, device="cuda:0")
    packed = torch.zeros((1, 64, 3), dtype=torch.float32, device="cuda:0")
    rt.render_device(packed.data_ptr(), 0, ids.data_ptr(), 1, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    sys.exit(0)
gpu = {}
for l in open(sys.argv[7]):
    t = l.split()
    if t and t[0] == "rtwtrace" and int(t[2]) // 64 == sample:
        gpu.setdefault(int(t[2]) % 64, []).append(l.rstrip())
print("gpu segments per lane", [len(gpu.get(k, [])) for k in range(64)], flush=True)
tx = (w + 7) // 8
r, c = divmod(tile, tx)
for lane in range(64):
    row, col = r * 8 + lane // 8, c * 8 + lane % 8
    j = h - 1 - row
    code = ("import sys; sys.path[:0]=[%r,%r]; import importlib; import oracle as orc; "
            "rtw=importlib.import_module('raytracer-weekend_amd'); s=rtw.Scene(); cam,bg=s.preset(%r,%r,seed=42); "
            "o=orc.OracleScene(s.dump(), s.images()); o.render(orc.camera_from_fields(cam.as_dict()), bg, %d, %d, %d, "
            "seed=2024, rows=[%d], threads=1)") % (ROOT, os.path.join(ROOT, "oracle"), name, w / h, w, h, sample + 1, j)
    p = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, ORACLE_TRACE=f"{j},{col},{sample}"),
                       capture_output=True, text=True, timeout=600)
    ol = [l for l in (p.stderr + p.stdout).splitlines() if l.startswith("depth")]
    gl = gpu.get(lane, [])
    if len(ol) != len(gl):
        print(f"lane {lane} pixel row {row} col {col} j {j}: oracle {len(ol)} segments, gpu {len(gl)}")
        for k in range(max(len(ol), len(gl))):
            print("  O", ol[k] if k < len(ol) else "-")
            print("  G", gl[k] if k < len(gl) else "-")
        break
print("done", flush=True)

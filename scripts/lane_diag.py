import importlib.util, sys, os, json
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
import bench
rtw = bench._load("rtw_amd", bench.PKG / "__init__.py", bench.PKG)
import torch
for cfg in sys.argv[1:]:
    name, w, h, spp, _ = bench.CONFIGS[cfg]
    s = rtw.Scene(); cam, bg = s.preset(name, rtw.camera_aspect(w, h), seed=42); s.commit(0)
    rt = rtw.Raytracer(s, cam, bg, w, h, min(spp, 32), seed=2024)
    out = torch.zeros((h, w, 3), dtype=torch.float32, device="cuda:0")
    st = rt.render_device(out.data_ptr(), 0, 0, 0, torch.cuda.current_stream().cuda_stream, flags=rtw.FLAG_COUNT_TRAVERSAL, want_stats=True)
    ps = st["phase_share"]; allv = ps["sample"]
    print(cfg, json.dumps({"descending": ps["node_loop"] / allv, "parked_waiting": ps["leaf_tests"] / allv, "done": ps["path_start"] / allv, "simd": st["simd_util"]}))

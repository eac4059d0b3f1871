"""Share of node-loop iterations (wave level) whose visiting lanes all visit the same node4 (and with
the same direction octant): run on a -DRTW_UNI_DIAG build (scripts/ab_flags.sh uni "-DRTW_UNI_DIAG")
    RTW_LIB_PATH=raytracer-weekend_amd/lib/ab/uni/librtw_amd.so python scripts/uni_diag.py cow-1080p"""
import json
import os
import sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
rtw = bench._load("rtw_amd", bench.PKG / "__init__.py", bench.PKG)
import torch  # noqa: E402
for cfg in sys.argv[1:]:
    name, w, h, spp, _ = bench.CONFIGS[cfg]
    s = rtw.Scene(); cam, bg = s.preset(name, rtw.camera_aspect(w, h), seed=42); s.commit(0)
    rt = rtw.Raytracer(s, cam, bg, w, h, min(spp, 16), seed=2024)
    out = torch.zeros((h, w, 3), dtype=torch.float32, device="cuda:0")
    st = rt.render_device(out.data_ptr(), 0, 0, 0, torch.cuda.current_stream().cuda_stream,
                          flags=rtw.FLAG_COUNT_TRAVERSAL, want_stats=True)
    ps = st["phase_share"]; allv = ps["sample"]
    print(cfg, json.dumps({"uniform_node_and_octant": ps["node_loop"] / allv, "uniform_node": ps["leaf_tests"] / allv,
                           "visiting_lanes_per_iteration": 64 * ps["path_start"] / allv}))

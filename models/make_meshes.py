"""Re-encode the reference's OBJ meshes as .rtwm (this build's binary mesh format).

The GPU box has no copy of /root/reference, so configs 4-5 load these files instead.
Parsing follows triangular.rs:151-218 / the wavefront_obj crate: coordinates parsed as
f64 and cast to f32, 1-based (or negative) indices, fan triangulation of polygons.
tests/test_assets.py checks that the C++ OBJ loader and these files give identical scenes.

    python models/make_meshes.py [/root/reference/models]
"""
import struct
import sys
from pathlib import Path

import numpy as np

MESHES = ["cow-nonormals", "monument_downscaled_polygon_reduced"]


def parse_obj(path: Path):
    V, VT, VN = [], [], []
    tris = []  # (v idx x3, t idx x3, n idx x3) with -1 = absent
    for line in path.read_text().splitlines():
        parts = line.split()
        if not parts or parts[0].startswith("#"):
            continue
        k = parts[0]
        if k == "v":
            V.append([float(x) for x in parts[1:4]])
        elif k == "vt":
            VT.append([float(x) for x in (parts[1:3] + ["0"])[:2]])
        elif k == "vn":
            VN.append([float(x) for x in parts[1:4]])
        elif k == "f":
            poly = []
            for tok in parts[1:]:
                f = tok.split("/")
                idx = []
                for pos, n in enumerate((len(V), len(VT), len(VN))):
                    if pos < len(f) and f[pos]:
                        i = int(f[pos])
                        idx.append(i - 1 if i > 0 else n + i)
                    else:
                        idx.append(-1)
                poly.append(idx)
            for q in range(1, len(poly) - 1):
                tris.append((poly[0], poly[q], poly[q + 1]))
    V = np.array(V, np.float64).astype(np.float32)
    VT = np.array(VT, np.float64).astype(np.float32).reshape(-1, 2)
    VN = np.array(VN, np.float64).astype(np.float32).reshape(-1, 3)
    n = len(tris)
    v = np.zeros((n, 9), np.float32)
    nn = np.zeros((n, 9), np.float32)
    uv = np.zeros((n, 6), np.float32)
    nm = np.zeros(n, np.uint8)
    um = np.zeros(n, np.uint8)
    for t, tri in enumerate(tris):
        for c, (vi, ti, ni) in enumerate(tri):
            v[t, 3 * c:3 * c + 3] = V[vi]
            if ti >= 0:
                uv[t, 2 * c:2 * c + 2] = VT[ti]
                um[t] |= 1 << c
            if ni >= 0:
                nn[t, 3 * c:3 * c + 3] = VN[ni]
                nm[t] |= 1 << c
    return v, nn, nm, uv, um


def write_rtwm(path: Path, v, nn, nm, uv, um):
    n = len(v)
    flags = (1 if nm.any() else 0) | (2 if um.any() else 0)
    with open(path, "wb") as f:
        f.write(b"RTWM" + struct.pack("<III", 1, n, flags))
        f.write(v.astype("<f4").tobytes())
        if flags & 1:
            f.write(nn.astype("<f4").tobytes())
            f.write(nm.tobytes())
        if flags & 2:
            f.write(uv.astype("<f4").tobytes())
            f.write(um.tobytes())


if __name__ == "__main__":
    src = Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/models")
    out = Path(__file__).resolve().parent
    for m in MESHES:
        arrs = parse_obj(src / f"{m}.obj")
        write_rtwm(out / f"{m}.rtwm", *arrs)
        print(m, len(arrs[0]), "triangles")

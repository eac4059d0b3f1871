"""OBJ loader (triangular.rs:151-312 semantics) vs the committed .rtwm meshes."""
from pathlib import Path

import pytest

REF_MODELS = Path("/root/reference/models")
ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.parametrize("stem,ntri", [("cow-nonormals", 5804), ("monument_downscaled_polygon_reduced", 7798)])
def test_rtwm_matches_obj(rtw, stem, ntri):
    b = rtw.Scene()
    m = b.lambertian_solid((0.5, 0.5, 0.5))
    assert b.load_wavefront_obj(ROOT / "models" / f"{stem}.rtwm", material_override=m) == ntri
    if not (REF_MODELS / f"{stem}.obj").exists():
        pytest.skip("reference models not mounted (GPU box)")
    a = rtw.Scene()
    m2 = a.lambertian_solid((0.5, 0.5, 0.5))
    assert a.load_wavefront_obj(REF_MODELS / f"{stem}.obj", material_override=m2) == ntri
    assert a.dump() == b.dump()  # f64 parse -> f32 cast identical, same vertex / uv / normal masks


def test_obj_reference_material_rules(rtw, tmp_path):
    """No usemtl -> DiffuseLight(1,0,1) (triangular.rs:177-182); usemtl without mtllib and an
    MTL texture that cannot be decoded are errors (the reference unwraps / panics)."""
    (tmp_path / "a.obj").write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nv 1 1 0\nf 1 2 3 4\n")
    s = rtw.Scene()
    assert s.load_wavefront_obj(tmp_path / "a.obj") == 2  # quad -> fan of 2 triangles
    text = s.dump()
    assert "mat 0 light 0" in text and "begin bvh" in text
    (tmp_path / "b.obj").write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nusemtl x\nf 1 2 3\n")
    with pytest.raises(rtw.RtwError) as e:
        rtw.Scene().load_wavefront_obj(tmp_path / "b.obj")
    assert e.value.code == rtw.RTW_EIO
    (tmp_path / "c.mtl").write_text("newmtl x\nillum 1\nmap_Kd missing.png\n")
    (tmp_path / "c.obj").write_text("mtllib c.mtl\nv 0 0 0\nv 1 0 0\nv 0 1 0\nvt 0 0\nvt 1 0\nvt 0 1\n"
                                    "usemtl x\nf 1/1 2/2 3/3\n")
    with pytest.raises(rtw.RtwError):
        rtw.Scene().load_wavefront_obj(tmp_path / "c.obj")
    (tmp_path / "d.obj").write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nvn 0 0 1\nf -3//1 -2//1 -1//1\n")
    s = rtw.Scene()
    assert s.load_wavefront_obj(tmp_path / "d.obj") == 1  # negative (relative) indices
    tri = [l for l in s.dump().splitlines() if l.startswith("tri")][0].split()
    assert tri[10] == "7"  # all three vertex normals present


def test_obj_error_leaves_no_open_group(rtw, tmp_path):
    """A material error (missing map_Kd loader, material not in the MTL) is reported by the loader
    and leaves the caller's scene with no open BvhNode group: a later commit fails for its own
    reason (no device here / succeeds on the GPU box), never with "group(s) still open"."""
    (tmp_path / "c.mtl").write_text("newmtl x\nillum 1\nmap_Kd missing.png\n")
    (tmp_path / "c.obj").write_text("mtllib c.mtl\nv 0 0 0\nv 1 0 0\nv 0 1 0\nvt 0 0\nvt 1 0\nvt 0 1\n"
                                    "usemtl x\nf 1/1 2/2 3/3\nusemtl y\nf 1/1 2/2 3/3\n")
    s = rtw.Scene()
    m = s.lambertian_solid((0.5, 0.5, 0.5))
    s.sphere((0, 0, 0), 1, m)
    with pytest.raises(rtw.RtwError) as e:
        s.load_wavefront_obj(tmp_path / "c.obj")
    assert e.value.code == rtw.RTW_EIO
    assert "begin bvh" not in s.dump()
    try:
        s.commit()
    except rtw.RtwError as err:
        assert err.code == rtw.RTW_ENODEV, err

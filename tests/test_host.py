"""Host-side logic and the C-ABI library, on CPU (no compute calls need a GPU here)."""
import ctypes as C
import json
import re
from pathlib import Path

import numpy as np
import pytest

import oracle_bind as O
from raytracingproject_amd import _native as N
from raytracingproject_amd import api, rtweekend, scenes

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"


def declared_functions() -> list[str]:
    text = (ROOT / "include" / "rt_hip.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    L = N.lib()
    names = declared_functions()
    assert len(names) >= 18
    for name in names:
        assert hasattr(L, name), name
    assert set(names) == set(N.SIGNATURES), "ctypes signature table out of sync with include/rt_hip.h"
    assert L.rt_abi_version() == N.RT_ABI_VERSION == 11
    assert C.sizeof(N.RtTuning) == 128   # sizeof(rt_tuning) (v5: + coh_refill, f64_kernel, grid_workgroups, front_spheres; v8: + sphere_grid_density; v9: + sphere_grid_time_slabs)


def test_comm_argument_validation():
    """RCCL entry points reject bad arguments (and NULL contexts) before touching RCCL;
    an id can be made without a GPU (it is a bootstrap address, rank 0 shares it)."""
    L = N.lib()
    uid = N.comm_unique_id()
    assert len(uid) == N.RT_COMM_ID_BYTES and any(uid)
    assert L.rt_comm_unique_id(None) == N.RT_ERR_INVALID
    assert L.rt_comm_init_rank(None, 2, 0, uid) == N.RT_ERR_INVALID
    assert L.rt_comm_init_all(None, 2) == N.RT_ERR_INVALID
    arr = (C.c_void_p * 2)(None, None)
    assert L.rt_comm_init_all(arr, 2) == N.RT_ERR_INVALID
    assert L.rt_comm_init_all(arr, 0) == N.RT_ERR_INVALID
    r, n = C.c_int(), C.c_int()
    assert L.rt_comm_rank(None, C.byref(r), C.byref(n)) == N.RT_ERR_INVALID
    assert L.rt_comm_destroy(None) == N.RT_ERR_INVALID
    assert L.rt_gather_shards(None, None, None, 8, 8, None) == N.RT_ERR_INVALID
    assert L.rt_finish_frame_u8(None, None, 8, 8, 1, 1, None, None) == N.RT_ERR_INVALID
    assert L.rt_render_frame_u8(None, None, 1, 1, None) == N.RT_ERR_INVALID
    assert L.rt_error_string(N.RT_ERR_COMM) != b"unknown error"


def test_struct_layouts_match_header():
    assert C.sizeof(N.RtCamera) == 8 + 6 * 24 + 8
    assert N.SPHERE_DTYPE.itemsize == 64 and N.MATERIAL_DTYPE.itemsize == 48
    assert C.sizeof(N.RtCameraDesc) == 8 + 16 + 8 + 72 + 16


def test_traversal_flags_match_header():
    """The Python traversal flags equal rt_hip.h's enum, and the default kernel is the
    coherent one with whole-record reads, root selection, pop culling (mesh and fp32 scenes
    without a sphere grid) and the uniform sphere grid (ABI 8)."""
    text = (ROOT / "include" / "rt_hip.h").read_text()
    enum = dict((k, int(v)) for k, v in re.findall(r"\b(RT_TRAV_[A-Z0-9]+) = (\d+)\b", text))
    assert len(enum) >= 6
    for k, v in enum.items():
        assert getattr(N, k) == v, k
    default = re.search(r"RT_TRAV_DEFAULT = ([A-Z0-9_ |]+)\}", text).group(1)
    bits = [enum[x.strip()] for x in default.split("|")]
    assert sum(bits) == (N.RT_TRAV_COH | N.RT_TRAV_SELROOT | N.RT_TRAV_B128 | N.RT_TRAV_CULL
                         | N.RT_TRAV_GRID) == 66136


def test_no_device_fails_loudly():
    """No CPU fallback: without a GPU, creating a renderer raises."""
    if N.lib().rt_device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(N.RtError):
        N.Renderer(0)


def test_rtweekend_stream_matches_reference():
    pm = json.loads((GOLDEN / "pixelmatch.json").read_text())
    rtweekend.reset_stream()
    assert [rtweekend.random_double() for _ in pm["first_random_doubles"]] == pm["first_random_doubles"]


def test_random_scene_builder_matches_reference():
    """scenes.random_spheres() == the 485 spheres of the reference binary, bit for bit."""
    rtweekend.reset_stream()
    world = scenes.random_spheres()
    S, M = api.flatten(world)
    rows = [l.split() for l in (GOLDEN / "scene_random.txt").read_text().splitlines() if not l.startswith("#")]
    assert len(S) == len(rows) == 485
    for k, row in enumerate(rows):
        v = [float(x) for x in row]
        assert S[k]["moving"] == int(v[0])
        assert S[k]["center"].tolist() == v[1:4]
        assert S[k]["center_vec"].tolist() == v[4:7]
        assert S[k]["radius"] == v[7]
        m = M[S[k]["mat"]]
        assert m["type"] == int(v[8])
        assert m["albedo"].tolist() == v[9:12]
        assert m["fuzz"] == v[12] and m["ir"] == v[13]


def test_camera_initialize_matches_reference():
    cams = json.loads((GOLDEN / "camera_init.json").read_text())
    for key, ref in cams.items():
        cam = scenes.main_camera()
        cam.image_width = int(key.split("_")[1])
        c = cam.native
        assert c.image_height == ref["image_height"]
        for f in ("center", "pixel00_loc", "pixel_delta_u", "pixel_delta_v", "defocus_disk_u", "defocus_disk_v"):
            assert list(getattr(c, f)) == ref[f], (key, f)


def test_camera_initialize_matches_oracle_for_other_fields():
    for w, aspect, vfov, dfa in ((97, 1.3, 35.0, 0.0), (1, 2.0, 90.0, 3.0), (640, 0.5, 10.0, 0.6)):
        cam = api.camera()
        cam.image_width, cam.aspect_ratio, cam.vfov, cam.defocus_angle = w, aspect, vfov, dfa
        cam.lookfrom, cam.lookat = (1.5, 2.0, -7.0), (0.25, 0.5, 0.0)
        c = cam.native
        o = O.OrcCamera()
        O.lib().orc_camera_defaults(C.byref(o))
        o.image_width, o.aspect_ratio, o.vfov, o.defocus_angle = w, aspect, vfov, dfa
        o.lookfrom[:] = (1.5, 2.0, -7.0)
        o.lookat[:] = (0.25, 0.5, 0.0)
        o.vup[:] = (0, 1, 0)
        o.focus_dist = 10.0
        O.lib().orc_camera_initialize(C.byref(o))
        assert c.image_height == o.image_height
        for f in ("center", "pixel00_loc", "pixel_delta_u", "pixel_delta_v", "defocus_disk_u", "defocus_disk_v"):
            assert list(getattr(c, f)) == list(getattr(o, f)), f


@pytest.mark.parametrize("W,H,n", [(1920, 1080, 1), (1920, 1080, 8), (401, 225, 3), (8, 8, 5), (1, 1, 2),
                                   (1280, 720, 7)])
def test_shard_layout_partitions_every_tile_once(W, H, n):
    seen = np.zeros(((W + 7) // 8) * ((H + 7) // 8), dtype=np.int32)
    total = 0
    for s in range(n):
        info = N.shard_layout(W, H, s, n)
        assert info.tiles_x == (W + 7) // 8 and info.num_tiles == len(seen)
        assert info.max_shard_tiles == -(-info.num_tiles // n)
        tiles = [lt * n + s for lt in range(info.shard_tiles)]
        assert all(t < info.num_tiles for t in tiles)
        seen[tiles] += 1
        total += info.shard_tiles
    assert total == len(seen) and np.all(seen == 1)


def test_shard_layout_rejects_bad_arguments():
    with pytest.raises(N.RtError):
        N.shard_layout(0, 10, 0, 1)
    with pytest.raises(N.RtError):
        N.shard_layout(10, 10, 2, 2)


def test_flatten_shares_materials_and_rejects_unknown():
    shared = api.lambertian((0.1, 0.2, 0.3))
    w = api.hittable_list()
    w.add(api.sphere((0, 0, 0), 1, shared))
    w.add(api.bvh_node(api.hittable_list(api.sphere((1, 0, 0), (1, 1, 0), 0.5, shared))))
    w.add(api.sphere((2, 0, 0), 1, api.metal((1, 1, 1), 3.0)))
    S, M = api.flatten(w)
    assert len(S) == 3 and len(M) == 2
    assert S[0]["mat"] == S[1]["mat"] == 0
    assert S[1]["moving"] == 1 and S[1]["center_vec"].tolist() == [0.0, 1.0, 0.0]
    assert M[1]["fuzz"] == 1.0  # material.h:33 clamp
    with pytest.raises(TypeError):
        api.flatten(object())


def test_write_ppm_format():
    import io
    rgb = np.array([[[220, 235, 255], [1, 2, 3]]], dtype=np.int32)
    buf = io.StringIO()
    api.write_ppm(buf, rgb)
    assert buf.getvalue() == "P3\n2 1\n255\n220 235 255\n1 2 3\n"

"""The instrumented kernel (rt_render_diag / rt_render_diag_ex, tools/diag.py): its
counters obey the invariants of the kernel they instrument.  Needs an MI355X."""
import pytest

from raytracingproject_amd import _native as N
from raytracingproject_amd import api, rtweekend, scenes

pytestmark = pytest.mark.gpu


def _diag(traversal: int, width: int = 96, spp: int = 8, depth: int = 50) -> tuple[dict, int, int]:
    rtweekend.reset_stream()
    world = scenes.random_spheres()
    cam_api = scenes.main_camera()
    cam_api.image_width, cam_api.samples_per_pixel = width, spp
    cam = cam_api.native
    with N.Renderer(0, 0x5EED, N.RT_PREC_F32) as r:
        r.set_tuning(traversal=traversal)
        r.upload_scene(*api.flatten(world))
        d = r.render_diag(cam, spp, depth)
        # the same frame through the product kernel: world.hit calls per pixel
        _, _, segs = r.render_frame(cam, spp, depth)
    return d, int(segs.sum()), cam.image_width * cam.image_height * spp


@pytest.mark.parametrize("traversal", [N.RT_TRAV_DEFAULT, N.RT_TRAV_DEFAULT | N.RT_TRAV_NOSUM])
def test_coherent_diag_counts_every_path_once(traversal):
    d, segs, paths = _diag(traversal)
    assert d["flushes"] == paths            # slot 11: every camera sample finishes exactly once
    assert d["x15"] <= paths                # primary hits popped (misses end in the batch)
    # secondaries traced in the bounce loop + camera rays = the product kernel's world.hit calls
    assert d["segments"] + paths == segs
    assert 0 < d["bounce_act"] <= 64 * d["bounce_it"]
    assert 0 < d["inner_act"] <= 64 * d["inner_it"] and 0 < d["leaf_act"] <= 64 * d["leaf_it"]
    # every finished sample went into its item's LDS sums or straight to HBM
    assert d["samples_in_item"] + d["samples_direct"] == paths


def test_coherent_diag_timeline_is_ordered():
    d, _, _ = _diag(N.RT_TRAV_DEFAULT)
    m = (1 << 64) - 1
    start, end = m - d["rt_start_min_not"], d["rt_end_max"]
    dry0, dry1 = m - d["rt_dry_min_not"], d["rt_dry_max"]
    assert d["waves"] > 0
    assert start <= dry0 <= dry1 <= end
    # per wave: (end - dry) + (dry - start) = its lifetime <= the kernel span
    assert d["rt_drain_sum"] + d["rt_busy_sum"] <= d["waves"] * (end - start)
    assert d["drain_bounce_it"] <= d["bounce_it"]


def test_diag_ex_rejects_bad_counts():
    rtweekend.reset_stream()
    cam_api = scenes.main_camera()
    cam_api.image_width, cam_api.samples_per_pixel = 32, 1
    cam = cam_api.native
    with N.Renderer(0, 0x5EED, N.RT_PREC_F32) as r:
        r.upload_scene(*api.flatten(scenes.four_spheres()))
        import ctypes as C
        c = (C.c_uint64 * (N.RT_DIAG_SLOTS + 1))()
        for n in (0, N.RT_DIAG_SLOTS + 1):
            assert r._L.rt_render_diag_ex(r.ctx, C.byref(cam), 1, 4, c, n) == N.RT_ERR_INVALID


def test_diag_refuses_uninstrumented_kernels():
    """rt_render_diag instruments exactly the kernel rt_render runs; a tuning with no
    instrumented build (here the kernel without pop culling) is refused, never substituted."""
    rtweekend.reset_stream()
    cam_api = scenes.main_camera()
    cam_api.image_width, cam_api.samples_per_pixel = 32, 1
    cam = cam_api.native
    with N.Renderer(0, 0x5EED, N.RT_PREC_F32) as r:
        r.set_tuning(traversal=N.RT_TRAV_COH | N.RT_TRAV_SELROOT | N.RT_TRAV_B128)
        r.upload_scene(*api.flatten(scenes.random_spheres()))
        with pytest.raises(N.RtError):
            r.render_diag(cam, 1, 4)
        r.render_frame(cam, 1, 4)   # the product kernel itself renders


@pytest.mark.parametrize("scene", ["mesh", "mixed"])
def test_mesh_diag_counts_every_path_once(scene):
    """Mesh scenes: the instrumented default mesh kernel finishes every camera sample
    once, its traced rays equal the product kernel's world.hit calls, and the mesh-BVH
    loop counters (node visits, triangle tests) are consistent."""
    rtweekend.reset_stream()
    world = scenes.mesh_only(level=3) if scene == "mesh" else scenes.mixed(level=3)
    S, M, T = api.flatten_scene(world)
    cam_api = scenes.main_camera()
    cam_api.image_width, cam_api.samples_per_pixel = 96, 8
    cam = cam_api.native
    paths = cam.image_width * cam.image_height * 8
    with N.Renderer(0, 0x5EED, N.RT_PREC_F32) as r:
        r.upload_scene(S, M, T)
        d = r.render_diag(cam, 8, 50)
        _, _, segs = r.render_frame(cam, 8, 50)
    assert d["flushes"] == paths
    assert d["segments"] + paths == int(segs.sum())
    assert 0 < d["mnode_act"] <= 64 * d["mnode_it"]
    assert 0 < d["mtri_act"] <= 64 * d["mtri_it"]

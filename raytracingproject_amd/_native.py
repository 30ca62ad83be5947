"""ctypes binding of the C ABI in include/rt_hip.h (librt_hip.so, built in-tree).

There is no fallback: if the library is missing or a call fails, this raises.  The
tests, smoke() and bench.py all reach the GPU through this module.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

import os

LIB_PATH = Path(os.environ.get("RT_LIB_PATH", Path(__file__).resolve().parent / "lib" / "librt_hip.so"))

RT_OK, RT_ERR_INVALID, RT_ERR_HIP, RT_ERR_NO_SCENE, RT_ERR_LIMIT, RT_ERR_COMM = 0, -1, -2, -3, -4, -5
RT_ABI_VERSION = 11
RT_TRAV_SELROOT, RT_TRAV_B128, RT_TRAV_COH = 8, 16, 64   # rt_hip.h traversal flags
RT_TRAV_NOSUM, RT_TRAV_TBIN, RT_TRAV_CULL, RT_TRAV_MTOP, RT_TRAV_MIFIF, RT_TRAV_MWHILE = 128, 256, 512, 4096, 8192, 16384
RT_TRAV_MQ = 32768
RT_TRAV_GRID = 65536   # fp32 sphere scenes: the uniform sphere grid (ABI 8)
RT_TRAV_GFLAT, RT_TRAV_G3D = 131072, 262144   # its flat walk (added by the library), keep the 3-D walk (ABI 11)
# (RT_TRAV_TBIN and RT_TRAV_MTOP: removed in ABI 6, refused by rt_set_tuning)
RT_TRAV_DEFAULT = RT_TRAV_COH | RT_TRAV_SELROOT | RT_TRAV_B128 | RT_TRAV_CULL | RT_TRAV_GRID
RT_DIAG_SLOTS = 32   # rt_hip.h: counters of rt_render_diag_ex
RT_COMM_ID_BYTES = 128
RT_LAMBERTIAN, RT_METAL, RT_DIELECTRIC = 0, 1, 2
RT_PREC_F32, RT_PREC_F64 = 0, 1
RT_MESH_BUILD_HOST, RT_MESH_BUILD_GPU, RT_MESH_BUILD_GPU_LBVH = 0, 1, 2   # (2: ABI 10)

# rt_sphere / rt_material as numpy structured dtypes (64 B / 48 B, C layout)
SPHERE_DTYPE = np.dtype([("center", "<f8", (3,)), ("radius", "<f8"), ("center_vec", "<f8", (3,)),
                         ("mat", "<i4"), ("moving", "<i4")])
MATERIAL_DTYPE = np.dtype([("type", "<i4"), ("pad", "<i4"), ("albedo", "<f8", (3,)), ("fuzz", "<f8"),
                           ("ir", "<f8")])
# rt_triangle (80 B)
TRIANGLE_DTYPE = np.dtype([("v0", "<f8", (3,)), ("v1", "<f8", (3,)), ("v2", "<f8", (3,)), ("mat", "<i4"),
                           ("pad", "<i4")])
assert SPHERE_DTYPE.itemsize == 64 and MATERIAL_DTYPE.itemsize == 48 and TRIANGLE_DTYPE.itemsize == 80

D3 = C.c_double * 3


class RtCamera(C.Structure):
    _fields_ = [("image_width", C.c_int32), ("image_height", C.c_int32), ("center", D3), ("pixel00_loc", D3),
                ("pixel_delta_u", D3), ("pixel_delta_v", D3), ("defocus_disk_u", D3), ("defocus_disk_v", D3),
                ("defocus_angle", C.c_double)]


class RtCameraDesc(C.Structure):
    _fields_ = [("aspect_ratio", C.c_double), ("image_width", C.c_int32), ("samples_per_pixel", C.c_int32),
                ("max_depth", C.c_int32), ("pad", C.c_int32), ("vfov", C.c_double), ("lookfrom", D3),
                ("lookat", D3), ("vup", D3), ("defocus_angle", C.c_double), ("focus_dist", C.c_double)]


class RtShardInfo(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("tile_w", "tile_h", "tiles_x", "tiles_y", "num_tiles", "shard",
                                         "num_shards", "shard_tiles", "max_shard_tiles")]


class RtSceneInfo(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("num_spheres", "num_materials", "bvh_nodes", "bvh_depth", "bvh_leaves",
                                         "big_spheres", "lds_bytes", "precision", "num_triangles",
                                         "mesh_nodes", "mesh_depth", "mesh_leaves", "render_block",
                                         "render_traversal", "render_waves_per_eu", "render_mesh_lds_stack")] + \
        [("grid_res", C.c_int32 * 3), ("grid_entries", C.c_int32),
         # ABI 10: the grid's build parameters and its walk's reach (rt_hip.h)
         ("grid_time_slabs", C.c_int32), ("grid_far_o", C.c_float), ("grid_density", C.c_double)]


class RtObjMesh(C.Structure):
    _fields_ = [("num_vertices", C.c_int32), ("num_faces", C.c_int32), ("num_triangles", C.c_int32),
                ("pad", C.c_int32), ("vertices", C.POINTER(C.c_double)), ("indices", C.POINTER(C.c_int32))]


class RtTuning(C.Structure):
    _fields_ = [("block", C.c_int32), ("max_leaf", C.c_int32), ("cost_traverse", C.c_double),
                ("cost_intersect", C.c_double), ("waves_per_eu", C.c_int32), ("traversal", C.c_int32),
                ("mesh_max_leaf", C.c_int32), ("mesh_lds_nodes", C.c_int32), ("mesh_cost_traverse", C.c_double),
                ("chunk_waves", C.c_int32), ("sample_buffer_mb", C.c_int32), ("mesh_builder", C.c_int32),
                ("mesh_waves_per_eu", C.c_int32), ("mesh_lds_stack", C.c_int32),
                ("mesh_block", C.c_int32), ("item_samples", C.c_int32), ("item_balance", C.c_double),
                ("mesh_item_balance", C.c_double), ("coh_refill", C.c_int32), ("f64_kernel", C.c_int32),
                ("grid_workgroups", C.c_int32), ("front_spheres", C.c_int32),
                ("sphere_grid_density", C.c_double), ("sphere_grid_time_slabs", C.c_int32)]


# name -> (restype, argtypes); the full exported surface of include/rt_hip.h
SIGNATURES = {
    "rt_abi_version": (C.c_int, []),
    "rt_device_count": (C.c_int, []),
    "rt_create": (C.c_void_p, [C.c_int, C.c_uint64, C.c_int]),
    "rt_destroy": (None, [C.c_void_p]),
    "rt_last_error": (C.c_char_p, [C.c_void_p]),
    "rt_error_string": (C.c_char_p, [C.c_int]),
    "rt_set_seed": (C.c_int, [C.c_void_p, C.c_uint64]),
    "rt_stream": (C.c_void_p, [C.c_void_p]),
    "rt_get_tuning": (C.c_int, [C.c_void_p, C.POINTER(RtTuning)]),
    "rt_set_tuning": (C.c_int, [C.c_void_p, C.POINTER(RtTuning)]),
    "rt_camera_initialize": (C.c_int, [C.POINTER(RtCameraDesc), C.POINTER(RtCamera)]),
    "rt_upload_scene": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int]),
    "rt_scene_info_get": (C.c_int, [C.c_void_p, C.POINTER(RtSceneInfo)]),
    "rt_grid_reach": (C.c_int, [C.c_void_p, C.POINTER(RtCamera), C.POINTER(C.c_int32)]),   # ABI 10
    "rt_upload_scene_ex": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_int]),
    "rt_obj_load": (C.c_int, [C.c_char_p, C.POINTER(RtObjMesh)]),
    "rt_obj_free": (None, [C.POINTER(RtObjMesh)]),
    "rt_shard_layout": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(RtShardInfo)]),
    "rt_render": (C.c_int, [C.c_void_p, C.POINTER(RtCamera), C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                            C.c_void_p, C.c_void_p]),
    "rt_last_kernel_ms": (C.c_int, [C.c_void_p, C.POINTER(C.c_float)]),
    "rt_render_range": (C.c_int, [C.c_void_p, C.POINTER(RtCamera), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                  C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]),
    "rt_unshard": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]),
    "rt_quantize": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]),
    "rt_render_frame": (C.c_int, [C.c_void_p, C.POINTER(RtCamera), C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                  C.c_void_p]),
    "rt_finish_frame_u8": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                     C.c_void_p]),
    "rt_host_alloc": (C.c_void_p, [C.c_size_t]),
    "rt_host_free": (None, [C.c_void_p]),
    "rt_render_frame_u8": (C.c_int, [C.c_void_p, C.POINTER(RtCamera), C.c_int, C.c_int, C.c_void_p]),
    "rt_comm_unique_id": (C.c_int, [C.c_char_p]),
    "rt_comm_init_rank": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_char_p]),
    "rt_comm_init_rank_timeout": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_char_p, C.c_int]),
    "rt_comm_init_all": (C.c_int, [C.POINTER(C.c_void_p), C.c_int]),
    "rt_comm_rank": (C.c_int, [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "rt_comm_destroy": (C.c_int, [C.c_void_p]),
    "rt_gather_shards": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p]),
    "rt_render_frame_multi": (C.c_int, [C.POINTER(C.c_void_p), C.c_int, C.POINTER(RtCamera), C.c_int, C.c_int,
                                        C.c_void_p, C.c_void_p]),
    "rt_render_diag": (C.c_int, [C.c_void_p, C.POINTER(RtCamera), C.c_int, C.c_int, C.POINTER(C.c_uint64)]),
    "rt_render_diag_ex": (C.c_int, [C.c_void_p, C.POINTER(RtCamera), C.c_int, C.c_int, C.POINTER(C.c_uint64),
                                    C.c_int]),
    "rt_trace_tape": (C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.c_int, C.POINTER(C.c_double), C.c_int,
                                C.POINTER(C.c_double), C.POINTER(C.c_int)]),
    "rt_trace_rays": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]),
    "rt_trace_rays_diag": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.POINTER(C.c_uint64)]),
}

# rt_hit (72 B): rt_trace_rays' per-ray hit record
HIT_DTYPE = np.dtype([("t", "<f8"), ("p", "<f8", (3,)), ("normal", "<f8", (3,)), ("id", "<i4"),
                      ("front_face", "<i4"), ("mat", "<i4"), ("pad", "<i4")])
assert HIT_DTYPE.itemsize == 72

_LIB = None


def lib() -> C.CDLL:
    """Load librt_hip.so (fails loudly if it was not built).

    torch (when installed) is imported first: the ROCm torch wheel carries its own
    libamdhip64 under a different DT_NEEDED name, and whichever HIP runtime loads
    second in a process cannot open the GPU.  With torch first, librt_hip.so binds to
    the already-loaded runtime and both share one device context."""
    global _LIB
    if _LIB is None:
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not LIB_PATH.exists():
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -m raytracingproject_amd.build` "
                               "(there is no CPU fallback)")
        L = C.CDLL(str(LIB_PATH))
        # RT_ALLOW_ABI_MISMATCH=1 (same-box A/B against an older build through RT_LIB_PATH,
        # tools/gpu_session.sh ab*): entry points that build lacks stay unbound, and its ABI
        # version is not enforced.  RT_LIB_PATH alone keeps both checks.
        ab = os.environ.get("RT_ALLOW_ABI_MISMATCH") == "1"
        for name, (res, args) in SIGNATURES.items():
            if ab and not hasattr(L, name):
                continue
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        if L.rt_abi_version() != RT_ABI_VERSION and not ab:
            raise RuntimeError(f"{LIB_PATH}: ABI version {L.rt_abi_version()}, this package expects "
                               f"{RT_ABI_VERSION} (rebuild it, or set RT_ALLOW_ABI_MISMATCH=1 for an A/B run)")
        _LIB = L
    return _LIB


class RtError(RuntimeError):
    pass


def render_frame_multi(renderers, cam, spp: int, max_depth: int):
    """rt_render_frame_multi: renderer r renders shard r of len(renderers); the frame is
    assembled on renderers[0]'s GPU.  -> (sums[H,W,3], rgb int32[H,W,3])."""
    L = lib()
    W, H = cam.image_width, cam.image_height
    r0 = renderers[0]
    sums = np.empty((H, W, 3), dtype=r0.dtype)
    rgb = np.empty((H, W, 3), dtype=np.int32)
    arr = (C.c_void_p * len(renderers))(*[r.ctx for r in renderers])
    rc = L.rt_render_frame_multi(arr, len(renderers), C.byref(cam), spp, max_depth, _ptr(sums), _ptr(rgb))
    if rc != RT_OK:
        raise RtError(f"rt_render_frame_multi: {L.rt_error_string(rc).decode()} ({L.rt_last_error(r0.ctx).decode()})")
    return sums, rgb


def comm_unique_id() -> bytes:
    """rt_comm_unique_id: an RCCL id (128 bytes) rank 0 shares with the other ranks."""
    buf = C.create_string_buffer(RT_COMM_ID_BYTES)
    rc = lib().rt_comm_unique_id(buf)
    if rc != RT_OK:
        raise RtError(f"rt_comm_unique_id: {lib().rt_error_string(rc).decode()}")
    return buf.raw


def comm_init_all(renderers) -> None:
    """rt_comm_init_all: one RCCL communicator over the renderers' GPUs (one process)."""
    L = lib()
    arr = (C.c_void_p * len(renderers))(*[r.ctx for r in renderers])
    rc = L.rt_comm_init_all(arr, len(renderers))
    if rc != RT_OK:
        raise RtError(f"rt_comm_init_all: {L.rt_error_string(rc).decode()} "
                      f"({L.rt_last_error(renderers[0].ctx).decode()})")


def host_alloc(nbytes: int) -> np.ndarray:
    """Page-locked host buffer (rt_host_alloc) as a uint8 array; freed with host_free."""
    p = lib().rt_host_alloc(nbytes)
    if not p:
        raise RtError(f"rt_host_alloc({nbytes}) failed")
    return np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(p))


def host_free(a: np.ndarray) -> None:
    lib().rt_host_free(C.c_void_p(a.ctypes.data))


def obj_load(path) -> tuple[np.ndarray, np.ndarray, int]:
    """rt_obj_load: (vertices[nv,3] f64, triangles[nt,3] i32 0-based, num_faces)."""
    m = RtObjMesh()
    rc = lib().rt_obj_load(str(path).encode(), C.byref(m))
    if rc != RT_OK:
        raise RtError(f"rt_obj_load({path}): {lib().rt_error_string(rc).decode()}")
    try:
        V = np.ctypeslib.as_array(m.vertices, (m.num_vertices * 3,)).reshape(-1, 3).copy() if m.num_vertices else \
            np.zeros((0, 3))
        F = np.ctypeslib.as_array(m.indices, (m.num_triangles * 3,)).reshape(-1, 3).copy() if m.num_triangles else \
            np.zeros((0, 3), np.int32)
        return V, F, m.num_faces
    finally:
        lib().rt_obj_free(C.byref(m))


def triangles(V: np.ndarray, F: np.ndarray, mat: int) -> np.ndarray:
    """Indexed mesh -> rt_triangle records, all with material index `mat`."""
    t = np.zeros(len(F), TRIANGLE_DTYPE)
    t["v0"], t["v1"], t["v2"] = V[F[:, 0]], V[F[:, 1]], V[F[:, 2]]
    t["mat"] = mat
    return t


def _ptr(a: np.ndarray) -> C.c_void_p:
    return C.c_void_p(a.ctypes.data)


def camera_initialize(desc: RtCameraDesc) -> RtCamera:
    cam = RtCamera()
    rc = lib().rt_camera_initialize(C.byref(desc), C.byref(cam))
    if rc != RT_OK:
        raise RtError(f"rt_camera_initialize: {rc}")
    return cam


def shard_layout(width: int, height: int, shard: int, num_shards: int) -> RtShardInfo:
    info = RtShardInfo()
    rc = lib().rt_shard_layout(width, height, shard, num_shards, C.byref(info))
    if rc != RT_OK:
        raise RtError(f"rt_shard_layout({width},{height},{shard},{num_shards}) = {rc}")
    return info


class Renderer:
    """One rt_ctx: a GPU, a precision, an RNG seed and an uploaded scene."""

    def __init__(self, device: int = 0, seed: int = 0x5EED, precision: int = RT_PREC_F32):
        self._L = lib()
        self.precision = precision
        self.dtype = np.float64 if precision == RT_PREC_F64 else np.float32
        self.ctx = self._L.rt_create(device, seed, precision)
        if not self.ctx:
            raise RtError(f"rt_create(device={device}) failed (no HIP device?)")

    def close(self) -> None:
        if self.ctx:
            self._L.rt_destroy(self.ctx)
            self.ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, what: str) -> None:
        if rc != RT_OK:
            msg = self._L.rt_last_error(self.ctx).decode()
            raise RtError(f"{what}: {self._L.rt_error_string(rc).decode()} ({msg})")

    def set_seed(self, seed: int) -> None:
        self._check(self._L.rt_set_seed(self.ctx, seed), "rt_set_seed")

    def tuning(self) -> RtTuning:
        t = RtTuning()
        self._check(self._L.rt_get_tuning(self.ctx, C.byref(t)), "rt_get_tuning")
        return t

    def set_tuning(self, **kw) -> None:
        t = self.tuning()
        for k, v in kw.items():
            setattr(t, k, v)
        self._check(self._L.rt_set_tuning(self.ctx, C.byref(t)), "rt_set_tuning")

    @property
    def stream(self) -> int:
        return self._L.rt_stream(self.ctx) or 0

    def upload_scene(self, spheres: np.ndarray, materials: np.ndarray, tris: np.ndarray | None = None) -> None:
        spheres = np.ascontiguousarray(spheres, dtype=SPHERE_DTYPE)
        materials = np.ascontiguousarray(materials, dtype=MATERIAL_DTYPE)
        if tris is None:
            self._check(self._L.rt_upload_scene(self.ctx, _ptr(spheres), len(spheres), _ptr(materials),
                                                len(materials)), "rt_upload_scene")
            return
        tris = np.ascontiguousarray(tris, dtype=TRIANGLE_DTYPE)
        self._check(self._L.rt_upload_scene_ex(self.ctx, _ptr(spheres), len(spheres), _ptr(materials), len(materials),
                                               _ptr(tris), len(tris)), "rt_upload_scene_ex")

    def scene_info(self) -> RtSceneInfo:
        info = RtSceneInfo()
        self._check(self._L.rt_scene_info_get(self.ctx, C.byref(info)), "rt_scene_info_get")
        return info

    def grid_reach(self, cam: RtCamera) -> bool:
        """rt_grid_reach: does a launch with this camera walk the sphere grid (else the tree)?"""
        w = C.c_int32()
        self._check(self._L.rt_grid_reach(self.ctx, C.byref(cam), C.byref(w)), "rt_grid_reach")
        return bool(w.value)

    def render_frame(self, cam: RtCamera, spp: int, max_depth: int, want_segments: bool = True):
        """Whole frame, host outputs: (sums[H,W,3], rgb int32[H,W,3], segments uint32[H,W])."""
        W, H = cam.image_width, cam.image_height
        sums = np.empty((H, W, 3), dtype=self.dtype)
        rgb = np.empty((H, W, 3), dtype=np.int32)
        segs = np.empty((H, W), dtype=np.uint32) if want_segments else None
        self._check(self._L.rt_render_frame(self.ctx, C.byref(cam), spp, max_depth, _ptr(sums), _ptr(rgb),
                                            _ptr(segs) if segs is not None else None), "rt_render_frame")
        return sums, rgb, segs

    def render_frame_u8(self, cam: RtCamera, spp: int, max_depth: int, out: np.ndarray | None = None) -> np.ndarray:
        """Whole frame, 8-bit host output (rt_render_frame_u8): uint8[H,W,3]."""
        W, H = cam.image_width, cam.image_height
        if out is None:
            out = np.empty((H, W, 3), dtype=np.uint8)
        assert out.dtype == np.uint8 and out.size == W * H * 3 and out.flags.c_contiguous
        self._check(self._L.rt_render_frame_u8(self.ctx, C.byref(cam), spp, max_depth, _ptr(out)),
                    "rt_render_frame_u8")
        return out.reshape(H, W, 3)

    def finish_u8(self, gathered_dev: int, width: int, height: int, num_shards: int, spp: int, rgb8_dev: int,
                  stream: int | None = None) -> None:
        """rt_finish_frame_u8: stacked shard buffers -> row-major uint8 frame (device)."""
        self._check(self._L.rt_finish_frame_u8(self.ctx, C.c_void_p(gathered_dev), width, height, num_shards, spp,
                                               C.c_void_p(rgb8_dev), C.c_void_p(stream or 0)), "rt_finish_frame_u8")

    def comm_init_rank(self, nranks: int, rank: int, uid: bytes, timeout_ms: int | None = None) -> None:
        """RCCL communicator rank `rank` of `nranks` (non-blocking init polled against a
        deadline: RtError if the other ranks do not all join within timeout_ms)."""
        assert len(uid) == RT_COMM_ID_BYTES
        if timeout_ms is None:
            self._check(self._L.rt_comm_init_rank(self.ctx, nranks, rank, uid), "rt_comm_init_rank")
        else:
            self._check(self._L.rt_comm_init_rank_timeout(self.ctx, nranks, rank, uid, timeout_ms),
                        "rt_comm_init_rank_timeout")

    def comm_rank(self) -> tuple[int, int]:
        r, n = C.c_int(), C.c_int()
        self._check(self._L.rt_comm_rank(self.ctx, C.byref(r), C.byref(n)), "rt_comm_rank")
        return r.value, n.value

    def comm_destroy(self) -> None:
        self._check(self._L.rt_comm_destroy(self.ctx), "rt_comm_destroy")

    def gather_shards(self, shard_dev: int, gathered_dev: int | None, width: int, height: int,
                      stream: int | None = None) -> None:
        """rt_gather_shards: ncclGather of this rank's shard to rank 0's stacked buffer."""
        self._check(self._L.rt_gather_shards(self.ctx, C.c_void_p(shard_dev), C.c_void_p(gathered_dev or 0), width,
                                             height, C.c_void_p(stream or 0)), "rt_gather_shards")

    def render(self, cam: RtCamera, spp: int, max_depth: int, shard: int, num_shards: int, out_sums_dev: int,
               out_segs_dev: int | None = None, stream: int | None = None) -> None:
        """Asynchronous shard render into device memory (torch tensors' data_ptr())."""
        self._check(self._L.rt_render(self.ctx, C.byref(cam), spp, max_depth, shard, num_shards,
                                      C.c_void_p(out_sums_dev), C.c_void_p(out_segs_dev or 0),
                                      C.c_void_p(stream or 0)), "rt_render")

    def render_range(self, cam: RtCamera, sample_begin: int, sample_count: int, max_depth: int, shard: int,
                     num_shards: int, accumulate: bool, out_sums_dev: int, out_segs_dev: int | None = None,
                     stream: int | None = None) -> None:
        self._check(self._L.rt_render_range(self.ctx, C.byref(cam), sample_begin, sample_count, max_depth, shard,
                                            num_shards, 1 if accumulate else 0, C.c_void_p(out_sums_dev),
                                            C.c_void_p(out_segs_dev or 0), C.c_void_p(stream or 0)),
                    "rt_render_range")

    def last_kernel_ms(self) -> float:
        ms = C.c_float()
        self._check(self._L.rt_last_kernel_ms(self.ctx, C.byref(ms)), "rt_last_kernel_ms")
        return float(ms.value)

    def unshard(self, gathered_dev: int, width: int, height: int, num_shards: int, frame_dev: int,
                stream: int | None = None) -> None:
        self._check(self._L.rt_unshard(self.ctx, C.c_void_p(gathered_dev), width, height, num_shards,
                                       C.c_void_p(frame_dev), C.c_void_p(stream or 0)), "rt_unshard")

    def quantize(self, frame_dev: int, width: int, height: int, spp: int, rgb_dev: int,
                 stream: int | None = None) -> None:
        self._check(self._L.rt_quantize(self.ctx, C.c_void_p(frame_dev), width, height, spp, C.c_void_p(rgb_dev),
                                        C.c_void_p(stream or 0)), "rt_quantize")

    def render_diag(self, cam: RtCamera, spp: int, max_depth: int) -> dict:
        c = (C.c_uint64 * RT_DIAG_SLOTS)()
        self._check(self._L.rt_render_diag_ex(self.ctx, C.byref(cam), spp, max_depth, c, RT_DIAG_SLOTS),
                    "rt_render_diag_ex")
        names = ["bounce_it", "bounce_act", "inner_it", "inner_act", "leaf_it", "leaf_act", "cyc_trav", "cyc_shade",
                 "cyc_hand", "cyc_all", "segments", "flushes", "k_it1", "k_it2", "k_it4", "x15",
                 # coherent kernel: wave timeline (s_memrealtime, 100 MHz; NOT-ed minima)
                 "rt_end_max", "rt_start_min_not", "rt_drain_sum", "rt_busy_sum", "rt_dry_min_not", "rt_dry_max",
                 "waves", "drain_bounce_it",
                 # coherent kernel: framebuffer traffic
                 "samples_in_item", "samples_direct", "item_flushes",
                 # mesh scenes: mesh BVH node visits and triangle tests (iterations, active lanes)
                 "mnode_it", "mnode_act", "mtri_it", "mtri_act", "x31"]
        return {n: int(c[k]) for k, n in enumerate(names)}

    def trace_rays(self, rays_dev: int, n: int, hits_dev: int, stream: int | None = None) -> None:
        """rt_trace_rays: n rays (7 values each, device) -> n rt_hit records (device)."""
        self._check(self._L.rt_trace_rays(self.ctx, C.c_void_p(rays_dev), n, C.c_void_p(hits_dev),
                                          C.c_void_p(stream or 0)), "rt_trace_rays")

    def trace_rays_host(self, rays: np.ndarray) -> np.ndarray:
        """rt_trace_rays through device copies: rays[n, 7] (context precision) -> HIT_DTYPE[n]."""
        import torch
        rays = np.ascontiguousarray(rays, dtype=self.dtype).reshape(-1, 7)
        n = len(rays)
        d_rays = torch.from_numpy(rays).to("cuda")
        d_hits = torch.empty(max(1, n) * HIT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        self.trace_rays(d_rays.data_ptr(), n, d_hits.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        return d_hits.cpu().numpy()[: n * HIT_DTYPE.itemsize].view(HIT_DTYPE)

    def trace_rays_diag(self, rays_dev: int, n: int, hits_dev: int) -> dict:
        c = (C.c_uint64 * 4)()
        self._check(self._L.rt_trace_rays_diag(self.ctx, C.c_void_p(rays_dev), n, C.c_void_p(hits_dev), c),
                    "rt_trace_rays_diag")
        return dict(zip(("inner_it", "inner_act", "leaf_it", "leaf_act"), (int(x) for x in c)))

    def trace_tape(self, ray7, depth: int, tape: np.ndarray):
        ray = (C.c_double * 7)(*ray7)
        tape = np.ascontiguousarray(tape, dtype=np.float64)
        out = (C.c_double * 3)()
        used = C.c_int()
        self._check(self._L.rt_trace_tape(self.ctx, ray, depth, tape.ctypes.data_as(C.POINTER(C.c_double)),
                                          len(tape), out, C.byref(used)), "rt_trace_tape")
        return (out[0], out[1], out[2]), used.value

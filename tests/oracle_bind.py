"""ctypes binding of oracle/liboracle.so -- TEST INFRASTRUCTURE (the checker).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this.  It
is never the thing measured or shipped.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import json
import subprocess
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
ORACLE_DIR = ROOT / "oracle"
LIB_PATH = ORACLE_DIR / "liboracle.so"
GOLDEN = ROOT / "tests" / "golden"
D3 = C.c_double * 3


class OrcSphere(C.Structure):
    _fields_ = [("center", D3), ("center_vec", D3), ("radius", C.c_double), ("moving", C.c_int32),
                ("mat", C.c_int32)]


class OrcMaterial(C.Structure):
    _fields_ = [("type", C.c_int32), ("pad", C.c_int32), ("albedo", D3), ("fuzz", C.c_double),
                ("ir", C.c_double)]


class OrcCamera(C.Structure):
    _fields_ = [("aspect_ratio", C.c_double), ("image_width", C.c_int32), ("samples_per_pixel", C.c_int32),
                ("max_depth", C.c_int32), ("image_height", C.c_int32), ("vfov", C.c_double), ("lookfrom", D3),
                ("lookat", D3), ("vup", D3), ("defocus_angle", C.c_double), ("focus_dist", C.c_double),
                ("center", D3), ("pixel00_loc", D3), ("pixel_delta_u", D3), ("pixel_delta_v", D3), ("u", D3),
                ("v", D3), ("w", D3), ("defocus_disk_u", D3), ("defocus_disk_v", D3)]


class OrcTriangle(C.Structure):
    _fields_ = [("v0", D3), ("v1", D3), ("v2", D3), ("mat", C.c_int32), ("pad", C.c_int32)]


class OrcRng(C.Structure):
    _fields_ = [("mode", C.c_int32), ("mt", C.c_uint32 * 624), ("mti", C.c_int32), ("key", C.c_uint32),
                ("ctr", C.c_uint32), ("draws", C.c_uint64)]


_LIB = None


def lib() -> C.CDLL:
    global _LIB
    if _LIB is None:
        if not LIB_PATH.exists():
            subprocess.run(["make", "-C", str(ORACLE_DIR), "liboracle.so"], check=True,
                           stdout=subprocess.DEVNULL)
        L = C.CDLL(str(LIB_PATH))
        P = C.POINTER
        L.orc_rng_init_mt.argtypes = [P(OrcRng)]
        L.orc_rng_init_counter.argtypes = [P(OrcRng)]
        L.orc_random_double.argtypes = [P(OrcRng)]
        L.orc_random_double.restype = C.c_double
        L.orc_scene_random.argtypes = [P(OrcRng), P(OrcSphere), P(OrcMaterial), C.c_int]
        L.orc_scene_four.argtypes = [P(OrcSphere), P(OrcMaterial), C.c_int]
        L.orc_scene_ground.argtypes = [P(OrcSphere), P(OrcMaterial), C.c_int]
        L.orc_camera_defaults.argtypes = [P(OrcCamera)]
        L.orc_camera_initialize.argtypes = [P(OrcCamera)]
        L.orc_get_ray.argtypes = [P(OrcCamera), P(OrcRng), C.c_int, C.c_int, P(C.c_double)]
        L.orc_ray_color.argtypes = [P(OrcSphere), P(OrcMaterial), C.c_int, P(C.c_double), C.c_int, P(OrcRng),
                                    P(C.c_double), P(C.c_uint64)]
        L.orc_write_color.argtypes = [P(C.c_double), C.c_int, P(C.c_int32)]
        L.orc_render_counter.argtypes = [P(OrcSphere), P(OrcMaterial), C.c_int, P(OrcCamera), C.c_uint64,
                                         P(C.c_int32), C.c_int, P(C.c_double), P(C.c_int32), P(C.c_uint64)]
        L.orc_trace_tape.argtypes = [P(OrcSphere), P(OrcMaterial), C.c_int, P(C.c_double), C.c_int,
                                     P(C.c_double), C.c_int, P(C.c_double)]
        L.orc_reference_main.argtypes = [C.c_int, C.c_int, P(C.c_int32)]
        L.orc_set_mesh.argtypes = [C.c_void_p, C.c_int]
        _LIB = L
    return _LIB


class OracleScene:
    """Spheres + materials (+ triangles, hit after the spheres by a linear scan)."""

    def __init__(self, name: str):
        self.s = (OrcSphere * 4096)()
        self.m = (OrcMaterial * 4096)()
        self.tris = None
        L = lib()
        if name == "arrays":
            self.n = 0
        elif name == "random":
            r = OrcRng()
            L.orc_rng_init_mt(C.byref(r))
            self.n = L.orc_scene_random(C.byref(r), self.s, self.m, 4096)
        elif name == "four":
            self.n = L.orc_scene_four(self.s, self.m, 4096)
        elif name == "ground":
            self.n = L.orc_scene_ground(self.s, self.m, 4096)
        else:
            raise ValueError(name)

    @classmethod
    def from_arrays(cls, S: np.ndarray, M: np.ndarray, T: np.ndarray | None = None) -> "OracleScene":
        """From the C-ABI arrays (rt_sphere / rt_material / rt_triangle numpy records)."""
        o = cls("arrays")
        if len(S) > 4096 or len(M) > 4096:
            raise ValueError("oracle scene capacity")
        for k, q in enumerate(S):
            o.s[k].center = D3(*q["center"])
            o.s[k].center_vec = D3(*q["center_vec"])
            o.s[k].radius = float(q["radius"])
            o.s[k].moving = int(q["moving"])
            o.s[k].mat = int(q["mat"])
        for k, q in enumerate(M):
            o.m[k].type = int(q["type"])
            o.m[k].albedo = D3(*q["albedo"])
            o.m[k].fuzz = min(float(q["fuzz"]), 1.0)   # material.h:33 (as rt_upload_scene)
            o.m[k].ir = float(q["ir"])
        o.n = len(S)
        if T is not None and len(T):
            assert T.dtype.itemsize == C.sizeof(OrcTriangle)
            o.tris = np.ascontiguousarray(T)
        return o

    @contextlib.contextmanager
    def active(self):
        """This scene's triangles as the oracle's mesh (global state in the C oracle) for
        the duration of one call; cleared afterwards so sphere-only callers see none."""
        if self.tris is not None:
            lib().orc_set_mesh(C.c_void_p(self.tris.ctypes.data), len(self.tris))
        try:
            yield
        finally:
            lib().orc_set_mesh(None, 0)


def camera(width: int, spp: int, depth: int = 50, aspect: float | None = None, vfov: float | None = None,
           defocus_angle: float | None = None) -> OrcCamera:
    c = OrcCamera()
    L = lib()
    L.orc_camera_defaults(C.byref(c))
    c.image_width, c.samples_per_pixel, c.max_depth = width, spp, depth
    if aspect is not None:
        c.aspect_ratio = aspect
    if vfov is not None:
        c.vfov = vfov
    if defocus_angle is not None:
        c.defocus_angle = defocus_angle
    L.orc_camera_initialize(C.byref(c))
    return c


def render_counter(scene: OracleScene, cam: OrcCamera, seed: int, ij: np.ndarray):
    """fp64 counter-RNG render of the pixels ij[n,2] -> (sums[n,3], rgb[n,3], segs[n])."""
    ij = np.ascontiguousarray(ij, dtype=np.int32)
    n = len(ij)
    sums = np.empty((n, 3), np.float64)
    rgb = np.empty((n, 3), np.int32)
    segs = np.empty(n, np.uint64)
    P = C.POINTER
    with scene.active():
        lib().orc_render_counter(scene.s, scene.m, scene.n, C.byref(cam), seed,
                                 ij.ctypes.data_as(P(C.c_int32)), n, sums.ctypes.data_as(P(C.c_double)),
                                 rgb.ctypes.data_as(P(C.c_int32)), segs.ctypes.data_as(P(C.c_uint64)))
    return sums, rgb, segs


def render_counter_full(scene: OracleScene, cam: OrcCamera, seed: int):
    W, H = cam.image_width, cam.image_height
    jj, ii = np.mgrid[0:H, 0:W]
    ij = np.stack([ii.ravel(), jj.ravel()], axis=1)
    sums, rgb, segs = render_counter(scene, cam, seed, ij)
    return sums.reshape(H, W, 3), rgb.reshape(H, W, 3), segs.reshape(H, W)


def trace_tape(scene: OracleScene, ray, depth: int, tape: np.ndarray):
    """orc_trace_tape -> (rgb[3], uniforms used)."""
    tape = np.ascontiguousarray(tape, dtype=np.float64)
    out = (C.c_double * 3)()
    with scene.active():
        used = lib().orc_trace_tape(scene.s, scene.m, scene.n, (C.c_double * 7)(*ray), depth,
                                    tape.ctypes.data_as(C.POINTER(C.c_double)), len(tape), out)
    return list(out), used


def write_color(c, spp: int):
    out = (C.c_int32 * 3)()
    lib().orc_write_color((C.c_double * 3)(*c), spp, out)
    return list(out)


def load_golden(name: str):
    z = np.load(GOLDEN / f"{name}.npz", allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    return {k: z[k] for k in ("ij", "sums", "rgb", "segments", "draws")}, meta


def golden_camera_args(meta) -> dict:
    a = meta["args"]
    kw = {"width": int(a[a.index("--width") + 1]), "spp": int(a[a.index("--spp") + 1])}
    if "--depth" in a:
        kw["depth"] = int(a[a.index("--depth") + 1])
    for flag, key in (("--aspect", "aspect"), ("--vfov", "vfov"), ("--defocus-angle", "defocus_angle")):
        if flag in a:
            kw[key] = float(a[a.index(flag) + 1])
    return kw


def golden_scene_name(meta) -> str:
    a = meta["args"]
    return a[a.index("--scene") + 1]

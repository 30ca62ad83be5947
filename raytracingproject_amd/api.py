"""Python mirror of the reference's header API (src/camera.h, hittable_list.h, bvh.h,
sphere.h, material.h), driving the MI355X renderer through the C ABI.

Same class names, constructor arguments and public camera fields as the reference, so
code written against the reference reads the same:

    world = hittable_list()
    world.add(sphere((0, -1000, 0), 1000, lambertian((0.5, 0.5, 0.5))))
    cam = camera()                      # the reference's CPUImpl::Camera slot
    cam.image_width = 400; ...
    cam.render(world)                   # PPM P3 on stdout, as camera.h:32-50

The C++ mirror (include/rt/*.h) is the drop-in for C++ callers; this module is what the
tests and bench use.  There is no CPU path here: render() and ray_color() run on the GPU.
"""
from __future__ import annotations

import sys
from typing import Sequence

import numpy as np

from . import _native as N
from . import rtweekend

Vec = Sequence[float]


# ---- materials (material.h:15-82) -------------------------------------------------
class material:
    type: int = -1


class lambertian(material):
    type = N.RT_LAMBERTIAN

    def __init__(self, albedo: Vec):
        self.albedo = tuple(float(x) for x in albedo)


class metal(material):
    type = N.RT_METAL

    def __init__(self, albedo: Vec, f: float):
        self.albedo = tuple(float(x) for x in albedo)
        self.fuzz = f if f < 1 else 1.0  # material.h:33


class dielectric(material):
    type = N.RT_DIELECTRIC

    def __init__(self, index_of_refraction: float):
        self.ir = float(index_of_refraction)


# ---- hittables (sphere.h, hittable_list.h, bvh.h) ------------------------------------
class hittable:
    pass


class sphere(hittable):
    """sphere(center, radius, mat) or sphere(center1, center2, radius, mat) (sphere.h:9-28)."""

    def __init__(self, *args):
        if len(args) == 3:
            center, radius, mat = args
            self.center1 = tuple(float(x) for x in center)
            self.center_vec = (0.0, 0.0, 0.0)
            self.is_moving = False
        elif len(args) == 4:
            c1, c2, radius, mat = args
            self.center1 = tuple(float(x) for x in c1)
            # center_vec = _center2 - _center1 (sphere.h:27)
            self.center_vec = tuple(float(b) - float(a) for a, b in zip(c1, c2))
            self.is_moving = True
        else:
            raise TypeError("sphere(center, radius, mat) or sphere(center1, center2, radius, mat)")
        self.radius = float(radius)
        self.mat = mat


class hittable_list(hittable):
    def __init__(self, obj: hittable | None = None):
        self.objects: list[hittable] = []
        if obj is not None:
            self.add(obj)

    def clear(self) -> None:
        self.objects.clear()

    def add(self, obj: hittable) -> None:
        self.objects.append(obj)


class bvh_node(hittable):
    """bvh_node(list) (bvh.h:10): the device layer always builds an SAH BVH over the
    list at upload, so this node simply wraps the list it was given."""

    def __init__(self, lst: hittable_list):
        self.list = lst


class triangle_mesh(hittable):
    """An indexed triangle mesh with one material (mesh path; the
    reference has no triangle primitive: its model loader is an empty stub,
    src/vulkan/model_loader.h:17-19).  vertices[nv, 3], faces[nt, 3] (0-based)."""

    def __init__(self, vertices, faces, mat: material):
        self.vertices = np.ascontiguousarray(vertices, dtype=np.float64).reshape(-1, 3)
        self.faces = np.ascontiguousarray(faces, dtype=np.int32).reshape(-1, 3)
        if len(self.faces) and (self.faces.min() < 0 or self.faces.max() >= len(self.vertices)):
            raise ValueError("face index out of range")
        self.mat = mat

    @classmethod
    def from_obj(cls, path, mat: material) -> "triangle_mesh":
        """Wavefront OBJ through rt_obj_load (positions + faces, fan-triangulated)."""
        V, F, _ = N.obj_load(path)
        return cls(V, F, mat)


def flatten(world: hittable) -> tuple[np.ndarray, np.ndarray]:
    """Flatten a sphere-only hittable graph into the rt_sphere / rt_material arrays of
    the C ABI (flatten_scene also returns the triangles of meshes)."""
    S, M, T = flatten_scene(world)
    if len(T):
        raise TypeError("world holds triangle meshes: use flatten_scene")
    return S, M


def flatten_scene(world: hittable) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Flatten a hittable graph into the rt_sphere / rt_material / rt_triangle arrays of
    the C ABI.  Materials shared between objects (shared_ptr in the reference) stay
    shared."""
    spheres: list[sphere] = []
    meshes: list[triangle_mesh] = []

    def walk(h: hittable) -> None:
        if isinstance(h, sphere):
            spheres.append(h)
        elif isinstance(h, triangle_mesh):
            meshes.append(h)
        elif isinstance(h, hittable_list):
            for o in h.objects:
                walk(o)
        elif isinstance(h, bvh_node):
            walk(h.list)
        else:
            raise TypeError(f"cannot flatten {type(h).__name__}")

    walk(world)
    mats: dict[int, int] = {}
    mat_objs: list[material] = []

    def mat_index(m: material) -> int:
        if id(m) not in mats:
            mats[id(m)] = len(mat_objs)
            mat_objs.append(m)
        return mats[id(m)]

    S = np.zeros(len(spheres), dtype=N.SPHERE_DTYPE)
    for k, s in enumerate(spheres):
        S[k]["center"] = s.center1
        S[k]["radius"] = s.radius
        S[k]["center_vec"] = s.center_vec
        S[k]["mat"] = mat_index(s.mat)
        S[k]["moving"] = 1 if s.is_moving else 0
    T = np.concatenate([N.triangles(m.vertices, m.faces, mat_index(m.mat)) for m in meshes]) if meshes else \
        np.zeros(0, N.TRIANGLE_DTYPE)
    M = np.zeros(len(mat_objs), dtype=N.MATERIAL_DTYPE)
    for k, m in enumerate(mat_objs):
        M[k]["type"] = m.type
        if isinstance(m, (lambertian, metal)):
            M[k]["albedo"] = m.albedo
        if isinstance(m, metal):
            M[k]["fuzz"] = m.fuzz
        if isinstance(m, dielectric):
            M[k]["ir"] = m.ir
    return S, M, T


# ---- camera (camera.h:10-126) --------------------------------------------------------
class camera:
    """Public fields of camera.h:15-26 with the same defaults."""

    def __init__(self, device: int = 0, seed: int = 0x5EED, precision: int = N.RT_PREC_F32):
        self.aspect_ratio = 1.0
        self.image_width = 100
        self.samples_per_pixel = 10
        self.max_depth = 10
        self.vfov = 90.0
        self.lookfrom = (0.0, 0.0, -1.0)
        self.lookat = (0.0, 0.0, 0.0)
        self.vup = (0.0, 1.0, 0.0)
        self.defocus_angle = 0.0
        self.focus_dist = 10.0
        self.device, self.seed, self.precision = device, seed, precision
        self._cam: N.RtCamera | None = None
        self._renderer: N.Renderer | None = None
        self._tape_renderer: N.Renderer | None = None
        self._scene_key = None

    def _desc(self) -> N.RtCameraDesc:
        d = N.RtCameraDesc()
        d.aspect_ratio = self.aspect_ratio
        d.image_width = self.image_width
        d.samples_per_pixel = self.samples_per_pixel
        d.max_depth = self.max_depth
        d.vfov = self.vfov
        d.lookfrom[:] = self.lookfrom
        d.lookat[:] = self.lookat
        d.vup[:] = self.vup
        d.defocus_angle = self.defocus_angle
        d.focus_dist = self.focus_dist
        return d

    def initialize(self) -> None:
        """camera.h:52-85 (in the library, fp64, reference operation order)."""
        self._cam = N.camera_initialize(self._desc())

    @property
    def image_height(self) -> int:
        if self._cam is None:
            self.initialize()
        return self._cam.image_height

    def image_size(self) -> tuple[int, int]:
        return self.image_width, self.image_height

    @property
    def native(self) -> N.RtCamera:
        if self._cam is None:
            self.initialize()
        return self._cam

    def _upload(self, r: N.Renderer, world: hittable) -> None:
        S, M, T = flatten_scene(world)
        r.upload_scene(S, M, T if len(T) else None)

    def render_arrays(self, world: hittable):
        """The render step without the text output: (sums, rgb, segments) on the host."""
        self.initialize()
        if self._renderer is None:
            self._renderer = N.Renderer(self.device, self.seed, self.precision)
        self._upload(self._renderer, world)
        return self._renderer.render_frame(self._cam, self.samples_per_pixel, self.max_depth)

    def render(self, world: hittable, out=None) -> None:
        """camera::render (camera.h:32-50): PPM P3 to `out` (default stdout)."""
        out = sys.stdout if out is None else out
        _, rgb, _ = self.render_arrays(world)
        write_ppm(out, rgb)

    # -- single-ray entry points of the reference API (tests.cpp:41-42) ---------------
    def get_ray(self, i: int, j: int):
        """camera.h:87-113 on the global reference stream (host, fp64)."""
        c = self.native
        du, dv = c.pixel_delta_u, c.pixel_delta_v
        pc = [(c.pixel00_loc[a] + i * du[a]) + j * dv[a] for a in range(3)]
        px = -0.5 + rtweekend.random_double()
        py = -0.5 + rtweekend.random_double()
        ps = [pc[a] + ((px * du[a]) + (py * dv[a])) for a in range(3)]
        if self.defocus_angle <= 0:
            origin = list(c.center)
        else:
            while True:  # random_in_unit_disk (vec3.h:121-127), y drawn first (g++ order)
                y = rtweekend.random_double(-1, 1)
                x = rtweekend.random_double(-1, 1)
                if x * x + y * y + 0.0 * 0.0 < 1:
                    break
            origin = [(c.center[a] + x * c.defocus_disk_u[a]) + y * c.defocus_disk_v[a] for a in range(3)]
        direction = [ps[a] - origin[a] for a in range(3)]
        time = rtweekend.random_double()
        return (*origin, *direction, time)

    def ray_color(self, r, depth: int, world: hittable):
        """camera_cpu.h:8-26 for ONE ray on the GPU (fp64), continuing the global
        reference stream: the device consumes a tape cut from a copy of the stream and
        the host stream then advances by exactly the number of uniforms used."""
        if self._tape_renderer is None:
            self._tape_renderer = N.Renderer(self.device, self.seed, N.RT_PREC_F64)
        key = id(world)
        if self._scene_key != key:
            self._upload(self._tape_renderer, world)
            self._scene_key = key
        n = 256
        while True:
            probe = rtweekend.stream().copy()
            tape = np.array([probe.canonical() for _ in range(n)], dtype=np.float64)
            col, used = self._tape_renderer.trace_tape(r, depth, tape)
            if used <= n:
                break
            n = used * 2
        for _ in range(used):
            rtweekend.random_double()
        return col


def write_ppm(out, rgb: np.ndarray) -> None:
    """PPM P3 exactly as camera.h:35 and color.h:32-34 print it."""
    H, W, _ = rgb.shape
    out.write(f"P3\n{W} {H}\n255\n")
    flat = rgb.reshape(-1, 3)
    out.write("".join(f"{r} {g} {b}\n" for r, g, b in flat.tolist()))

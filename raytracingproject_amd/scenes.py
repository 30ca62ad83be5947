"""Scene construction as the reference does it (host side).

random_spheres() is src/main.cpp:12-53 on the reference's own mt19937 stream, with the
g++ argument-evaluation order the committed image.ppm encodes (right to left: in
point3(a + 0.9*rd(), 0.2, b + 0.9*rd()) the z coordinate takes the first draw).  It
yields the same 485 spheres as the reference binary bit for bit (tests/golden/
scene_random.txt, dumped from the reference itself).
"""
from __future__ import annotations

import math

from .api import camera, dielectric, hittable_list, lambertian, metal, sphere, triangle_mesh
from .rtweekend import random_double


def _random_vec(lo=None, hi=None):
    # vec3::random() / vec3::random(min,max) (vec3.h:63-69): right-to-left arguments
    z = random_double(lo, hi)
    y = random_double(lo, hi)
    x = random_double(lo, hi)
    return (x, y, z)


def random_spheres() -> hittable_list:
    """main.cpp:12-53.  Consumes exactly 4471 draws of the global stream."""
    world = hittable_list()
    ground = lambertian((0.5, 0.5, 0.5))
    world.add(sphere((0, -1000, 0), 1000, ground))
    for a in range(-11, 11):
        for b in range(-11, 11):
            choose_mat = random_double()
            cz = b + 0.9 * random_double()
            cx = a + 0.9 * random_double()
            center = (float(cx), 0.2, float(cz))
            d = (center[0] - 4, center[1] - 0.2, center[2] - 0)
            if math.sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]) > 0.9:
                if choose_mat < 0.8:
                    rhs = _random_vec()          # color::random() * color::random(): right operand first
                    lhs = _random_vec()
                    albedo = (lhs[0] * rhs[0], lhs[1] * rhs[1], lhs[2] * rhs[2])
                    dy = random_double(0, .5)
                    center2 = (center[0] + 0, center[1] + dy, center[2] + 0)
                    world.add(sphere(center, center2, 0.2, lambertian(albedo)))
                elif choose_mat < 0.95:
                    albedo = _random_vec(0.5, 1)
                    fuzz = random_double(0, 0.5)
                    world.add(sphere(center, 0.2, metal(albedo, fuzz)))
                else:
                    world.add(sphere(center, 0.2, dielectric(1.5)))
    world.add(sphere((0, 1, 0), 1.0, dielectric(1.5)))
    world.add(sphere((-4, 1, 0), 1.0, lambertian((0.4, 0.2, 0.1))))
    world.add(sphere((4, 1, 0), 1.0, metal((0.7, 0.6, 0.5), 0.0)))
    return world


def four_spheres() -> hittable_list:
    """Config 1 (BASELINE.json): the ground (main.cpp:14-15) + the three big spheres
    (main.cpp:46-53)."""
    world = hittable_list()
    world.add(sphere((0, -1000, 0), 1000, lambertian((0.5, 0.5, 0.5))))
    world.add(sphere((0, 1, 0), 1.0, dielectric(1.5)))
    world.add(sphere((-4, 1, 0), 1.0, lambertian((0.4, 0.2, 0.1))))
    world.add(sphere((4, 1, 0), 1.0, metal((0.7, 0.6, 0.5), 0.0)))
    return world


def ground_only() -> hittable_list:
    """tests/tests.cpp:26-29."""
    world = hittable_list()
    world.add(sphere((0, -1000, 0), 1000, lambertian((0.5, 0.5, 0.5))))
    return world


# ---- mesh configs (BASELINE.json configs 4/5; SURVEY.md §8(d): procedural mesh, since
# assets/models holds no .obj).  Both read the mesh back through an OBJ file when given
# one (rt_obj_load), else use meshgen's arrays directly (identical vertices: write_obj
# prints repr() doubles, which strtod reads back exactly).
MESH_LEVEL = 7   # 327,680 triangles


def mesh_only(level: int = MESH_LEVEL, obj_path=None) -> hittable_list:
    """Config 4: the ground (main.cpp:14-15) and a displaced icosphere ("blob") of
    20 * 4^level triangles where main.cpp puts its glass sphere, lambertian like
    main.cpp's material2."""
    from . import meshgen
    world = hittable_list()
    world.add(sphere((0, -1000, 0), 1000, lambertian((0.5, 0.5, 0.5))))
    mat = lambertian((0.4, 0.2, 0.1))
    if obj_path is not None:
        world.add(triangle_mesh.from_obj(obj_path, mat))
    else:
        V, F = meshgen.blob(level, radius=1.6, center=(0.0, 1.0, 0.0))
        world.add(triangle_mesh(V, F, mat))
    return world


def mixed(level: int = MESH_LEVEL, obj_path=None) -> hittable_list:
    """Config 5: the reference's 485 random spheres plus a metal blob between the big
    spheres and the camera (meshgen.MESH_CENTER)."""
    from . import meshgen
    world = random_spheres()
    mat = metal((0.7, 0.6, 0.5), 0.05)
    if obj_path is not None:
        world.add(triangle_mesh.from_obj(obj_path, mat))
    else:
        V, F = meshgen.blob(level, radius=meshgen.MESH_RADIUS, center=meshgen.MESH_CENTER)
        world.add(triangle_mesh(V, F, mat))
    return world


def main_camera(cam: camera | None = None, **kw) -> camera:
    """The camera of main.cpp:55-68 (also tests.cpp:12-23)."""
    cam = cam or camera(**kw)
    cam.aspect_ratio = 16.0 / 9.0
    cam.image_width = 400
    cam.samples_per_pixel = 30
    cam.max_depth = 50
    cam.vfov = 20
    cam.lookfrom = (13, 2, 3)
    cam.lookat = (0, 0, 0)
    cam.vup = (0, 1, 0)
    cam.defocus_angle = 0.6
    cam.focus_dist = 10.0
    return cam

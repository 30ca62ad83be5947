"""Deterministic procedural meshes for the mesh configs (BASELINE.json configs 4/5).

The reference ships no .obj (assets/models holds only viking_room.png),
so the mesh workloads use a generated one: a subdivided icosphere with a smooth radial
displacement ("blob"), written as OBJ and read back through rt_obj_load like any model.
Level L has 20 * 4^L triangles (L=7: 327,680; L=8: 1,310,720).
"""
from __future__ import annotations

import math

import numpy as np


def icosphere(level: int) -> tuple[np.ndarray, np.ndarray]:
    t = (1.0 + math.sqrt(5.0)) / 2.0
    v = [(-1, t, 0), (1, t, 0), (-1, -t, 0), (1, -t, 0), (0, -1, t), (0, 1, t), (0, -1, -t), (0, 1, -t),
         (t, 0, -1), (t, 0, 1), (-t, 0, -1), (-t, 0, 1)]
    f = [(0, 11, 5), (0, 5, 1), (0, 1, 7), (0, 7, 10), (0, 10, 11), (1, 5, 9), (5, 11, 4), (11, 10, 2), (10, 7, 6),
         (7, 1, 8), (3, 9, 4), (3, 4, 2), (3, 2, 6), (3, 6, 8), (3, 8, 9), (4, 9, 5), (2, 4, 11), (6, 2, 10),
         (8, 6, 7), (9, 8, 1)]
    verts = [np.array(p, dtype=np.float64) / np.linalg.norm(p) for p in v]
    faces = np.array(f, dtype=np.int64)
    V = np.array(verts)
    for _ in range(level):
        # split every edge once (shared midpoints), 1 triangle -> 4
        e = np.concatenate([faces[:, [0, 1]], faces[:, [1, 2]], faces[:, [2, 0]]])
        e.sort(axis=1)
        uniq, inv = np.unique(e, axis=0, return_inverse=True)
        inv = inv.reshape(3, -1)
        mid = V[uniq[:, 0]] + V[uniq[:, 1]]
        mid /= np.linalg.norm(mid, axis=1, keepdims=True)
        base = len(V)
        V = np.concatenate([V, mid])
        a, b, c = faces[:, 0], faces[:, 1], faces[:, 2]
        ab, bc, ca = base + inv[0], base + inv[1], base + inv[2]
        faces = np.concatenate([np.stack([a, ab, ca], 1), np.stack([b, bc, ab], 1), np.stack([c, ca, bc], 1),
                                np.stack([ab, bc, ca], 1)])
    return V, faces


def blob(level: int, radius: float = 1.0, center=(0.0, 0.0, 0.0), amp: float = 0.18) -> tuple[np.ndarray, np.ndarray]:
    """Icosphere with a smooth deterministic bump field on the radius."""
    V, F = icosphere(level)
    x, y, z = V[:, 0], V[:, 1], V[:, 2]
    bump = (np.sin(5.0 * x + 1.3) * np.cos(4.0 * y - 0.7) + 0.6 * np.sin(7.0 * z + 2.1 * x)) / 1.6
    r = radius * (1.0 + amp * bump)
    return V * r[:, None] + np.asarray(center, dtype=np.float64), F


def write_obj(path, V: np.ndarray, F: np.ndarray) -> None:
    with open(path, "w") as f:
        f.write(f"# procedural mesh: {len(V)} vertices, {len(F)} triangles\n")
        f.write("".join(f"v {a!r} {b!r} {c!r}\n" for a, b, c in V.tolist()))
        f.write("".join(f"f {a + 1} {b + 1} {c + 1}\n" for a, b, c in F.tolist()))


# The mesh workloads: a blob standing in the random-spheres scene, in view of main.cpp's
# camera (lookfrom (13,2,3) -> (0,0,0)), between the glass and the metal big spheres.
MESH_CENTER = (2.0, 1.15, 2.2)
MESH_RADIUS = 1.0

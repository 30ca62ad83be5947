import sys
sys.path.insert(0, "/root/repo")
import numpy as np
from raytracingproject_amd import _native as N
from raytracingproject_amd import api, scenes, rtweekend
S, M = api.flatten(scenes.ground_only())
V = np.array([[0, 1, 0], [1, 1, 0], [0, 2, 0], [3, 1, 0], [4, 1, 0], [3, 2, 0]], dtype=np.float64)
F = np.array([[0, 1, 2], [3, 4, 5]], dtype=np.int32)
M2 = np.concatenate([M, M[:1]])
T = N.triangles(V, F, len(M))
c = V[F].mean(axis=1)[0]
rays = np.array([[*(c + [0, 0, 5]), 0, 0, -1, 0],        # x, y zero
                 [*(c + [0, 0, 5]), 0.01, 0, -1, 0],     # y zero
                 [*(c + [0, 0, 5]), 0, 0.01, -1, 0],     # x zero
                 [*(c + [0, 0, 5]), 0.01, 0.01, -1, 0],
                 [*(c + [0, 0, 5]), -0.0, -0.0, -1, 0]])
with N.Renderer(0, 0x5EED, N.RT_PREC_F32) as r:
    r.upload_scene(S, M2, T)
    h = r.trace_rays_host(rays)
    print("mesh f32", h["id"].tolist(), h["t"].tolist())
    r.set_tuning(mesh_lds_nodes=0)
    r.upload_scene(S, M2, T)
    h = r.trace_rays_host(rays)
    print("mesh f32 no LDS top", h["id"].tolist(), h["t"].tolist())
rtweekend.reset_stream()
S, M = api.flatten(scenes.random_spheres())
g = np.random.default_rng(3)
o = g.uniform([-11, 0.3, -11], [11, 2, 11], (4000, 3))
axes = np.eye(3)[g.integers(0, 3, 4000)] * g.choice([-1, 1], (4000, 1))
rays = np.concatenate([o, axes, g.uniform(0, 1, (4000, 1))], axis=1)
out = {}
for prec in (N.RT_PREC_F64, N.RT_PREC_F32):
    with N.Renderer(0, 0x5EED, prec) as r:
        r.upload_scene(S, M)
        out[prec] = r.trace_rays_host(rays)
print("spheres axis-aligned: same id", float((out[0]["id"] == out[1]["id"]).mean()),
      "f32 miss where f64 hit", int(((out[0]["id"] == -1) & (out[1]["id"] >= 0)).sum()),
      "f64 hits", int((out[1]["id"] >= 0).sum()))

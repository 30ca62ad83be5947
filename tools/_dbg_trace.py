import sys
sys.path.insert(0, "/root/repo")
import numpy as np
from raytracingproject_amd import _native as N
from raytracingproject_amd import api, scenes
S, M = api.flatten(scenes.ground_only())
V = np.array([[0, 1, 0], [1, 1, 0], [0, 2, 0], [3, 1, 0], [4, 1, 0], [3, 2, 0]], dtype=np.float64)
F = np.array([[0, 1, 2], [3, 4, 5]], dtype=np.int32)
M2 = np.concatenate([M, M[:1]])
T = N.triangles(V, F, len(M))
cent = V[F].mean(axis=1)
rays = np.concatenate([cent + [0, 0, 5], np.tile([0, 0, -1.0], (2, 1)), np.zeros((2, 1))], axis=1)
rays = np.concatenate([rays, [[0, 5, 0, 0, 1, 0, 0.5]], [[0.3, 1.3, 5, 0.01, 0.02, -1, 0]]])
for builder in (N.RT_MESH_BUILD_HOST, N.RT_MESH_BUILD_GPU):
    for prec in (N.RT_PREC_F64, N.RT_PREC_F32):
        with N.Renderer(0, 0x5EED, prec) as r:
            r.set_tuning(mesh_builder=builder)
            r.upload_scene(S, M2, T)
            info = r.scene_info()
            h = r.trace_rays_host(rays)
            print(builder, prec, info.num_triangles, info.mesh_nodes, info.mesh_depth, h["id"].tolist(), h["t"].tolist())

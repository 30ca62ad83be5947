#!/usr/bin/env python3
"""Time the mesh kernel over triangle-BVH build and traversal knobs (rt_tuning mesh_*).

python tools/mesh_sweep.py [--scene mesh|mixed] [--spp 16] [--reps 3]
One JSON line per setting: kernel ms (min over reps) and Mrays/s at 1920x1080.
"""
import argparse
import itertools
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from raytracingproject_amd import _native as N  # noqa: E402
from raytracingproject_amd import api, rtweekend, scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", choices=["mesh", "mixed"], default="mesh")
    ap.add_argument("--level", type=int, default=scenes.MESH_LEVEL)
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--leaf", default="1,2,4,8")
    ap.add_argument("--cost", default="0.5,1,2")
    ap.add_argument("--lds", default="0,256,512")
    ap.add_argument("--block", default="512")
    ap.add_argument("--wpe", default="0")
    ap.add_argument("--mstack", default="16", help="mesh_lds_stack values (LDS stack entries per lane)")
    a = ap.parse_args()
    import torch
    rtweekend.reset_stream()
    world = scenes.mesh_only(a.level) if a.scene == "mesh" else scenes.mixed(a.level)
    S, M, T = api.flatten_scene(world)
    cam_api = scenes.main_camera()
    cam_api.image_width, cam_api.samples_per_pixel = 1920, a.spp
    cam = cam_api.native
    lay = N.shard_layout(cam.image_width, cam.image_height, 0, 1)
    out = torch.empty(lay.max_shard_tiles * 64 * 3, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    r = N.Renderer(0, 0x5EED, N.RT_PREC_F32)
    rays = cam.image_width * cam.image_height * a.spp
    for leaf, cost in itertools.product([int(x) for x in a.leaf.split(",")], [float(x) for x in a.cost.split(",")]):
        r.set_tuning(mesh_max_leaf=leaf, mesh_cost_traverse=cost, mesh_lds_nodes=0)
        r.upload_scene(S, M, T)
        info = r.scene_info()
        for lds, block, wpe, mst in itertools.product([int(x) for x in a.lds.split(",")],
                                                      [int(x) for x in a.block.split(",")],
                                                      [int(x) for x in a.wpe.split(",")],
                                                      [int(x) for x in a.mstack.split(",")]):
            try:
                r.set_tuning(mesh_lds_nodes=lds, mesh_block=block, mesh_waves_per_eu=wpe, mesh_lds_stack=mst)
            except N.RtError as e:
                print(json.dumps({"leaf": leaf, "cost": cost, "lds": lds, "block": block, "error": str(e)}))
                continue
            try:
                r.render(cam, a.spp, 50, 0, 1, out.data_ptr())
            except N.RtError as e:
                print(json.dumps({"leaf": leaf, "cost": cost, "lds": lds, "block": block, "wpe": wpe, "error": str(e)}))
                continue
            ms = []
            for _ in range(a.reps):
                r.render(cam, a.spp, 50, 0, 1, out.data_ptr())
                ms.append(r.last_kernel_ms())
            print(json.dumps({"scene": a.scene, "leaf": leaf, "cost": cost, "lds": lds, "block": block, "wpe": wpe,
                              "mstack": mst, "lds_bytes": r.scene_info().lds_bytes, "nodes": info.mesh_nodes, "depth": info.mesh_depth, "leaves": info.mesh_leaves,
                              "ms": round(min(ms), 3), "mrays": round(rays / min(ms) / 1e3, 1)}), flush=True)
    r.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Tuning sweep on one GPU: workgroup size x BVH shape -> render-kernel time.

python tools/sweep.py [--width 1920 --spp 64] ; prints one JSON line per config.
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
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--blocks", default="1024")
    ap.add_argument("--leaves", default="4,6,8")
    ap.add_argument("--costs", default="0.25,0.5")
    ap.add_argument("--wpe", default="8")
    ap.add_argument("--trav", default="600")
    a = ap.parse_args()
    import torch
    rtweekend.reset_stream()
    S, M = api.flatten(scenes.random_spheres())
    cam_api = scenes.main_camera()
    cam_api.image_width, cam_api.samples_per_pixel = a.width, a.spp
    cam = cam_api.native
    W, H = cam.image_width, cam.image_height
    r = N.Renderer(0, 0x5EED, N.RT_PREC_F32)
    lay = N.shard_layout(W, H, 0, 1)
    out = torch.empty(lay.max_shard_tiles * 64 * 3, dtype=torch.float32, device="cuda")
    segs = torch.empty(lay.max_shard_tiles * 64, dtype=torch.int32, device="cuda")
    best = None
    first = {}
    for block, leaf, cost, wpe, trav in itertools.product(
            map(int, a.blocks.split(",")), map(int, a.leaves.split(",")), map(float, a.costs.split(",")),
            map(int, a.wpe.split(",")), map(int, a.trav.split(","))):
        try:
            r.set_tuning(block=block, max_leaf=leaf, cost_intersect=cost, cost_traverse=1.0, waves_per_eu=wpe,
                         traversal=trav)
            r.upload_scene(S, M)
        except N.RtError as e:
            continue
        info = r.scene_info()
        times = []
        try:
            for _ in range(a.reps + 1):
                r.render(cam, a.spp, 50, 0, 1, out.data_ptr(), segs.data_ptr())
                times.append(r.last_kernel_ms())
        except N.RtError as e:
            print(json.dumps({"block": block, "wpe": wpe, "trav": trav, "error": str(e)}))
            continue
        ms = min(times[1:])
        torch.cuda.synchronize()
        key = (leaf, cost)   # same BVH: frames of different kernel variants (fp32 rounding may differ)
        same = None
        if key in first:
            same = bool(torch.equal(first[key], out))
        else:
            first[key] = out.clone()
        rays = W * H * a.spp
        rec = {"block": block, "max_leaf": leaf, "cost_intersect": cost, "wpe": wpe, "trav": trav,
               "same": same, "ms": round(ms, 3),
               "mrays": round(rays / ms / 1e3, 1), "nodes": info.bvh_nodes, "depth": info.bvh_depth,
               "lds": info.lds_bytes, "segs_per_primary": round(float(segs.to(torch.int64).sum()) / rays, 4)}
        print(json.dumps(rec), flush=True)
        if best is None or ms < best["ms"]:
            best = rec
    print("BEST", json.dumps(best))


if __name__ == "__main__":
    main()

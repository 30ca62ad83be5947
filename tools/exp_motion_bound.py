#!/usr/bin/env python3
"""Upper bound on what motion-aware culling could buy: render-kernel time of the
random-spheres scene as is, with its 389 moving spheres frozen at their mid-motion
centres (boxes shrink to the static sphere), and frozen at t = 0.

python tools/exp_motion_bound.py [--width 1920 --spp 64]; one JSON line per variant.
"""
import argparse
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
    a = ap.parse_args()
    import torch
    rtweekend.reset_stream()
    S, M = api.flatten(scenes.random_spheres())
    mid = S.copy()
    mid["center"] = mid["center"] + 0.5 * mid["center_vec"]
    mid["center_vec"] = 0
    mid["moving"] = 0
    t0 = S.copy()
    t0["center_vec"] = 0
    t0["moving"] = 0
    cam_api = scenes.main_camera()
    cam_api.image_width, cam_api.samples_per_pixel = a.width, a.spp
    cam = cam_api.native
    W, H = cam.image_width, cam.image_height
    r = N.Renderer(0, 0x5EED, N.RT_PREC_F32)
    lay = N.shard_layout(W, H, 0, 1)
    out = torch.empty(lay.max_shard_tiles * 64 * 3, dtype=torch.float32, device="cuda")
    segs = torch.empty(lay.max_shard_tiles * 64, dtype=torch.int32, device="cuda")
    for block in map(int, a.blocks.split(",")):
        for name, SS in (("moving", S), ("static_mid", mid), ("static_t0", t0)):
            try:
                r.set_tuning(block=block)
                r.upload_scene(SS, M)
            except N.RtError as e:
                print(json.dumps({"block": block, "scene": name, "error": str(e)}))
                continue
            times = []
            for _ in range(a.reps + 1):
                r.render(cam, a.spp, 50, 0, 1, out.data_ptr(), segs.data_ptr())
                times.append(r.last_kernel_ms())
            ms = min(times[1:])
            info = r.scene_info()
            rays = W * H * a.spp
            print(json.dumps({"block": block, "scene": name, "ms": round(ms, 3), "mrays": round(rays / ms / 1e3, 1),
                              "nodes": info.bvh_nodes, "lds": info.lds_bytes,
                              "segs_per_primary": round(float(segs.to(torch.int64).sum()) / rays, 4)}), flush=True)


if __name__ == "__main__":
    main()

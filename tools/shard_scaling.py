#!/usr/bin/env python3
"""Predict multi-GPU strong scaling from one GPU: kernel time of shard r of N (the work one
rank does at N GPUs) for N = 1, 2, 4, 8, against the 1-GPU frame.

python tools/shard_scaling.py [--width 1920 --spp 256] [--scene random|mesh|mixed]
efficiency(N) = t(1) / (N * max_r t(shard r of N)); the RCCL gather adds ~3 MB per rank.
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
    ap.add_argument("--scene", choices=["random", "mesh", "mixed"], default="random",
                    help="mesh / mixed: BASELINE configs 4 / 5 geometry (meshgen blob, level 7)")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--block", type=int, default=0, help="0: the library's default")
    ap.add_argument("--chunk-waves", type=int, default=None, help="rt_tuning.chunk_waves (default: library's)")
    ap.add_argument("--tune", default="", help="more rt_tuning overrides, k=v,k=v")
    a = ap.parse_args()
    import torch
    rtweekend.reset_stream()
    if a.scene == "random":
        S, M = api.flatten(scenes.random_spheres())
        T = None
    else:
        world = scenes.mesh_only() if a.scene == "mesh" else scenes.mixed()
        S, M, T = api.flatten_scene(world)
    cam_api = scenes.main_camera()
    cam_api.image_width, cam_api.samples_per_pixel = a.width, a.spp
    cam = cam_api.native
    W, H = cam.image_width, cam.image_height
    r = N.Renderer(0, 0x5EED, N.RT_PREC_F32)
    if a.block:
        r.set_tuning(block=a.block)
    if a.chunk_waves is not None:
        r.set_tuning(chunk_waves=a.chunk_waves)
    over = {k: (float(v) if "." in v else int(v)) for k, v in (kv.split("=") for kv in filter(None, a.tune.split(",")))}
    if over:
        r.set_tuning(**over)
    r.upload_scene(S, M, T)
    full = N.shard_layout(W, H, 0, 1)
    out = torch.empty(full.max_shard_tiles * 64 * 3, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    t1 = None
    for n in map(int, a.ns.split(",")):
        worst = 0.0
        for shard in sorted({0, n - 1}):
            ms = []
            for _ in range(a.reps):
                r.render(cam, a.spp, 50, shard, n, out.data_ptr())
                ms.append(r.last_kernel_ms())
            worst = max(worst, min(ms))
        if n == 1:
            t1 = worst
        lay = N.shard_layout(W, H, 0, n)
        print(json.dumps({"scene": a.scene, "width": W, "spp": a.spp, "n": n, "block": r.tuning().block, "chunk_waves": r.tuning().chunk_waves, **over, "shard_tiles": lay.max_shard_tiles, "kernel_ms": round(worst, 3),
                          "efficiency": round(t1 / (n * worst), 3), "speedup": round(t1 / worst, 2)}), flush=True)
    r.close()


if __name__ == "__main__":
    main()

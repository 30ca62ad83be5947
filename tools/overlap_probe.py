#!/usr/bin/env python3
"""Consecutive frames on one stream vs alternating streams: does overlapping frame k's
drain (the persistent kernel's tail, when waves finish their last paths) with frame k+1's
start pay, for the whole frame and for shard 0 of N (one rank's work at N GPUs)?

python tools/overlap_probe.py [--frames 8] [--ns 1,8]
Each line: N, streams, ms per frame (wall, K frames back to back), and the frames'
8-bit agreement with the first stream layout (the frames are independent).
"""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from raytracingproject_amd import _native as N  # noqa: E402
from raytracingproject_amd import api, rtweekend, scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--ns", default="1,8")
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch
    rtweekend.reset_stream()
    S, M = api.flatten(scenes.random_spheres())
    cam_api = scenes.main_camera()
    cam_api.image_width, cam_api.samples_per_pixel = a.width, a.spp
    cam = cam_api.native
    W, H = cam.image_width, cam.image_height
    r = N.Renderer(0, 0x5EED, N.RT_PREC_F32)
    r.upload_scene(S, M)
    for n in map(int, a.ns.split(",")):
        lay = N.shard_layout(W, H, 0, n)
        bufs = [torch.empty(lay.max_shard_tiles * 64 * 3, dtype=torch.float32, device="cuda") for _ in range(2)]
        streams = [torch.cuda.Stream() for _ in range(2)]
        ref = None
        for nstreams in (1, 2, 1, 2):
            best = None
            for _ in range(a.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for k in range(a.frames):
                    s = streams[k % nstreams]
                    r.render(cam, a.spp, 50, 0, n, bufs[k % 2].data_ptr(), None, s.cuda_stream)
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) * 1e3 / a.frames
                best = ms if best is None else min(best, ms)
            out = bufs[(a.frames - 1) % 2].cpu()
            same = None if ref is None else bool(torch.equal(out, ref))
            if ref is None:
                ref = out
            print(json.dumps({"n": n, "streams": nstreams, "frames": a.frames, "ms_per_frame": round(best, 3),
                              "identical_to_first": same}), flush=True)
    r.close()


if __name__ == "__main__":
    main()

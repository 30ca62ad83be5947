#!/usr/bin/env python3
"""Frames in flight: K back-to-back frames of one shard (shard 0 of N) on one stream
versus alternating over F streams with F output buffers, so that the next frame's
workgroups fill the CUs while the previous frame's last paths finish.

python tools/pipeline_probe.py [--ns 1,8] [--frames 12] [--inflight 1,2,3]
Prints one JSON line per (N, F): wall ms per frame over the K frames (one sync at the end).
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
    ap.add_argument("--ns", default="1,8")
    ap.add_argument("--frames", type=int, default=12)
    ap.add_argument("--inflight", default="1,2,3")
    ap.add_argument("--spp", type=int, default=256)
    a = ap.parse_args()
    import torch
    rtweekend.reset_stream()
    S, M = api.flatten(scenes.random_spheres())
    cam_api = scenes.main_camera()
    cam_api.image_width, cam_api.samples_per_pixel = 1920, a.spp
    cam = cam_api.native
    r = N.Renderer(0, 0x5EED, N.RT_PREC_F32)
    r.upload_scene(S, M)
    for n in map(int, a.ns.split(",")):
        lay = N.shard_layout(cam.image_width, cam.image_height, 0, n)
        for f in map(int, a.inflight.split(",")):
            streams = [torch.cuda.Stream() for _ in range(f)]
            bufs = [torch.empty(lay.max_shard_tiles * 64 * 3, dtype=torch.float32, device="cuda") for _ in range(f)]
            for k in range(2 * f):   # warm-up: every buffer's accumulator slot exists
                r.render(cam, a.spp, 50, 0, n, bufs[k % f].data_ptr(), None, streams[k % f].cuda_stream)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(a.frames):
                r.render(cam, a.spp, 50, 0, n, bufs[k % f].data_ptr(), None, streams[k % f].cuda_stream)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / a.frames * 1e3
            print(json.dumps({"n": n, "frames_in_flight": f, "frames": a.frames, "ms_per_frame": round(ms, 3),
                              "gpu_mrays": round(lay.shard_tiles * 64 * a.spp / ms / 1e3, 1)}), flush=True)
    r.close()


if __name__ == "__main__":
    main()

"""Progressive rendering with snapshots: the role of the reference's
Vulkan frame loop (src/vulkan/graphical_environment_vulkan.cpp:208-225), rebuilt as HIP
accumulation plus a file dump.

Samples are added to the running per-pixel sums in batches (rt_render_range with
accumulate), so the frame after every batch is the frame of that many samples, and the
last one is bit-identical to a single launch of all samples.  After each batch the sums
are un-interleaved and quantised on the device (write_color, color.h:14-35) and the 8-bit
image is written as PPM.

    python -m raytracingproject_amd.progressive --scene random --width 400 --spp 64 \\
        --every 8 --out frames/frame_%03d.ppm
"""
from __future__ import annotations

import argparse
import time
from pathlib import Path

import numpy as np

from . import _native as N
from . import api, ppm, rtweekend, scenes


def world_for(name: str, mesh_level: int):
    if name == "random":
        rtweekend.reset_stream()
        return scenes.random_spheres()
    if name == "four":
        return scenes.four_spheres()
    if name == "mesh":
        return scenes.mesh_only(mesh_level)
    if name == "mixed":
        rtweekend.reset_stream()
        return scenes.mixed(mesh_level)
    raise ValueError(name)


def render_progressive(world, cam_api, spp: int, every: int, out_pattern: str | None = None, binary: bool = True,
                       device: int = 0, seed: int = 0x5EED, precision: int = N.RT_PREC_F32, callback=None,
                       callback_sums: bool = False):
    """Render `spp` samples in batches of `every`; after each batch quantise and (if
    `out_pattern` is set) write `out_pattern % batch_index` as P6 (or P3); then
    `callback(batch_index, samples_so_far, image)` if given -- or, with
    `callback_sums=True` (r06), `callback(batch_index, samples_so_far, image, sums)` with
    the snapshot's fp per-pixel sums [H, W, 3].  Returns the final int32 [H, W, 3] image
    and the fp sums [H, W, 3]."""
    import torch
    cam_api.samples_per_pixel = spp
    cam = cam_api.native
    W, H, depth = cam.image_width, cam.image_height, cam_api.max_depth
    S, M, T = api.flatten_scene(world)
    r = N.Renderer(device, seed, precision)
    try:
        r.upload_scene(S, M, T if len(T) else None)
        lay = N.shard_layout(W, H, 0, 1)
        dt = torch.float64 if precision == N.RT_PREC_F64 else torch.float32
        dev = torch.device("cuda", device)
        sums = torch.zeros(lay.max_shard_tiles * 64 * 3, dtype=dt, device=dev)
        frame = torch.empty(W * H * 3, dtype=dt, device=dev)
        rgb = torch.empty(W * H * 3, dtype=torch.int32, device=dev)
        torch.cuda.synchronize(dev)
        done, k = 0, 0
        while done < spp:
            n = min(every, spp - done)
            r.render_range(cam, done, n, depth, 0, 1, done > 0, sums.data_ptr())
            done += n
            r.unshard(sums.data_ptr(), W, H, 1, frame.data_ptr())
            r.quantize(frame.data_ptr(), W, H, done, rgb.data_ptr())
            torch.cuda.synchronize(dev)
            img = rgb.cpu().numpy().reshape(H, W, 3)
            fsum = frame.cpu().numpy().reshape(H, W, 3)
            if out_pattern:
                path = Path(out_pattern % k)
                path.parent.mkdir(parents=True, exist_ok=True)
                (ppm.write_p6 if binary else ppm.write_p3)(path, img)
            if callback:
                if callback_sums:
                    callback(k, done, img, fsum)
                else:
                    callback(k, done, img)
            k += 1
        return img, fsum
    finally:
        r.close()


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--scene", choices=["random", "four", "mesh", "mixed"], default="random")
    ap.add_argument("--mesh-level", type=int, default=scenes.MESH_LEVEL)
    ap.add_argument("--width", type=int, default=400)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--every", type=int, default=8)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--out", default="frames/frame_%03d.ppm")
    ap.add_argument("--p3", action="store_true", help="text PPM (the reference's format) instead of P6")
    a = ap.parse_args()
    cam = scenes.main_camera()
    cam.image_width, cam.max_depth = a.width, a.depth
    t0 = time.perf_counter()
    render_progressive(world_for(a.scene, a.mesh_level), cam, a.spp, a.every, a.out, binary=not a.p3,
                       callback=lambda k, n, img: print(f"snapshot {k}: {n} samples, mean {img.mean():.2f}",
                                                     flush=True))
    print(f"done in {time.perf_counter() - t0:.2f} s")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

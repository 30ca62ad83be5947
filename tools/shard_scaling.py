#!/usr/bin/env python3
"""Predict multi-GPU strong scaling from one GPU: kernel time of shard r of N (the work one
rank does at N GPUs) for N = 1, 2, 4, 8, against the 1-GPU frame.

python tools/shard_scaling.py [--width 1920 --spp 256] [--scene random|mesh|mixed] [--step]
efficiency(N) = t(1) / (N * max_r t(shard r of N)); the RCCL gather adds ~3 MB per rank.

--step (r06): also time, on this one GPU, what rank 0 does per bench.py step
at N besides its own shard -- the gather's destination writes (N shard buffers written into
the stacked buffer: a device copy of N x shard bytes), rt_finish_frame_u8 over the N-shard
buffer (unshard + quantise) and the pinned device-to-host copy of the 8-bit frame -- and
predict the step: kernel(max shard) + gather write + xGMI transfer + finish_u8, the host copy
overlapping the next frame's render (bench.py's two frames in flight) unless it is longer.
The xGMI transfer is not measurable on one GPU: it is modelled as one shard over one link at
--xgmi-gbs (each peer sends over its own link to rank 0) plus --rccl-us of launch latency.
"""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from raytracingproject_amd import _native as N  # noqa: E402
from raytracingproject_amd import api, rtweekend, scenes  # noqa: E402


def step_model(r, torch, W, H, spp, n, lay, kernel_ms, t1, reps, xgmi_gbs, rccl_us):
    """Rank 0's per-step work at N = n beside its shard's kernel, timed on this GPU."""
    shard_elems = lay.max_shard_tiles * 64 * 3
    shard = torch.rand(shard_elems, dtype=torch.float32, device="cuda")
    gathered = torch.empty(n * shard_elems, dtype=torch.float32, device="cuda")
    rgb8 = torch.empty(W * H * 3, dtype=torch.uint8, device="cuda")
    host8 = torch.empty(W * H * 3, dtype=torch.uint8, pin_memory=True)

    def timed(fn):
        best = float("inf")
        for _ in range(max(reps, 3)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1))
        return best

    def dest_writes():   # what the gather writes into rank 0's stacked buffer
        for k in range(n):
            gathered[k * shard_elems:(k + 1) * shard_elems].copy_(shard)

    stream = torch.cuda.current_stream().cuda_stream
    g_ms = timed(dest_writes)
    f_ms = timed(lambda: r.finish_u8(gathered.data_ptr(), W, H, n, spp, rgb8.data_ptr(), stream))
    c_ms = timed(lambda: host8.copy_(rgb8, non_blocking=True))
    x_ms = 0.0 if n == 1 else shard_elems * 4 / (xgmi_gbs * 1e9) * 1e3 + rccl_us * 1e-3
    dev_ms = kernel_ms + (g_ms + x_ms if n > 1 else 0.0) + f_ms
    step_ms = max(dev_ms, c_ms)
    mrays = W * H * spp / (step_ms * 1e-3) / 1e6
    return {"gather_dest_write_ms": round(g_ms, 4), "xgmi_model_ms": round(x_ms, 4), "finish_u8_ms": round(f_ms, 4),
            "host_copy_ms": round(c_ms, 4), "step_ms_pred": round(step_ms, 3), "mrays_pred": round(mrays, 1),
            "kernel_only_speedup": round(t1 / kernel_ms, 2), "_t1": t1}


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
    ap.add_argument("--step", action="store_true", help="rank 0's per-step work beside the kernel (r06)")
    ap.add_argument("--xgmi-gbs", type=float, default=50.0,
                    help="--step: assumed one-direction xGMI link rate for the gather (GB/s)")
    ap.add_argument("--rccl-us", type=float, default=30.0, help="--step: assumed RCCL gather latency (us)")
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
    t1 = step1 = None
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
        row = {"scene": a.scene, "width": W, "spp": a.spp, "n": n, "block": r.tuning().block,
               "chunk_waves": r.tuning().chunk_waves, **over, "shard_tiles": lay.max_shard_tiles,
               "kernel_ms": round(worst, 3), "efficiency": round(t1 / (n * worst), 3), "speedup": round(t1 / worst, 2)}
        if a.step:
            row.update(step_model(r, torch, W, H, a.spp, n, lay, worst, t1, a.reps, a.xgmi_gbs, a.rccl_us))
            row.pop("_t1")
            if n == 1:
                step1 = row["step_ms_pred"]
            row["step_speedup_pred"] = round(step1 / row["step_ms_pred"], 2)
        print(json.dumps(row), flush=True)
    r.close()


if __name__ == "__main__":
    main()

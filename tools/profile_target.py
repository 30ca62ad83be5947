#!/usr/bin/env python3
"""Minimal profiling target: N renders of a bench workload (default: random spheres
1920x1080 @ 256 spp, fp32, default tuning; --scene mesh/mixed for configs 3/4) through
the C ABI, nothing else on the GPU.  --meta FILE writes the PMC keys of this launch
(raytracingproject_amd/measure.py: the same keys bench.py looks profiles up by).

rocprofv3 --kernel-trace --stats ... -- python3 tools/profile_target.py [--frames 3]
"""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from raytracingproject_amd import _native as N  # noqa: E402
from raytracingproject_amd import api, rtweekend, scenes  # noqa: E402
from raytracingproject_amd.measure import pmc_tuning_key, pmc_workload_key  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--scene", choices=["random", "mesh", "mixed"], default="random")
    ap.add_argument("--mesh-level", type=int, default=scenes.MESH_LEVEL)
    ap.add_argument("--precision", choices=["f32", "f64"], default="f32")
    ap.add_argument("--tune", default="", help="rt_tuning overrides, e.g. traversal=728,coh_refill=32")
    ap.add_argument("--meta", default=None, help="write the PMC keys of this launch to this JSON file")
    a = ap.parse_args()
    import torch
    rtweekend.reset_stream()
    world = {"random": scenes.random_spheres, "mesh": lambda: scenes.mesh_only(a.mesh_level),
             "mixed": lambda: scenes.mixed(a.mesh_level)}[a.scene]()
    S, M, T = api.flatten_scene(world)
    cam_api = scenes.main_camera()
    cam_api.image_width, cam_api.samples_per_pixel = a.width, a.spp
    cam = cam_api.native
    f64 = a.precision == "f64"
    r = N.Renderer(0, 0x5EED, N.RT_PREC_F64 if f64 else N.RT_PREC_F32)
    tune = {}
    for kv in filter(None, a.tune.split(",")):
        k, v = kv.split("=")
        tune[k] = float(v) if "." in v else int(v)
    if tune:
        r.set_tuning(**tune)
    r.upload_scene(S, M, T if len(T) else None)
    info = r.scene_info()
    keys = {"workload": pmc_workload_key(a.scene, a.mesh_level, cam.image_width, cam.image_height, a.spp),
            "tuning": pmc_tuning_key(r.tuning(), info, {0: "host", 1: "gpu", 2: "gpu-lbvh"}[r.tuning().mesh_builder], a.precision)}
    print(f"render_block {info.render_block} kernel {info.render_traversal} lds_bytes {info.lds_bytes} "
          f"mesh_nodes {info.mesh_nodes} keys {json.dumps(keys)}", flush=True)
    if a.meta:
        Path(a.meta).parent.mkdir(parents=True, exist_ok=True)
        Path(a.meta).write_text(json.dumps(keys) + "\n")
    lay = N.shard_layout(cam.image_width, cam.image_height, 0, 1)
    out = torch.empty(lay.max_shard_tiles * 64 * 3, dtype=torch.float64 if f64 else torch.float32, device="cuda")
    for _ in range(a.frames):
        r.render(cam, a.spp, 50, 0, 1, out.data_ptr())
        print(f"frame {r.last_kernel_ms():.3f} ms", flush=True)


if __name__ == "__main__":
    main()

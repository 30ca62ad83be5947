#!/usr/bin/env python3
"""Kernel variants (rt_tuning overrides, RT_* env knobs) against the default kernel: frame
time and agreement (8-bit frame, segment counts).

python tools/variant_probe.py [--scene random|mesh|mixed] [--spp 256] [--frames 3]
    [--variants "traversal=88;block=512,traversal=8;coh_refill=32"]
Each line: kernel variant, best/mean kernel ms of the frames, and the 8-bit frame's
difference from the default kernel's (max LSB, share identical).
"""
import argparse
import hashlib
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from raytracingproject_amd import _native as N  # noqa: E402
from raytracingproject_amd import api, rtweekend, scenes  # noqa: E402


def run(world, cam, spp, frames, tune, depth=50, env=None, precision=N.RT_PREC_F32):
    for k, v in (env or {}).items():
        os.environ[k] = str(v)
    with N.Renderer(0, 0x5EED, precision) as r:
        r.set_tuning(**tune)
        r.upload_scene(*world)
        info = r.scene_info()
        run.info = {"lds": info.lds_bytes, "nodes": info.bvh_nodes, "depth": info.bvh_depth, "leaves": info.bvh_leaves,
                    "block": info.render_block, "kernel": getattr(info, "render_traversal", None)}
        r.render_frame(cam, spp, depth)   # warm-up (module load, buffers): the first variant is not penalised
        ms = []
        for _ in range(frames):
            sums, rgb, segs = r.render_frame(cam, spp, depth)
            ms.append(r.last_kernel_ms())
    for k in (env or {}):
        os.environ.pop(k, None)
    return ms, rgb, segs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--variants", default="")
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--scene", choices=["random", "mesh", "mixed"], default="random")
    ap.add_argument("--mesh-level", type=int, default=7)
    ap.add_argument("--precision", choices=["f32", "f64"], default="f32")
    a = ap.parse_args()
    prec = N.RT_PREC_F64 if a.precision == "f64" else N.RT_PREC_F32
    rtweekend.reset_stream()
    if a.scene == "random":
        world = api.flatten(scenes.random_spheres())
    else:
        import tempfile
        from raytracingproject_amd import meshgen
        with tempfile.TemporaryDirectory() as td:
            path = Path(td) / "blob.obj"
            if a.scene == "mesh":
                V, F = meshgen.blob(a.mesh_level, radius=1.6, center=(0.0, 1.0, 0.0))
            else:
                V, F = meshgen.blob(a.mesh_level, radius=meshgen.MESH_RADIUS, center=meshgen.MESH_CENTER)
            meshgen.write_obj(path, V, F)
            rtweekend.reset_stream()
            w = scenes.mesh_only(obj_path=path) if a.scene == "mesh" else scenes.mixed(obj_path=path)
            S, M, T = api.flatten_scene(w)
            world = (S, M, T if len(T) else None)
    c = scenes.main_camera()
    c.image_width, c.samples_per_pixel = a.width, a.spp
    cam = c.native
    ms0, rgb0, segs0 = run(world, cam, a.spp, a.frames, {}, depth=a.depth, precision=prec)
    # (digests: frames of different libraries -- RT_LIB_PATH -- compared across processes)
    print(json.dumps({"variant": "default", "best_ms": min(ms0), "ms": ms0, "scene": run.info,
                      "rgb_sha": hashlib.sha256(rgb0.tobytes()).hexdigest()[:16],
                      "segs_sha": hashlib.sha256(segs0.tobytes()).hexdigest()[:16]}), flush=True)
    vs = []
    for v in a.variants.split(";"):
        if v:
            kv = dict(x.split("=") for x in v.split(","))
            env = {k: kv.pop(k) for k in list(kv) if k.startswith("RT_")}
            vs.append(({k: (float(x) if "." in x else int(x)) for k, x in kv.items()}, env))
    for tune, env in vs:
        t0 = time.time()
        ms, rgb, segs = run(world, cam, a.spp, a.frames, tune, depth=a.depth, env=env, precision=prec)
        d = np.abs(rgb.astype(np.int64) - rgb0)
        bad = np.argwhere((d.max(axis=2) > 0) | (segs != segs0))[:8].tolist()
        print(json.dumps({"variant": {**tune, **env}, "best_ms": min(ms), "ms": ms, "scene": run.info,
                          "speedup": min(ms0) / min(ms), "max_lsb": int(d.max()),
                          "identical": float((d == 0).mean()), "segs_equal": bool(np.array_equal(segs, segs0)),
                          "segs_per_primary": float(segs.sum()) / (rgb.shape[0] * rgb.shape[1] * a.spp),
                          "segs0_per_primary": float(segs0.sum()) / (rgb.shape[0] * rgb.shape[1] * a.spp),
                          "wall_s": time.time() - t0, "first_diff_yx": bad}), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Upper bound of ray sorting for the bounce loop: trace the same
batch of first-bounce (scattered) rays of the C3 frame through rt_trace_rays in the order
the render kernel's waves see them (8x8 tile by tile), shuffled, and sorted by direction
octant + origin cell (Morton), and report the node / sphere loop lane utilisation
(rt_trace_rays_diag) and the kernel time of each order.

Sorting *within* a wave cannot change its work (a wave runs until its slowest lane, so
which lane holds which ray is irrelevant); what sorting can buy is rays of one wave that
are alike, i.e. regrouping across waves.  Globally sorted batches are the best case any
such regrouping could approach; the `wg*` orders are what a workgroup could do in the
render kernel: rays regrouped only within consecutive groups of 1,024 (16 waves of 64,
tile order) -- by octant, or by octant then origin.

--bounce b measures the rays of scattering event b (1 = the first scattered rays; b > 1:
the surviving paths' later rays, still in their paths' tile order).

python tools/sort_bound.py [--width 1920 --spp 2 --bounce 1]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from raytracingproject_amd import _native as N  # noqa: E402
from raytracingproject_amd import api, rtweekend, scenes  # noqa: E402


def camera_rays(cam, spp: int, g: np.random.Generator) -> np.ndarray:
    """get_ray (camera.h:87-113) for every pixel and sample, tile-major (8x8 tiles, the
    samples of a tile together) -- the order of the render kernel's camera-ray batches."""
    W, H = cam.image_width, cam.image_height
    ty, tx, sy, sx = np.meshgrid(np.arange((H + 7) // 8), np.arange((W + 7) // 8), np.arange(8), np.arange(8),
                                 indexing="ij")
    x, y = (tx * 8 + sx).ravel(), (ty * 8 + sy).ravel()
    keep = (x < W) & (y < H)
    x, y = np.repeat(x[keep], spp), np.repeat(y[keep], spp)
    p00, du, dv = (np.array(cam.pixel00_loc), np.array(cam.pixel_delta_u), np.array(cam.pixel_delta_v))
    n = len(x)
    ps = p00 + (x[:, None] + g.uniform(-0.5, 0.5, (n, 1))) * du + (y[:, None] + g.uniform(-0.5, 0.5, (n, 1))) * dv
    r = np.sqrt(g.uniform(0, 1, n))
    ang = g.uniform(0, 2 * np.pi, n)
    o = np.array(cam.center) + (r * np.cos(ang))[:, None] * np.array(cam.defocus_disk_u) + \
        (r * np.sin(ang))[:, None] * np.array(cam.defocus_disk_v)
    return np.concatenate([o, ps - o, g.uniform(0, 1, (n, 1))], axis=1)


def unit(v):
    return v / np.linalg.norm(v, axis=1, keepdims=True)


def in_unit_sphere(n, g):
    v = g.normal(size=(n, 3))
    return unit(v) * g.uniform(0, 1, (n, 1)) ** (1 / 3)


def scatter(rays, hits, M, g):
    """material::scatter (material.h:15-82) in numpy: the first-bounce rays of the hits."""
    h = hits[hits["id"] >= 0]
    d = rays[hits["id"] >= 0][:, 3:6]
    tm = rays[hits["id"] >= 0][:, 6:7]
    n = h["normal"]
    typ = M["type"][h["mat"]]
    out = n + unit(g.normal(size=n.shape))                                      # lambertian
    ud = unit(d)
    refl = ud - 2 * np.sum(ud * n, axis=1, keepdims=True) * n
    metal = refl + M["fuzz"][h["mat"]][:, None] * in_unit_sphere(len(n), g)
    out = np.where((typ == N.RT_METAL)[:, None], metal, out)
    ratio = np.where(h["front_face"] != 0, 1 / 1.5, 1.5)[:, None]
    cos_t = np.minimum(np.sum(-ud * n, axis=1, keepdims=True), 1.0)
    perp = ratio * (ud + cos_t * n)
    par = -np.sqrt(np.abs(1 - np.sum(perp * perp, axis=1, keepdims=True))) * n
    r0 = ((1 - ratio) / (1 + ratio)) ** 2
    tir = ratio * np.sqrt(1 - cos_t ** 2) > 1
    schlick = r0 + (1 - r0) * (1 - cos_t) ** 5 > g.uniform(0, 1, (len(n), 1))
    glass = np.where(tir | schlick, refl, perp + par)
    out = np.where((typ == N.RT_DIELECTRIC)[:, None], glass, out)
    return np.concatenate([h["p"], out, tm], axis=1)


def morton3(q: np.ndarray) -> np.ndarray:
    def spread(v):
        v = v.astype(np.uint64) & 0x3FF
        v = (v | (v << 16)) & 0x30000FF
        v = (v | (v << 8)) & 0x300F00F
        v = (v | (v << 4)) & 0x30C30C3
        return (v | (v << 2)) & 0x9249249
    return spread(q[:, 0]) | (spread(q[:, 1]) << 1) | (spread(q[:, 2]) << 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--spp", type=int, default=2)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--bounce", type=int, default=1)
    ap.add_argument("--group", type=int, default=1024)
    a = ap.parse_args()
    import torch
    g = np.random.default_rng(7)
    rtweekend.reset_stream()
    S, M = api.flatten(scenes.random_spheres())
    cam_api = scenes.main_camera()
    cam_api.image_width = a.width
    cam = cam_api.native
    r = N.Renderer(0, 0x5EED, N.RT_PREC_F32)
    r.upload_scene(S, M)
    prim = camera_rays(cam, a.spp, g)
    hits = r.trace_rays_host(prim.astype(np.float32))
    sec = scatter(prim, hits, M, g)
    for _ in range(a.bounce - 1):
        hits = r.trace_rays_host(sec.astype(np.float32))
        sec = scatter(sec, hits, M, g)
    lo, hi = sec[:, :3].min(axis=0), sec[:, :3].max(axis=0)
    cell = np.floor((sec[:, :3] - lo) / np.maximum(hi - lo, 1e-9) * 1023).astype(np.int64)
    octant = ((sec[:, 3] < 0) * 1 + (sec[:, 4] < 0) * 2 + (sec[:, 5] < 0) * 4).astype(np.uint64)
    mort = morton3(cell)
    grp = np.arange(len(sec)) // a.group   # the workgroup a ray belongs to (tile order)
    orders = {
        "tile_order": np.arange(len(sec)),
        "shuffled": g.permutation(len(sec)),
        "octant_then_origin": np.lexsort((mort, octant)),
        "origin_then_octant": np.lexsort((octant, mort)),
        f"wg{a.group}_octant": np.lexsort((octant, grp)),
        f"wg{a.group}_octant_then_origin": np.lexsort((mort, octant, grp)),
    }
    dev_hits = torch.empty(len(sec) * N.HIT_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    for name, idx in orders.items():
        rays = torch.from_numpy(np.ascontiguousarray(sec[idx], dtype=np.float32)).to("cuda")
        torch.cuda.synchronize()
        d = r.trace_rays_diag(rays.data_ptr(), len(sec), dev_hits.data_ptr())
        ms = []
        for _ in range(a.reps):
            r.trace_rays(rays.data_ptr(), len(sec), dev_hits.data_ptr())
            ms.append(r.last_kernel_ms())
        print(json.dumps({"order": name, "bounce": a.bounce, "spp": a.spp, "rays": len(sec), "best_ms": round(min(ms), 3),
                          "inner_lane_util": round(d["inner_act"] / (64 * d["inner_it"]), 4),
                          "leaf_lane_util": round(d["leaf_act"] / (64 * d["leaf_it"]), 4),
                          "inner_visits_per_ray": round(d["inner_act"] / len(sec), 3),
                          "leaf_tests_per_ray": round(d["leaf_act"] / len(sec), 3),
                          "wave_iters_per_64_rays": round(64 * (d["inner_it"] + d["leaf_it"]) / len(sec), 2)}),
              flush=True)
    r.close()


if __name__ == "__main__":
    t0 = time.time()
    main()

#!/usr/bin/env python3
"""Watertightness probe for the fp32 triangle test.

GPU mode: rays from inside the closed config-4 blob (327,680 triangles, centre (0, 1, 0))
through rt_trace_rays in fp32; every ray must hit something (the blob, or the ground where
it cuts the blob).  The rays that miss ("leaks") are traced again in fp64 and saved with
the triangle the fp64 test hits, per tuning variant (host SAH tree, GPU LBVH tree), so a
leak can be pinned on the triangle test (same ray leaks with either tree) or on the tree.

    python tools/leak_probe.py --rays 33554432 --out gpurun_out/leaks.npz

CPU mode (--analyze FILE): restates the fp32 Moller-Trumbore test in numpy for each leaked
ray against the fp64 triangle and the triangles sharing its vertices, and prints the
barycentrics and the conditioning |o - v0| / edge length.
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from raytracingproject_amd import meshgen, scenes  # noqa: E402

CENTER = np.array([0.0, 1.0, 0.0])


def make_rays(rng, n, spread):
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    o = CENTER + rng.uniform(-spread, spread, size=(n, 3))
    return np.concatenate([o, d, np.zeros((n, 1))], axis=1).astype(np.float32)


def gpu(args):
    from raytracingproject_amd import _native as N
    from raytracingproject_amd import api
    S, M, T = api.flatten_scene(scenes.mesh_only(scenes.MESH_LEVEL))
    out = {}
    report = {}
    for name, tune in (("host", {}), ("gpu_lbvh", {"mesh_builder": N.RT_MESH_BUILD_GPU})):
        rng = np.random.default_rng(args.seed)
        leaks = []
        t0 = time.perf_counter()
        with N.Renderer(0, 0x5EED, N.RT_PREC_F32) as r:
            if tune:
                r.set_tuning(**tune)
            r.upload_scene(S, M, T)
            done = 0
            while done < args.rays:
                n = min(args.batch, args.rays - done)
                rays = make_rays(rng, n, args.spread)
                h = r.trace_rays_host(rays)
                miss = h["id"] == -1
                leaks.append(rays[miss])
                done += n
        L = np.concatenate(leaks) if leaks else np.zeros((0, 7), np.float32)
        with N.Renderer(0, 0x5EED, N.RT_PREC_F64) as r:
            r.upload_scene(S, M, T)
            h64 = r.trace_rays_host(L.astype(np.float64)) if len(L) else np.zeros(0, N.HIT_DTYPE)
        out[f"{name}_rays"] = L
        out[f"{name}_id64"] = h64["id"] if len(L) else np.zeros(0, np.int32)
        out[f"{name}_t64"] = h64["t"] if len(L) else np.zeros(0)
        report[name] = {"rays": args.rays, "leaks": int(len(L)), "rate": len(L) / args.rays,
                        "fp64_misses_of_those": int((out[f"{name}_id64"] == -1).sum()),
                        "s": round(time.perf_counter() - t0, 1)}
        print(name, json.dumps(report[name]), flush=True)
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    np.savez_compressed(args.out, n_spheres=len(S), **out)
    print(json.dumps(report))


def mt_f32(o, d, v0, e1, e2):
    """fp32 Moller-Trumbore in numpy float32 (no FMA: close to, not bit-equal with, the GPU)."""
    f = np.float32

    def cross(a, b):
        return np.array([a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]], f)

    pv = cross(d, e2)
    det = f(np.dot(e1, pv))
    inv = f(1) / det
    tv = (o - v0).astype(f)
    u = f(np.dot(tv, pv)) * inv
    qv = cross(tv, e1)
    v = f(np.dot(d, qv)) * inv
    t = f(np.dot(e2, qv)) * inv
    return float(u), float(v), float(t), float(det)


def analyze(path):
    z = np.load(path)
    S0 = int(z["n_spheres"])
    V, F = meshgen.blob(scenes.MESH_LEVEL, radius=1.6, center=(0.0, 1.0, 0.0))
    vert_tris = {}
    for k, tri in enumerate(F):
        for v in tri:
            vert_tris.setdefault(int(v), []).append(k)
    for name in ("host", "gpu_lbvh"):
        rays, ids = z[f"{name}_rays"], z[f"{name}_id64"]
        print(f"== {name}: {len(rays)} leaks")
        for ray, i64 in zip(rays[:20], ids[:20]):
            o, d = ray[:3].astype(np.float32), ray[3:6].astype(np.float32)
            if i64 < S0:
                print("  fp64 hit sphere", i64)
                continue
            k = int(i64) - S0
            near = sorted({t for v in F[k] for t in vert_tris[int(v)]})
            print(f"  ray o={o.tolist()} d={d.tolist()} fp64 triangle {k}")
            for t in near:
                a, b, c = V[F[t]]
                v0 = a.astype(np.float32)
                e1 = (b - a).astype(np.float32)
                e2 = (c - a).astype(np.float32)
                u, v, tt, det = mt_f32(o, d, v0, e1, e2)
                cond = np.linalg.norm(o - a) / max(np.linalg.norm(b - a), np.linalg.norm(c - a))
                inside = -1e-6 <= u <= 1 + 1e-6 and -1e-6 <= v and u + v <= 1 + 1e-6
                if abs(u) < 1e-3 or abs(v) < 1e-3 or abs(1 - u - v) < 1e-3 or t == k:
                    print(f"    tri {t}{'*' if t == k else ' '} u={u:+.9f} v={v:+.9f} w={1 - u - v:+.9f} "
                          f"t={tt:.6f} det={det:.3e} cond={cond:.0f} {'IN' if inside else ''}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=1 << 25)
    ap.add_argument("--batch", type=int, default=1 << 22)
    ap.add_argument("--spread", type=float, default=0.3, help="origins uniform in a cube of this half-size")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default="gpurun_out/leaks.npz")
    ap.add_argument("--analyze", default=None)
    a = ap.parse_args()
    if a.analyze:
        analyze(a.analyze)
    else:
        gpu(a)


if __name__ == "__main__":
    main()

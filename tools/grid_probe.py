#!/usr/bin/env python3
"""CPU estimate of a uniform sphere grid's work on the C3 field (round 5).

Traces a sample of C3's paths brute force over main.cpp's spheres (approximate scattering:
enough for the ray distribution), then walks each ray's cells through a uniform grid over
the small spheres' swept boxes and counts cells visited and spheres listed in them, up to
the ray's closest hit -- the work the grid kernel would do, against the tree's 7.1 node
visits (two box tests each) and 5.5 sphere tests per scattered ray (§5 counters).

python tools/grid_probe.py [--paths 40000] [--rays 20000] [--regroup | --slabs]

--slabs: the kernel's loop iterations per ray and per wave of 64 scattered rays when each ray
is clipped to the box of the spheres at its time's slab (rt_scene.h GridHdr), by slab count.

--defer (r06): regrouping in time instead of across waves -- a wave that traces only its
long (near-horizontal) rays once enough of them wait, and its short ones otherwise, each trace
round costing its slowest lane plus a shade pass of `shade` loop iterations: wave iterations
per 64 traced rays against tracing every lane every round.
"""
import argparse
import math
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from raytracingproject_amd import rtweekend, scenes  # noqa: E402


def field():
    rtweekend.reset_stream()
    w = scenes.random_spheres()
    C = np.array([o.center1 for o in w.objects], float)
    V = np.array([o.center_vec for o in w.objects], float)
    R = np.array([o.radius for o in w.objects], float)
    M = np.array([{"lambertian": 0, "metal": 1}.get(type(o.mat).__name__, 2) for o in w.objects])
    return C, V, R, M


def paths(C, V, R, M, n, rng, depth=12, times=False):
    """Closest hits of n C3 camera paths (no defocus), brute force; rays of every bounce
    (times: also the rays' times, and the camera rays left out)."""
    W, H = 1920, 1080
    lf, la, vup = np.array([13, 2, 3.0]), np.zeros(3), np.array([0, 1, 0.0])
    fd, hh = 10.0, math.tan(math.radians(20) / 2)
    vh = 2 * hh * fd
    vw = vh * W / H
    ww = (lf - la) / np.linalg.norm(lf - la)
    u = np.cross(vup, ww)
    u /= np.linalg.norm(u)
    v = np.cross(ww, u)
    px, py = rng.random(n) * W, rng.random(n) * H
    o = np.repeat(lf[None], n, 0)
    d = lf - fd * ww + (px[:, None] / W - 0.5) * vw * u - (py[:, None] / H - 0.5) * vh * v - o
    tm = rng.random(n)
    out = []
    for _ in range(depth):
        cc = C[None] + tm[:, None, None] * V[None]
        oc = cc - o[:, None]
        a = (d * d).sum(1)[:, None]
        h = (oc * d[:, None]).sum(2)
        c = (oc * oc).sum(2) - R[None] ** 2
        disc = h * h - a * c
        sq = np.sqrt(np.maximum(disc, 0))
        t0, t1 = (h - sq) / a, (h + sq) / a
        t = np.where(disc >= 0, np.where(t0 > 1e-3, t0, np.where(t1 > 1e-3, t1, np.inf)), np.inf)
        k = t.argmin(1)
        th = t[np.arange(len(k)), k]
        if not times:
            out.append((o.copy(), d.copy(), th.copy()))
        elif _:
            out.append((o.copy(), d.copy(), th.copy(), tm.copy()))
        hit = np.isfinite(th)
        p = o + np.where(hit, th, 0)[:, None] * d
        nrm = (p - (C[k] + tm[:, None] * V[k])) / R[k][:, None]
        ru = rng.normal(size=(len(k), 3))
        ru /= np.linalg.norm(ru, axis=1)[:, None]
        dn = d / np.linalg.norm(d, axis=1)[:, None]
        refl = dn - 2 * (dn * nrm).sum(1)[:, None] * nrm
        m = M[k][:, None]
        nd = np.where(m == 0, nrm + ru, np.where(m == 1, refl + 0.2 * ru, dn))
        keep = hit & ~((M[k] == 1) & ((nd * nrm).sum(1) <= 0))
        o, d, tm = p[keep], nd[keep], tm[keep]
        if not len(o):
            break
    return [np.concatenate(x) for x in zip(*out)]


def walk(C, V, R, O, D, TH, density, sample, rng):
    small = np.where(R < 1.0)[0][1:] if R[0] >= 64 else np.where(R < 1.0)[0]
    lo = np.minimum(C[small], C[small] + V[small]) - R[small, None]
    hi = np.maximum(C[small], C[small] + V[small]) + R[small, None]
    glo, ghi = lo.min(0), hi.max(0)
    E = ghi - glo
    cell = (E.prod() / (density * len(small))) ** (1 / 3)
    res = np.maximum(1, np.round(E / cell)).astype(int)
    cs = E / res
    cnt = np.zeros(res, int)
    for a, b in zip(((lo - glo) / cs).astype(int).clip(0, res - 1), ((hi - glo) / cs).astype(int).clip(0, res - 1)):
        cnt[a[0]:b[0] + 1, a[1]:b[1] + 1, a[2]:b[2] + 1] += 1
    ncell = ntest = 0
    for i in rng.choice(len(O), sample, replace=False):
        o, d, th = O[i], D[i], TH[i]
        inv = 1 / np.where(d == 0, 1e-30, d)
        t0, t1 = (glo - o) * inv, (ghi - o) * inv
        tn, tf = max(np.minimum(t0, t1).max(), 1e-3), min(np.maximum(t0, t1).min(), th)
        if tn > tf:
            continue
        ix = np.clip(((o + tn * d - glo) / cs).astype(int), 0, res - 1)
        step = np.where(d > 0, 1, -1)
        tmx = (glo + (ix + (step > 0)) * cs - o) * inv
        dt = np.abs(cs * inv)
        while True:
            ncell += 1
            ntest += cnt[tuple(ix)]
            ax = int(np.argmin(tmx))
            if tmx[ax] >= tf:
                break
            ix[ax] += step[ax]
            if not 0 <= ix[ax] < res[ax]:
                break
            tmx[ax] += dt[ax]
    return res.tolist(), ncell / sample, ntest / sample


def loop_iterations(C, V, R, O, D, TH, res, TM=None, slabs=1):
    """Iterations of the kernel's single step-and-test loop per ray (a step and a test per
    iteration) over a grid of the given resolution; with ray times TM, each ray clipped to
    the spheres' box over its time slab (of `slabs`), as the kernel does."""
    small = np.where(R < 1.0)[0][1:] if R[0] >= 64 else np.where(R < 1.0)[0]
    lo = np.minimum(C[small], C[small] + V[small]) - R[small, None]
    hi = np.maximum(C[small], C[small] + V[small]) + R[small, None]
    glo, ghi = lo.min(0), hi.max(0)
    sbox = []
    for k in range(slabs):
        c0, c1 = C[small] + k / slabs * V[small], C[small] + (k + 1) / slabs * V[small]
        sbox.append(((np.minimum(c0, c1) - R[small, None]).min(0), (np.maximum(c0, c1) + R[small, None]).max(0)))
    res = np.array(res)
    cs = (ghi - glo) / res
    cnt = np.zeros(res, int)
    for a, b in zip(((lo - glo) / cs).astype(int).clip(0, res - 1), ((hi - glo) / cs).astype(int).clip(0, res - 1)):
        cnt[a[0]:b[0] + 1, a[1]:b[1] + 1, a[2]:b[2] + 1] += 1
    out = np.zeros(len(O), int)
    for i in range(len(O)):
        o, d, th = O[i], D[i], TH[i]
        inv = 1 / np.where(d == 0, 1e-30, d)
        blo, bhi = (glo, ghi) if TM is None else sbox[min(int(TM[i] * slabs), slabs - 1)]
        t0, t1 = (blo - o) * inv, (bhi - o) * inv
        tn, tf = max(np.minimum(t0, t1).max(), 1e-3), min(np.maximum(t0, t1).min(), th)
        if tn > tf:
            continue
        ix = np.clip(((o + tn * d - glo) / cs).astype(int), 0, res - 1)
        step = np.where(d > 0, 1, -1)
        tmx = (glo + (ix + (step > 0)) * cs - o) * inv
        dt = np.abs(cs * inv)
        it, pending = 0, cnt[tuple(ix)]
        while True:
            it += 1
            if pending > 0:
                pending -= 1
            if pending == 0:
                ax = int(np.argmin(tmx))
                if tmx[ax] >= tf or not 0 <= ix[ax] + step[ax] < res[ax]:
                    break
                ix[ax] += step[ax]
                tmx[ax] += dt[ax]
                pending = cnt[tuple(ix)]
        out[i] = it
    return out


def regroup_bound(its, key, groups=(128, 256, 512, 1024)):
    """Wave iterations (the longest of 64 lanes) for rays in random order against rays sorted
    by `key` within groups of G (what G lanes exchanging rays could reach), and by the exact
    iteration count (the bound of any key)."""
    n = len(its) // 1024 * 1024
    its, key = its[:n], key[:n]
    wave = lambda order: its[order].reshape(-1, 64).max(1).mean()
    base = np.arange(n)
    print(f"loop iterations per ray {its.mean():.2f}; random waves {wave(base):.2f} per wave "
          f"(lane utilisation {its.mean() / wave(base):.3f})")
    for g in groups:
        by_key = np.concatenate([b[np.argsort(key[b])] for b in base.reshape(-1, g)])
        exact = np.concatenate([b[np.argsort(its[b])] for b in base.reshape(-1, g)])
        print(f"groups of {g}: by the key {wave(by_key):.2f} ({its.mean() / wave(by_key):.3f}), "
              f"exact {wave(exact):.2f} ({its.mean() / wave(exact):.3f})")


def defer_bound(its, key, shades=(0, 4, 8, 12)):
    """A wave of 64 lanes, each holding a ray of the stream (in order); per round it traces
    either its long rays (key < tau: near-horizontal) once at least L wait, or its short ones,
    refilling the traced lanes from the stream."""
    n = len(its)

    def sim(tau, lth, shade):
        nxt, lanes, cost, traced = 64, np.arange(64), 0.0, 0
        while nxt < n - 64:
            lk = key[lanes] < tau
            nl = int(lk.sum())
            sel = np.ones(64, bool) if tau <= 0 else (lk if (nl >= lth or nl == 64) else ~lk)
            cost += shade + its[lanes[sel]].max()
            k = int(sel.sum())
            traced += k
            lanes[sel] = np.arange(nxt, nxt + k)
            nxt += k
        return cost / traced * 64

    for shade in shades:
        base = sim(0, 0, shade)
        best = min((sim(t, l, shade), t, l) for t in (0.05, 0.1, 0.2, 0.3, 0.5) for l in (8, 16, 32, 48))
        print(f"shade {shade}: every lane every round {base:.2f} per 64 rays; best deferral {best[0]:.2f} "
              f"(tau {best[1]}, L {best[2]}) {best[0] / base - 1:+.1%}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--paths", type=int, default=40000)
    ap.add_argument("--rays", type=int, default=20000)
    ap.add_argument("--regroup", action="store_true",
                    help="the bound of regrouping rays by elevation before the walk (round 5)")
    ap.add_argument("--slabs", action="store_true", help="the walk clipped to time-slab boxes (round 5)")
    ap.add_argument("--defer", action="store_true", help="regrouping in time within a wave (round 6)")
    ap.add_argument("--slab-count", type=int, default=0,
                    help="--regroup over scattered rays clipped to this many time slabs (0: all rays, no slabs)")
    a = ap.parse_args()
    rng = np.random.default_rng(1)
    C, V, R, M = field()
    if a.slabs:
        O, D, TH, TM = paths(C, V, R, M, a.paths, rng, times=True)
        idx = np.random.default_rng(0).permutation(len(O))[:a.rays // 64 * 64]
        print(f"{len(O)} scattered rays over {a.paths} paths, {len(idx)} walked")
        for k in (1, 4, 8, 16, 32, 64):
            its = loop_iterations(C, V, R, O[idx], D[idx], TH[idx], (29, 1, 29), TM[idx], k)
            print(f"slabs {k}: loop iterations per ray {its.mean():.2f}, per wave of 64 "
                  f"{its.reshape(-1, 64).max(1).mean():.2f}", flush=True)
        return
    O, D, TH = paths(C, V, R, M, a.paths, rng)
    print(f"{len(O)} rays over {a.paths} paths")
    if a.defer:
        O, D, TH, TM = paths(C, V, R, M, a.paths, np.random.default_rng(1), times=True)
        idx = np.random.default_rng(0).permutation(len(O))[:a.rays]
        its = loop_iterations(C, V, R, O[idx], D[idx], TH[idx], (29, 1, 29), TM[idx], 32)
        defer_bound(its, np.abs(D[idx, 1]) / np.linalg.norm(D[idx], axis=1))
        return
    if a.regroup and a.slab_count:
        O, D, TH, TM = paths(C, V, R, M, a.paths, np.random.default_rng(1), times=True)
        idx = np.random.default_rng(0).permutation(len(O))[:a.rays]
        its = loop_iterations(C, V, R, O[idx], D[idx], TH[idx], (29, 1, 29), TM[idx], a.slab_count)
        regroup_bound(its, np.abs(D[idx, 1]) / np.linalg.norm(D[idx], axis=1))
        return
    if a.regroup:
        idx = np.random.default_rng(0).permutation(len(O))[:a.rays]
        its = loop_iterations(C, V, R, O[idx], D[idx], TH[idx], (29, 1, 29))
        regroup_bound(its, np.abs(D[idx, 1]) / np.linalg.norm(D[idx], axis=1))
        return
    for dens in (0.5, 1.0, 2.0, 3.0):
        res, cells, tests = walk(C, V, R, O, D, TH, dens, min(a.rays, len(O)), np.random.default_rng(0))
        print(f"density {dens}: {res} cells; per ray {cells:.2f} cells, {tests:.2f} sphere tests")


if __name__ == "__main__":
    main()

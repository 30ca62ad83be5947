#!/usr/bin/env python3
"""Phase breakdown of the persistent fp32 render kernel (instrumented build, rt_render_diag).

python tools/diag.py [--width 1920 --spp 64] [--scene random|four|mesh|mixed]
Mesh scenes run the default mesh kernel (their own block and traversal) and add the
mesh-BVH loop counters: node visits and triangle tests per traced ray, lane utilisation.
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
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--block", type=int, default=1024)
    ap.add_argument("--scene", choices=["random", "four", "mesh", "mixed"], default="random")
    ap.add_argument("--mesh-level", type=int, default=7)
    ap.add_argument("--trav", type=int, default=600)
    ap.add_argument("--wpe", type=int, default=8)
    ap.add_argument("--depth", type=int, default=50)
    a = ap.parse_args()
    rtweekend.reset_stream()
    mesh = a.scene in ("mesh", "mixed")
    if mesh:
        world = (scenes.mesh_only if a.scene == "mesh" else scenes.mixed)(level=a.mesh_level)
        flat = api.flatten_scene(world)
    else:
        world = scenes.random_spheres() if a.scene == "random" else scenes.four_spheres()
        flat = api.flatten(world)
    cam_api = scenes.main_camera()
    cam_api.image_width, cam_api.samples_per_pixel = a.width, a.spp
    cam = cam_api.native
    r = N.Renderer(0, 0x5EED, N.RT_PREC_F32)
    if not mesh:
        r.set_tuning(traversal=a.trav, waves_per_eu=a.wpe, block=a.block)
    r.upload_scene(*flat)
    d = r.render_diag(cam, a.spp, a.depth)
    info = r.scene_info()
    rays = cam.image_width * cam.image_height * a.spp

    def q(n, m):
        return n / m if m else None
    cyc = d["cyc_trav"] + d["cyc_shade"] + d["cyc_hand"]
    out = {
        "config": f"{a.scene} {cam.image_width}x{cam.image_height}@{a.spp} depth={a.depth} traversal={info.render_traversal} block={info.render_block}",
        "segments_per_primary": d["segments"] / rays,
        "bounce_lane_util": q(d["bounce_act"], 64 * d["bounce_it"]),
        "inner_lane_util": q(d["inner_act"], 64 * d["inner_it"]),
        "leaf_lane_util": q(d["leaf_act"], 64 * d["leaf_it"]),
        "inner_lane_visits_per_segment": d["inner_act"] / d["segments"],
        "leaf_sphere_tests_per_segment": d["leaf_act"] / d["segments"],
        "inner_wave_iters_per_bounce_iter": q(d["inner_it"], d["bounce_it"]),
        "leaf_wave_iters_per_bounce_iter": q(d["leaf_it"], d["bounce_it"]),
        "share_trav": q(d["cyc_trav"], cyc), "share_shade": q(d["cyc_shade"], cyc), "share_hand": q(d["cyc_hand"], cyc),
        "flushes_per_pixel": d["flushes"] / (cam.image_width * cam.image_height),
        "cycles_per_bounce_iter": q(cyc, d["bounce_it"]),
        # K traversals per lane per bounce iteration (a per-lane queue of K rays): wave
        # step iterations relative to K=1 (the slowest lane of K consecutive calls)
        "k2_vs_k1_steps": q(d["k_it2"], d["k_it1"]) if d["k_it1"] else None,
        "k4_vs_k1_steps": d["k_it4"] / d["k_it1"] if d["k_it1"] else None,
        "k1_step_util": (d["inner_act"] + d["leaf_act"]) / (64 * d["k_it1"]) if d["k_it1"] else None,
        "raw": d,
    }
    if a.trav & 64:
        # coherent primaries (render_coherent): bounce loop = scattered rays only;
        # cyc_shade includes the batches (cyc_hand); k_it1 batches, k_it2 batch wave
        # steps, k_it4 batch lane steps, x15 primary hits popped
        out = {
            "config": out["config"],
            "secondaries_per_primary": d["segments"] / rays,
            "bounce_lane_util": q(d["bounce_act"], 64 * d["bounce_it"]),
            "inner_lane_util": q(d["inner_act"], 64 * d["inner_it"]),
            "leaf_lane_util": q(d["leaf_act"], 64 * d["leaf_it"]),
            "inner_visits_per_secondary": d["inner_act"] / d["segments"],
            "leaf_tests_per_secondary": d["leaf_act"] / d["segments"],
            "batch_step_util": q(d["k_it4"], 64 * d["k_it2"]),
            "batch_steps_per_primary": d["k_it4"] / rays,
            "batch_wave_steps_per_batch": q(d["k_it2"], d["k_it1"]),
            "pops_per_primary": d["x15"] / rays,
            "share_trav": d["cyc_trav"] / d["cyc_all"],
            "share_batch": d["cyc_hand"] / d["cyc_all"],
            "share_shade": (d["cyc_shade"] - d["cyc_hand"]) / d["cyc_all"],
            # framebuffer traffic: where finished samples went
            "samples_direct_share": d["samples_direct"] / max(1, d["samples_in_item"] + d["samples_direct"]),
            "item_flushes_per_pixel": d["item_flushes"] / (cam.image_width * cam.image_height),
        }
        # wave timeline (s_memrealtime, 100 MHz): how long the queue takes to run dry and
        # how long the waves then take to drain their FIFOs and paths in flight
        if d["waves"]:
            m = (1 << 64) - 1
            t0, t_end = m - d["rt_start_min_not"], d["rt_end_max"]
            dry0, dry1 = m - d["rt_dry_min_not"], d["rt_dry_max"]
            us = lambda ticks: ticks / 100.0   # noqa: E731
            out["timeline_us"] = {
                "kernel_span": us(t_end - t0), "first_dry": us(dry0 - t0), "last_dry": us(dry1 - t0),
                "mean_busy_until_dry": us(d["rt_busy_sum"] / d["waves"]),
                "mean_drain": us(d["rt_drain_sum"] / d["waves"]),
                "last_end_after_first_dry": us(t_end - dry0),
                "waves": d["waves"],
                "drain_bounce_iters_per_wave": d["drain_bounce_it"] / d["waves"],
                "bounce_iters_per_wave": d["bounce_it"] / d["waves"],
            }
        if mesh:
            traced = rays + d["segments"]   # camera rays (batches) + scattered rays
            out["mesh"] = {
                "node_visits_per_ray": d["mnode_act"] / traced,
                "tri_tests_per_ray": d["mtri_act"] / traced,
                "node_lane_util": d["mnode_act"] / max(1, 64 * d["mnode_it"]),
                "tri_lane_util": d["mtri_act"] / max(1, 64 * d["mtri_it"]),
                "node_wave_iters_per_wave_ray_round": d["mnode_it"] / max(1, d["bounce_it"] + d["k_it1"]),
            }
        out["raw"] = d
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

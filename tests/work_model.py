#!/usr/bin/env python3
"""Algorithmic work per primary ray for the benchmark configs: the
survey's probe method re-derived for the committed level-7 mesh (VERDICT r03 "Next" 2).

Test infrastructure: drives tests/cpp/work_model.cpp (the oracle's path logic with
world.hit answered by traversals of the product's host-built trees, counting node visits,
box tests, primitive tests, world.hit calls and hits) over a fixed pixel sample of each
config and turns the counts into the two algorithmic figures per primary ray:

  bytes  = 128 B per 4-wide mesh node visit (Node4, one L2 line) + 48 B per triangle test
           (TriF) -- the HBM-resident mesh data a ray must touch; the sphere scene is
           LDS-resident (64 B per sphere-tree node visit, 32 B per sphere test, reported
           apart as lds_bytes_per_primary);
  flop   = the survey's cost model (24 per box test, 40 per sphere test, 18 + 40 per hit
           for the hit record and scatter, 40 per camera ray, 15 per sky miss) plus 46 per
           Moller-Trumbore triangle test (2 cross products, 4 dot products, a reciprocal and
           4 scaled compares, oracle/rt_oracle.c tri_hit).

`python tests/work_model.py [--out profiles/r04/work_model_r04.json]` writes the constants
raytracingproject_amd/measure.py carries (WORK_MODEL); tests/test_work_model.py checks the
probe against the linear-scan oracle and the constants against a smaller re-run.
"""
from __future__ import annotations

import argparse
import json
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

FLOP_BOX, FLOP_SPHERE, FLOP_TRI, FLOP_HIT, FLOP_SCATTER, FLOP_CAMERA, FLOP_SKY = 24, 40, 46, 18, 40, 40, 15
BYTES_NODE4, BYTES_TRI, BYTES_NODE, BYTES_SPHERE = 128, 48, 64, 32
SEED = 0x5EED

# the benchmark configs (bench.py defaults): scene, frame width, spp
CONFIGS = {"c3": ("random", 1920, 256), "c4": ("mesh", 1920, 128), "c5": ("mixed", 3840, 1024)}


def build(out_dir: Path | None = None) -> Path:
    out_dir = out_dir or ROOT / "raytracingproject_amd" / "build" / "work_model"
    out_dir.mkdir(parents=True, exist_ok=True)
    exe = out_dir / "work_model"
    srcs = [ROOT / "tests" / "cpp" / "work_model.cpp", ROOT / "raytracingproject_amd" / "csrc" / "rt_bvh.cpp"]
    orc = ROOT / "oracle" / "rt_oracle.c"
    deps = srcs + [orc, ROOT / "oracle" / "rt_oracle.h", ROOT / "raytracingproject_amd" / "csrc" / "rt_bvh.h",
                   ROOT / "raytracingproject_amd" / "csrc" / "rt_scene.h"]
    if not exe.exists() or any(d.stat().st_mtime > exe.stat().st_mtime for d in deps):
        oo = out_dir / "rt_oracle.o"
        subprocess.run(["gcc", "-O2", "-std=c11", "-ffp-contract=off", "-c", str(orc), "-o", str(oo)], check=True)
        subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", f"-I{ROOT / 'include'}", *map(str, srcs),
                        str(oo), "-o", str(exe), "-lm"], check=True)
    return exe


def scene_arrays(scene: str, level: int | None = None):
    from raytracingproject_amd import api, rtweekend, scenes
    rtweekend.reset_stream()
    if scene == "random":
        world = scenes.random_spheres()
    elif scene == "four":
        world = scenes.four_spheres()
    elif scene == "mesh":
        world = scenes.mesh_only() if level is None else scenes.mesh_only(level=level)
    else:
        world = scenes.mixed() if level is None else scenes.mixed(level=level)
    S, M, T = api.flatten_scene(world)
    return S, M, T


def run_probe(exe: Path, S, M, T, width: int, npix: int, spp: int, frame: Path | None = None) -> dict:
    with tempfile.TemporaryDirectory(prefix="rt_wm_") as d:
        d = Path(d)
        for name, a in (("s.bin", S), ("m.bin", M), ("t.bin", T)):
            (d / name).write_bytes(np.ascontiguousarray(a).tobytes() if a is not None and len(a) else b"")
        cmd = [str(exe), str(d / "s.bin"), str(d / "m.bin"), str(d / "t.bin"), str(width), str(npix), str(spp),
               hex(SEED)]
        if frame is not None:
            cmd += ["--frame", str(frame)]
        out = subprocess.run(cmd, check=True, capture_output=True, text=True).stdout
    return json.loads(out.strip().splitlines()[-1])


def model(c: dict) -> dict:
    """Per-primary algorithmic bytes and FLOP from the probe's counts."""
    misses = c["segments"] - c["hits"]
    flop = (FLOP_BOX * (c["sphere_box_tests"] + c["mesh_box_tests"]) + FLOP_SPHERE * c["sphere_tests"] +
            FLOP_TRI * c["triangle_tests"] + (FLOP_HIT + FLOP_SCATTER) * c["hits"] + FLOP_CAMERA + FLOP_SKY * misses)
    return {"hbm_bytes_per_primary": BYTES_NODE4 * c["mesh_node_visits"] + BYTES_TRI * c["triangle_tests"],
            "lds_bytes_per_primary": BYTES_NODE * c["sphere_node_visits"] + BYTES_SPHERE * c["sphere_tests"],
            "flop_per_primary_ray": flop}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=str(ROOT / "profiles" / "r04" / "work_model_r04.json"))
    ap.add_argument("--npix", type=int, default=32768)
    ap.add_argument("--spp", type=int, default=8, help="samples per sampled pixel (indices 0..spp-1)")
    a = ap.parse_args()
    exe = build()
    res = {"method": __doc__.split("\n\n")[1].replace("\n", " "), "seed": hex(SEED), "npix": a.npix,
           "spp_sampled": a.spp, "configs": {}}
    for name, (scene, width, spp) in CONFIGS.items():
        S, M, T = scene_arrays(scene)
        c = run_probe(exe, S, M, T, width, a.npix, a.spp)
        res["configs"][name] = {"scene": scene, "width": width, "spp": spp, "counts": c, **model(c)}
        print(name, json.dumps(res["configs"][name]), flush=True)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=1) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""The algorithmic work model (tests/work_model.py, tests/cpp/work_model.cpp) on the CPU:

* the probe's BVH-answered world.hit reproduces the linear-scan oracle's paths (fp64 sums
  and world.hit counts of whole small frames, spheres, mesh and mixed scenes), so its
  counts describe the reference's own paths;
* the constants bench.py carries (raytracingproject_amd/measure.py WORK_MODEL, written by
  `python tests/work_model.py` into profiles/r04/work_model_r04.json) agree with a smaller
  independent re-run, and the random-spheres counts agree with the survey's (SURVEY.md §3:
  2.580 world.hit calls per primary ray).
"""
import json

import numpy as np
import pytest

import oracle_bind as O
import work_model as WM
from raytracingproject_amd import measure

SEED = WM.SEED


@pytest.fixture(scope="module")
def exe():
    return WM.build()


@pytest.mark.parametrize("scene,level", [("four", None), ("random", None), ("mesh", 3), ("mixed", 3)])
def test_probe_paths_equal_linear_oracle(exe, tmp_path, scene, level):
    S, M, T = WM.scene_arrays(scene, level)
    W, spp = 48, 2
    out = tmp_path / "frame.bin"
    c = WM.run_probe(exe, S, M, T, W, 0, spp, frame=out)
    H = c["height"]
    got = np.fromfile(out, dtype=np.float64).reshape(H, W, 3)
    osc = O.OracleScene.from_arrays(S, M, T if len(T) else None)
    with osc.active():
        ref, _, segs = O.render_counter_full(osc, O.camera(W, spp), SEED)
    assert np.array_equal(got, ref)
    assert c["segments"] * W * H * spp == pytest.approx(float(segs.sum()), abs=0.5)
    assert c["world_hit_calls_check"] == c["segments"]
    if len(T):
        assert c["triangle_tests"] > 0 and c["mesh_node_visits"] > 0


def test_random_scene_matches_survey(exe):
    S, M, T = WM.scene_arrays("random")
    c = WM.run_probe(exe, S, M, T, 1920, 2048, 4)
    assert 2.45 < c["segments"] < 2.70            # 2.580 per primary ray
    assert c["mesh_node_visits"] == 0 and c["triangle_tests"] == 0
    m = WM.model(c)
    # the product's SAH tree needs fewer box tests than the survey's median-split probe
    # (116.1 node tests per primary ray, 3,500 FLOP)
    assert c["sphere_box_tests"] < 116.1 and m["flop_per_primary_ray"] < 3500


@pytest.mark.slow
@pytest.mark.parametrize("cfg", ["c4", "c5"])
def test_committed_constants_reproduce(exe, cfg):
    """A smaller independent sample (other pixels: a different count) lands within 8 % of
    the committed constants."""
    scene, width, _ = WM.CONFIGS[cfg]
    S, M, T = WM.scene_arrays(scene)
    c = WM.run_probe(exe, S, M, T, width, 1500, 4)
    m = WM.model(c)
    k = measure.WORK_MODEL[cfg]
    assert m["hbm_bytes_per_primary"] == pytest.approx(k["hbm_bytes_per_primary"], rel=0.08)
    assert m["flop_per_primary_ray"] == pytest.approx(k["flop_per_primary_ray"], rel=0.08)


def test_committed_constants_are_the_profile():
    d = json.loads((WM.ROOT / "profiles" / "r04" / "work_model_r04.json").read_text())
    for cfg, k in measure.WORK_MODEL.items():
        for key in ("hbm_bytes_per_primary", "lds_bytes_per_primary", "flop_per_primary_ray"):
            assert k[key] == pytest.approx(d["configs"][cfg][key], rel=1e-9), (cfg, key)


def test_bench_mesh_roofline_fields():
    """bench.py's mesh roofline object from the committed constants (r04c C4 numbers:
    265.4 M primary rays, 40.445 ms, 11.28 GB of PMC traffic per launch)."""
    import bench
    rays = 1920 * 1080 * 128
    r = bench.mesh_roofline("mesh", 7, rays, 40.445, 11280627856.0, "x.json", 0)
    k = measure.WORK_MODEL["c4"]
    assert r["bound"] == "hbm" and r["frac"] == pytest.approx(11280627856.0 / 40.445e-3 / 1e9 / 8000, rel=1e-3)
    assert r["algorithmic_bytes_per_launch"] == pytest.approx(rays * k["hbm_bytes_per_primary"], rel=1e-6)
    assert r["valu"]["frac"] == pytest.approx(rays * k["flop_per_primary_ray"] / 40.445e-3 / 157.3e12, abs=1e-4)
    assert 0 < r["traffic_over_algorithmic"] < 1    # L2 / Infinity Cache serve most of the mesh data
    assert "work_model" not in bench.mesh_roofline("mesh", 5, rays, 40.0, None, None, 0)   # other meshes: no model

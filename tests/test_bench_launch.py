"""bench.py's launch contract (CPU): `python bench.py --gpus N` with N > 1 and no launcher
starts torch.distributed.run as a child process with the same arguments and returns its
exit code, and the parent never loads torch or librt_hip (it must not touch the GPU before
the ranks do, and must never exec)."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]

_PROBE = r"""
import json, subprocess, sys
sys.path.insert(0, %r)
import bench
seen = []
def fake_call(cmd, *a, **k):
    seen.append(list(cmd))
    return 7
subprocess.call = fake_call
rc = bench.main(sys.argv[1:])
print(json.dumps({"rc": rc, "cmds": seen,
                  "torch": "torch" in sys.modules,
                  "native": any(m.startswith("raytracingproject_amd._native") for m in sys.modules)}))
"""


def _probe(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, "-c", _PROBE % str(ROOT), *args], capture_output=True, text=True,
                       timeout=120, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_parent_spawns_launcher_without_touching_gpu():
    args = ["--gpus", "8", "--steps", "3", "--warmup", "1", "--no-cpu-baseline"]
    out = _probe(args)
    assert out["rc"] == 7                       # the launcher's exit code comes back
    assert len(out["cmds"]) == 1
    cmd = out["cmds"][0]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "8"
    assert cmd[cmd.index("--nnodes") + 1] == "1"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert int(cmd[cmd.index("--master-port") + 1]) > 0
    assert Path(cmd[cmd.index("--master-port") + 2]).name == "bench.py"
    assert cmd[-len(args):] == args             # the same arguments reach every rank
    assert not out["torch"] and not out["native"]


def test_ranks_and_single_gpu_do_not_respawn():
    # N = 1: no launcher (the run proceeds and needs a GPU, so only the decision is checked)
    import bench
    a = bench.parse(["--gpus", "1"])
    assert bench.launcher_command(a, ["--gpus", "1"]) is None
    # a rank under torch.distributed.run (WORLD_SIZE set) never launches again
    a = bench.parse(["--gpus", "2"])
    old = os.environ.get("WORLD_SIZE")
    os.environ["WORLD_SIZE"] = "2"
    try:
        assert bench.launcher_command(a, ["--gpus", "2"]) is None
    finally:
        if old is None:
            del os.environ["WORLD_SIZE"]
        else:
            os.environ["WORLD_SIZE"] = old


def test_pmc_summaries_latest_round_first():
    """roofline.traffic comes from the first profiles/pmc summary whose key matches: the
    latest round's tag first (r03v < r03ah < r03bs < r04f < r04k), so a re-profiled kernel's
    counters win over an older round's under the same key."""
    import bench
    tags = [Path(p).stem.rsplit("_", 1)[-1] for p in bench.parse(["--no-cpu-baseline"]).pmc]
    order = [(t[:3], len(t), t) for t in tags]
    assert order == sorted(order, reverse=True)
    assert tags.index("r04k") < tags.index("r04f") < tags.index("r03bs") < tags.index("r03v")


def test_f64_side_line_layout():
    """--precision f32 at N = 1 adds the reference-precision kernel's figure (f64_side)
    without touching the headline keys: frame time, Mrays/s and a FLOP-model fraction of
    the FP64 vector peak."""
    import bench
    d = bench.f64_side_line(1920, 1080, 256, [97.0, 98.0], "render_kernel<double, EXACT>")
    assert set(d) == {"ms_per_frame", "frames", "mrays", "roofline", "kernel", "timed"}
    assert d["ms_per_frame"] == 97.5 and d["frames"] == 2
    assert abs(d["mrays"] - 1920 * 1080 * 256 / 0.0975 / 1e6) < 1e-3
    rl = d["roofline"]
    assert rl["unit"] == "TFLOP/s" and rl["peak"] == bench.PEAK_FP64_TFLOPS and rl["bound"] == "valu"
    assert abs(rl["frac"] - rl["achieved"] / rl["peak"]) < 1e-3
    assert bench.parse([]).f64_side_frames == 2 and bench.parse(["--f64-side-frames", "0"]).f64_side_frames == 0


def test_pmc_key_separates_shard_launches():
    """A full-frame PMC profile must not price an N-way shard launch: the
    workload key carries the shard count for N > 1, so roofline.traffic stays null there
    unless a per-shard profile was filed."""
    from raytracingproject_amd.measure import pmc_workload_key
    assert pmc_workload_key("random", 7, 1920, 1080, 256) == "1920x1080x256"
    assert pmc_workload_key("mixed", 7, 3840, 2160, 1024, 1) == "mixed7:3840x2160x1024"
    k8 = pmc_workload_key("mesh", 7, 1920, 1080, 128, 8)
    assert k8 != pmc_workload_key("mesh", 7, 1920, 1080, 128) and k8.endswith("/shard_of_8")


def test_sphere_roofline_key_set():
    """the sphere line's roofline object has exactly these keys; the survey's
    tree-model scene_bytes_gbs is gone."""
    import bench
    r = bench.sphere_roofline(False, True, 35.6, 0, 530841600, 2.5e9, "profiles/pmc/x.json")
    assert tuple(r) == bench.ROOFLINE_KEYS and "scene_bytes_gbs" not in r
    assert r["unit"] == "TFLOP/s" and r["bound"] == "valu" and r["peak"] == bench.PEAK_FP32_TFLOPS
    assert abs(r["frac"] - 530841600 * 3500 / 35.6e-3 / 1e12 / bench.PEAK_FP32_TFLOPS) < 1e-4
    assert bench.sphere_roofline(True, True, 70.0, 1, 1000, None, None)["hbm_gbs"] is None

#!/usr/bin/env python3
"""Benchmark: Mrays/sec + frame time, random-spheres 1920x1080 @ 256 spp (BASELINE.json).

One step = one frame of the reference's random-spheres scene (main.cpp:12-53, 485
spheres built on its mt19937 stream) at 1920x1080, 256 samples per pixel, depth 50,
rendered by the fp32 HIP megakernel, from the render call to the 8-bit frame in host
memory (camera::render's loop to the framebuffer, camera.h:32-50).
With N ranks (one process per GPU, launched by torch.distributed.run) each rank renders
the 8x8 tiles t = rank (mod N) and the finished shard buffers are gathered to rank 0 by
RCCL through the C ABI (rt_gather_shards = ncclGather over xGMI; torch.distributed only
bootstraps the communicator and runs the barriers).  Rank 0 un-interleaves and quantises
the frame to bytes on the device (rt_finish_frame_u8: write_color, color.h:14-35) and
copies it to page-locked host memory on a second stream, overlapped with the next frame's
render (two device/host frame buffers).  The timed region ends when the last frame is in
host memory.

value = primary camera rays of all ranks (W*H*spp per step) / max-over-ranks time.

--scene mesh / mixed run BASELINE.json configs 3/4 instead (procedural OBJ mesh read
through rt_obj_load, HBM-resident triangle BVH; the reference has no triangle path, so
these lines carry no CPU baseline).  --precision f64 times the reference-precision kernel
(fp64, the reference's operation order: bit-exact to the reference goldens) instead of
the fp32 one; it is a side line, not the headline.

At N > 1 every rank's render-kernel time is all-gathered (kernel_ms_per_rank: min / max /
argmax = the slowest shard) and rank 0 times the gather itself with HIP events around
rt_gather_shards on the render stream (gather_ms); roofline.achieved / frac are the
slowest rank's (its kernel time, its shard's rays).

Launch contract: under torch.distributed.run (WORLD_SIZE set) this process is one rank.
`python bench.py --gpus N` with N > 1 and no launcher starts
`python -m torch.distributed.run --nnodes 1 --nproc-per-node N --master-addr 127.0.0.1
--master-port <free> bench.py <same arguments>` as a child process before anything
touches the GPU (the parent imports neither torch nor librt_hip) and returns its exit code.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--scene random|mesh|mixed]
                       [--precision f32|f64]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

FLOP_PER_PRIMARY = 3500.0    # algorithmic FLOP per primary ray
PEAK_FP32_TFLOPS = 157.3     # MI355X_MICROARCH.md: FP32 vector (= FP32 MFMA) peak
PEAK_FP64_TFLOPS = 78.6      # MI355X spec: FP64 vector peak (half the FP32 vector rate)
PEAK_HBM_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E spec peak
PEAK_L2_GBS = 34500.0        # MI355X_MICROARCH.md §L2: aggregate L2 bandwidth (8 XCDs)
PMC_DIRS = [ROOT / "profiles" / "pmc"]   # tools/pmc_traffic.py summaries, one per (workload, kernel) key


def parse(argv: list[str] | None = None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--scene", choices=["random", "mesh", "mixed"], default="random")
    p.add_argument("--precision", choices=["f32", "f64"], default="f32",
                   help="f64: the reference-precision kernel (bit-exact to the reference goldens)")
    p.add_argument("--mesh-level", type=int, default=7, help="procedural blob: 20*4^level triangles")
    p.add_argument("--mesh-obj", default=None, help="OBJ file for --scene mesh/mixed (default: generated)")
    p.add_argument("--tune", default="",
                   help="rt_tuning overrides for experiments, e.g. mesh_lds_stack=8,block=256 (named in config)")
    p.add_argument("--mesh-builder", choices=["host", "gpu", "gpu-lbvh"], default="host",
                   help="triangle BVH: binned SAH on the host, the GPU build (LBVH + treelet restructuring), "
                        "or the plain GPU LBVH")
    p.add_argument("--width", type=int, default=None, help="default: the config's (1920; mixed 3840)")
    p.add_argument("--spp", type=int, default=None, help="default: the config's (256; mesh 128; mixed 1024)")
    p.add_argument("--depth", type=int, default=50)
    p.add_argument("--seed", type=lambda s: int(s, 0), default=0x5EED)
    p.add_argument("--cpu-workers", type=int, default=None,
                   help="reference CPU processes (default: every CPU this process may use)")
    p.add_argument("--cpu-spp", type=int, default=8)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--f64-side-frames", type=int, default=2,
                   help="--precision f32 at N = 1: warm fp64-kernel frames timed after the headline loop "
                        "(the line's f64_side; 0 = off)")
    p.add_argument("--gather", choices=["capi", "torch", "host"], default="capi",
                   help="capi: RCCL ncclGather through the C ABI (rt_gather_shards; default); torch: "
                        "torch.distributed.gather on the nccl (RCCL) backend; host: stage shards through host memory "
                        "and gather over gloo (lets N ranks share one GPU to test the N>1 path; never reported)")
    p.add_argument("--comm-at-1", action="store_true",
                   help="capi: create the communicator and gather even with one rank (tests the RCCL path on 1 GPU)")
    p.add_argument("--dump", default=None, help="rank 0 writes the final 8-bit frame (uint8 HxWx3) to this .npy")
    p.add_argument("--comm-timeout-ms", type=int, default=120000,
                   help="capi: a rank whose peers do not all join the RCCL init within this time gives up "
                        "(then every rank falls back to torch.distributed's gather)")
    p.add_argument("--test-comm-failure", action="store_true",
                   help="tests only: treat the C-ABI communicator as failed (exercises the torch.distributed fallback)")
    p.add_argument("--pmc", nargs="*", default=None,
                   help="PMC traffic summaries (tools/pmc_traffic.py) to take roofline.traffic from "
                        "(default: every profiles/pmc/*.json, the latest round's first: <cfg>_<name>_rNN*.json)")
    a = p.parse_args(argv)
    if a.pmc is None:
        def round_tag(f):   # r03v < r03ah < r03bs < r04f: round, then tag length, then letters
            tag = Path(f).stem.rsplit("_", 1)[-1]
            return tag[:3], len(tag), tag
        a.pmc = sorted((str(f) for d in PMC_DIRS if d.is_dir() for f in d.glob("*.json")), key=round_tag, reverse=True)
    dw, ds = {"random": (1920, 256), "mesh": (1920, 128), "mixed": (3840, 1024)}[a.scene]
    a.width = dw if a.width is None else a.width
    a.spp = ds if a.spp is None else a.spp
    return a


def mesh_world(args, rank: int):
    """Config 3/4 world; the mesh goes through an OBJ file and rt_obj_load like a model
    would (written once per rank into a private temp dir unless --mesh-obj is given)."""
    import tempfile

    from raytracingproject_amd import meshgen, rtweekend, scenes
    path = args.mesh_obj
    tmp = None
    t0 = time.perf_counter()
    if path is None:
        tmp = tempfile.TemporaryDirectory(prefix=f"rt_mesh_r{rank}_")
        path = Path(tmp.name) / f"blob{args.mesh_level}.obj"
        if args.scene == "mesh":
            V, F = meshgen.blob(args.mesh_level, radius=1.6, center=(0.0, 1.0, 0.0))
        else:
            V, F = meshgen.blob(args.mesh_level, radius=meshgen.MESH_RADIUS, center=meshgen.MESH_CENTER)
        meshgen.write_obj(path, V, F)
    t1 = time.perf_counter()
    rtweekend.reset_stream()
    world = scenes.mesh_only(obj_path=path) if args.scene == "mesh" else scenes.mixed(obj_path=path)
    t2 = time.perf_counter()
    if tmp is not None:
        tmp.cleanup()
    return world, {"obj_generate_s": round(t1 - t0, 3), "obj_load_s": round(t2 - t1, 3)}


def host_cpus() -> dict:
    """What this process may run on: logical CPUs of the host, the affinity mask, the
    cgroup CPU quota (a GPU box's share of a large host), and physical cores if known."""
    logical = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = logical
    quota = None
    try:   # cgroup v2: "max 100000" or "<quota> <period>"
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    physical = None
    try:
        ids = set()
        for cpu in os.sched_getaffinity(0):
            t = Path(f"/sys/devices/system/cpu/cpu{cpu}/topology")
            ids.add(((t / "physical_package_id").read_text().strip(), (t / "core_id").read_text().strip()))
        physical = len(ids) or None
    except (OSError, AttributeError):
        pass
    usable = affinity if quota is None else max(1, min(affinity, int(quota + 0.5)))
    return {"host_logical_cpus": logical, "affinity_cpus": affinity, "cgroup_cpu_quota": quota,
            "physical_cores_in_affinity": physical, "usable_cpus": usable}


def cpu_baseline(workers: int | None, spp: int, width: int) -> dict | None:
    """The reference CPU path timed on this host's cores: oracle/_ref/ref_golden (the
    unmodified reference sources, g++) if it was built, else the C restatement.  One
    process per usable CPU (the affinity mask, capped by the cgroup quota), each rendering
    rows j = r (mod workers) of the random-spheres frame at `spp`."""
    ref = ROOT / "oracle" / "_ref" / "ref_golden"
    port = ROOT / "oracle" / "rt_oracle_cli"
    exe, kind = (ref, "reference") if ref.exists() else (port, "port")
    if not exe.exists():
        return None
    cpus = host_cpus()
    workers = cpus["usable_cpus"] if workers is None else max(1, min(workers, cpus["affinity_cpus"]))
    t0 = time.perf_counter()
    procs = [subprocess.Popen([str(exe), "bench", "--width", str(width), "--spp", str(spp), "--rows-mod",
                               str(workers), "--rows-rem", str(r)], stdout=subprocess.PIPE, text=True)
             for r in range(workers)]
    outs = [json.loads(p.communicate()[0]) for p in procs]
    wall = time.perf_counter() - t0
    rays = sum(o["rays"] for o in outs)
    render_s = max(o["seconds"] for o in outs)
    core_s = sum(o["seconds"] for o in outs)
    return {"value": rays / render_s / 1e6, "unit": "Mrays/s", "cores": workers, "kind": kind,
            "sample": f"random-spheres {width}x{outs[0]['H']} @ {spp} spp, rows interleaved over {workers} "
                      f"processes ({rays} primary rays, {core_s:.1f} core-s, scene build excluded)",
            "single_core_mrays": rays / core_s / 1e6, "wall_s": wall,
            "segments_per_primary": sum(o["segments"] for o in outs) / rays, **cpus}


ROOFLINE_KEYS = ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "kernel_ms", "kernel_rank",
                 "flop_per_primary_ray", "primary_rays_per_launch", "traffic_source", "hbm_gbs", "hbm_frac")


def sphere_roofline(f64: bool, coherent: bool, kernel_ms: float, kernel_rank: int, rays_launch: int,
                    traffic: float | None, traffic_src: str | None) -> dict:
    """The roofline object of a sphere line (configs 1-3): FP32 (FP64) VALU with SURVEY.md
    §8(d)'s FLOP_PER_PRIMARY per primary ray over the slowest rank's kernel time, and the
    PMC-measured HBM traffic beside it.  (r06: the survey's 4,170 scene bytes per primary ray,
    a median-split tree model, no longer describes what the grid kernel reads -- dropped.)"""
    achieved = rays_launch * FLOP_PER_PRIMARY / (kernel_ms * 1e-3) / 1e12
    peak = PEAK_FP64_TFLOPS if f64 else PEAK_FP32_TFLOPS
    gbs = traffic / (kernel_ms * 1e-3) / 1e9 if traffic else None
    kernel = ("render_kernel<double, EXACT> (coherent primaries on persistent lanes over the work queue, reference "
              "operation order; samples stored, ordered reduce_kernel)" if f64 else
              "render_kernel<float> (coherent primaries: per-tile camera-ray batches + bounce loop, work queue) + "
              "finalize_kernel" if coherent else "render_kernel<float> (persistent lanes, work queue) + finalize_kernel")
    out = {"bound": "valu", "achieved": round(achieved, 3), "peak": peak, "unit": "TFLOP/s",
           "frac": round(achieved / peak, 4), "traffic": traffic, "kernel": kernel, "kernel_ms": round(kernel_ms, 3),
           "kernel_rank": kernel_rank, "flop_per_primary_ray": FLOP_PER_PRIMARY, "primary_rays_per_launch": rays_launch,
           "traffic_source": traffic_src, "hbm_gbs": round(gbs, 2) if gbs else None,
           "hbm_frac": round(gbs / PEAK_HBM_GBS, 6) if gbs else None}
    assert tuple(out) == ROOFLINE_KEYS
    return out


def mesh_roofline(scene: str, mesh_level: int, rays: int, kernel_ms: float, traffic: float | None,
                  traffic_src: str | None, kernel_rank: int) -> dict:
    """The roofline object of a mesh line (configs 4/5): HBM with the PMC-measured traffic
    (north_star), and beside it the algorithmic work model (measure.WORK_MODEL, the survey's
    probe method re-derived for the level-7 mesh by tests/work_model.py): a VALU fraction,
    the algorithmic mesh bytes against HBM and L2 bandwidth, and traffic / algorithmic bytes
    (the share of the mesh data the rays touch that reaches HBM; the rest is served by
    L2 / Infinity Cache)."""
    from raytracingproject_amd.measure import WORK_MODEL
    s = kernel_ms * 1e-3
    gbs = traffic / s / 1e9 if traffic else None
    rl = {"bound": "hbm", "achieved": round(gbs, 2) if gbs else None, "peak": PEAK_HBM_GBS, "unit": "GB/s",
          "frac": round(gbs / PEAK_HBM_GBS, 5) if gbs else None, "traffic": traffic,
          "kernel": "render_kernel<float, MESH>",
          "achieved_is": "PMC HBM bytes per launch (FETCH x2 + WRITE) / kernel time",
          "kernel_ms": round(kernel_ms, 3), "kernel_rank": kernel_rank, "primary_rays_per_launch": rays,
          "traffic_source": traffic_src}
    wm = WORK_MODEL["c4" if scene == "mesh" else "c5"] if mesh_level == 7 else None
    if wm:
        alg = rays * wm["hbm_bytes_per_primary"]
        tflops = rays * wm["flop_per_primary_ray"] / s / 1e12
        agbs = alg / s / 1e9
        rl.update({
            "work_model": "c4" if scene == "mesh" else "c5",
            "algorithmic_bytes_per_primary": round(wm["hbm_bytes_per_primary"], 2),
            "lds_bytes_per_primary": round(wm["lds_bytes_per_primary"], 2),
            "flop_per_primary_ray": round(wm["flop_per_primary_ray"], 2),
            "algorithmic_bytes_per_launch": round(alg),
            "algorithmic_gbs": round(agbs, 1),
            "algorithmic_hbm_frac": round(agbs / PEAK_HBM_GBS, 4),
            "algorithmic_l2_frac": round(agbs / PEAK_L2_GBS, 4),
            "valu": {"achieved": round(tflops, 3), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(tflops / PEAK_FP32_TFLOPS, 4)},
            "traffic_over_algorithmic": round(traffic / alg, 4) if traffic else None})
    return rl


def f64_side_line(W: int, H: int, spp: int, frame_ms: list[float], kernel: str) -> dict:
    """The reference-precision figure beside an fp32 headline: the
    fp64 kernel (the reference's operation order, bit-exact to its goldens; vec3.h:10 is
    double) timed on warm frames of the same workload, its FLOP model fraction against the
    FP64 vector peak.  frame_ms: render-call times (kernel + ordered reduction) per frame."""
    ms = float(np.mean(frame_ms))
    rays = W * H * spp
    tflops = rays * FLOP_PER_PRIMARY / (ms * 1e-3) / 1e12
    return {"ms_per_frame": round(ms, 3), "frames": len(frame_ms), "mrays": round(rays / (ms * 1e-3) / 1e6, 3),
            "roofline": {"bound": "valu", "achieved": round(tflops, 3), "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(tflops / PEAK_FP64_TFLOPS, 4), "flop_per_primary_ray": FLOP_PER_PRIMARY},
            "kernel": kernel, "timed": "HIP events around rt_render on its stream, after the headline's timed "
                                       "loop (not part of value / ms_per_step)"}


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_command(args, argv: list[str]) -> list[str] | None:
    """`python bench.py --gpus N` (N > 1) outside a launcher: the torch.distributed.run
    command that starts one rank per GPU with the same arguments, or None when this
    process is already a rank (WORLD_SIZE set) or N = 1."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(args.gpus),
            "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
            str(Path(__file__).resolve()), *argv]


def main(argv: list[str] | None = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    cmd = launcher_command(args, argv)
    if cmd is not None:
        # The parent never touches the GPU (no torch, no librt_hip): it starts the ranks as
        # a child process (never exec) and returns the launcher's exit code.
        print(f"bench.py: --gpus {args.gpus} without a launcher; running {' '.join(cmd[1:8])} ...",
              file=sys.stderr, flush=True)
        return subprocess.call(cmd)
    import torch
    import torch.distributed as dist

    from raytracingproject_amd import _native as N
    from raytracingproject_amd import api, rtweekend, scenes
    from raytracingproject_amd.distributed import FrameGather

    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world_size != args.gpus:
        if world_size == 1 and args.gpus > 1:
            print(f"--gpus {args.gpus} needs torch.distributed.run with {args.gpus} processes", file=sys.stderr)
            return 2
    device_index = local_rank if args.gather != "host" else 0
    if args.gather != "host" and local_rank >= torch.cuda.device_count():   # (counting does not init HIP)
        print(f"rank {rank}: local rank {local_rank} but {torch.cuda.device_count()} visible GPU(s); one GPU per "
              "rank is needed (--gather host lets ranks share one GPU, test mode)", file=sys.stderr)
        return 2
    torch.cuda.set_device(device_index)
    dev = torch.device("cuda", device_index)
    if world_size > 1 or args.comm_at_1:
        if args.gather == "torch":
            dist.init_process_group("nccl", device_id=dev)
        else:   # capi: RCCL through the C ABI, gloo only for the id broadcast and barriers
            dist.init_process_group("gloo")
    use_dist = dist.is_initialized()
    capi = args.gather == "capi" and use_dist
    coll_dev = dev if args.gather == "torch" else "cpu"   # the default group's tensors (nccl: device)

    # CPU baseline first (rank 0, N=1 only) so it never overlaps the timed GPU region
    cpu = None
    if rank == 0 and world_size == 1 and not args.no_cpu_baseline and args.scene == "random" and \
            args.precision == "f32":
        cpu = cpu_baseline(args.cpu_workers, args.cpu_spp, args.width)

    # scene + camera: the reference's main.cpp, at the benchmark resolution/spp
    mesh_times = {}
    if args.scene == "random":
        rtweekend.reset_stream()
        world = scenes.random_spheres()
    else:
        world, mesh_times = mesh_world(args, rank)
    cam_api = scenes.main_camera()
    cam_api.image_width, cam_api.samples_per_pixel, cam_api.max_depth = args.width, args.spp, args.depth
    cam = cam_api.native
    W, H, spp, depth = cam.image_width, cam.image_height, args.spp, args.depth

    f64 = args.precision == "f64"
    r = N.Renderer(device_index, args.seed, N.RT_PREC_F64 if f64 else N.RT_PREC_F32)
    tdtype = torch.float64 if f64 else torch.float32
    if args.mesh_builder == "gpu":
        r.set_tuning(mesh_builder=N.RT_MESH_BUILD_GPU)
    elif args.mesh_builder == "gpu-lbvh":
        r.set_tuning(mesh_builder=N.RT_MESH_BUILD_GPU_LBVH)
    overrides = {}
    for kv in filter(None, args.tune.split(",")):
        k, v = kv.split("=")
        overrides[k] = float(v) if "." in v else int(v)
    if overrides:
        r.set_tuning(**overrides)
    S, M, T = api.flatten_scene(world)
    tun = r.tuning()
    t_up = time.perf_counter()
    r.upload_scene(S, M, T if len(T) else None)
    upload_s = time.perf_counter() - t_up
    info = r.scene_info()
    # PMC profiles are only valid for the same launch shape (and, for meshes, the same tree)
    from raytracingproject_amd.measure import pmc_tuning_key
    tuning_key = pmc_tuning_key(tun, info, args.mesh_builder, args.precision)
    lay = N.shard_layout(W, H, rank, world_size)
    fg = FrameGather(torch, dist, W, H, rank, world_size, dev if args.gather != "host" else "cpu", tdtype)
    shard_dev = fg.shard if args.gather != "host" else torch.zeros(fg.elems, dtype=tdtype, device=dev)
    gathered_dev = fg.gathered if args.gather != "host" else None
    if args.gather == "host" and rank == 0:
        gathered_dev = torch.zeros(world_size * fg.elems, dtype=tdtype, device=dev)
    gather_group, gather_note = None, None
    if capi:
        # the RCCL communicator behind the C ABI: rank 0's id reaches the others over gloo
        uid = [N.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        try:
            if args.test_comm_failure:
                raise N.RtError("forced by --test-comm-failure")
            r.comm_init_rank(world_size, rank, uid[0], timeout_ms=args.comm_timeout_ms)
            ok = 1
        except N.RtError as e:   # keep the run: the same RCCL gather through torch.distributed
            print(f"rank {rank}: C-ABI communicator failed ({e}); gathering through torch.distributed",
                  file=sys.stderr)
            ok = 0
        flag = torch.tensor([ok], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if not int(flag.item()):
            if ok:
                r.comm_destroy()
            capi = False
            args.gather = "torch"
            gather_group = dist.new_group(backend="nccl")
            gather_note = "C-ABI RCCL communicator failed; shards gathered by torch.distributed (nccl = RCCL)"
    seg_buf = torch.zeros(lay.max_shard_tiles * 64, dtype=torch.int32, device=dev)
    nbuf = 2   # frames in flight on the host side: frame k's copy overlaps frame k+1's render
    if rank == 0:
        rgb8 = [torch.empty(W * H * 3, dtype=torch.uint8, device=dev) for _ in range(nbuf)]
        host8 = [torch.empty(W * H * 3, dtype=torch.uint8, pin_memory=True) for _ in range(nbuf)]
    copy_done = [None] * nbuf
    # all device work of a step on one non-default torch stream: the render kernel, the
    # RCCL gather (enqueued on the same stream after the render), unshard + quantise to
    # bytes; the kernel-time events are recorded on that same stream.  The copy to host
    # memory runs on a second stream.
    stream = torch.cuda.Stream(dev)
    copy_stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    assert sp != 0
    kernel_events = []
    gather_events = []
    nframe = [0]

    def step(timed: bool, count_segments: bool = False):
        if timed:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        r.render(cam, spp, depth, rank, world_size, shard_dev.data_ptr(),
                 seg_buf.data_ptr() if count_segments else None, sp)
        if timed:
            e1.record(stream)
            kernel_events.append((e0, e1))
        if capi:
            if timed:
                g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                g0.record(stream)
            r.gather_shards(shard_dev.data_ptr(), gathered_dev.data_ptr() if rank == 0 else None, W, H, sp)
            if timed:
                g1.record(stream)
                gather_events.append((g0, g1))
            src = gathered_dev
        elif world_size == 1:
            src = shard_dev
        elif args.gather == "torch":
            src = fg.gather(gather_group)
        else:
            fg.shard.copy_(shard_dev.cpu())
            g = fg.gather()
            if rank == 0:
                gathered_dev.copy_(g.to(dev))
            src = gathered_dev
        if rank == 0:
            b = nframe[0] % nbuf
            if copy_done[b] is not None:
                stream.wait_event(copy_done[b])   # frame buffer b is free once its last copy is done
            r.finish_u8(src.data_ptr(), W, H, world_size, spp, rgb8[b].data_ptr(), sp)
            ready = torch.cuda.Event()
            ready.record(stream)
            copy_stream.wait_event(ready)
            with torch.cuda.stream(copy_stream):
                host8[b].copy_(rgb8[b], non_blocking=True)
            copy_done[b] = torch.cuda.Event()
            copy_done[b].record(copy_stream)
        nframe[0] += 1

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize(dev)
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize(dev)   # every stream: the last frame is in host memory
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    last_frame = (nframe[0] - 1) % nbuf
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in kernel_events])) if kernel_events else float("nan")
    # the gather as enqueued on the render stream after the kernel (it waits for the
    # slowest rank's shard, so on rank 0 it includes the other ranks' lag)
    gather_ms = float(np.mean([a.elapsed_time(b) for a, b in gather_events])) if gather_events else None
    # active pixels of this shard x spp (edge tiles may be partial)
    tiles = np.arange(lay.shard_tiles) * world_size + rank
    tx, ty = tiles % lay.tiles_x, tiles // lay.tiles_x
    rays_shard = int((np.minimum(8, W - tx * 8) * np.minimum(8, H - ty * 8)).sum()) * spp
    per_rank_ms, per_rank_rays = [kernel_ms], [rays_shard]
    if use_dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        km = torch.tensor([kernel_ms, float(rays_shard)], dtype=torch.float64, device=coll_dev)
        allk = [torch.zeros_like(km) for _ in range(world_size)]
        dist.all_gather(allk, km)
        per_rank_ms = [float(x[0].item()) for x in allk]
        per_rank_rays = [int(x[1].item()) for x in allk]
    # the roofline is taken on the SLOWEST rank (its kernel time and its shard's rays), so
    # a slow or throttled GPU shows in the fraction, not only in kernel_ms_per_rank
    slowest = int(np.argmax(per_rank_ms))

    # latency of one frame on its own (render -> host bytes, nothing overlapped)
    torch.cuda.synchronize(dev)
    if use_dist:
        dist.barrier()
    t1 = time.perf_counter()
    step(False)
    torch.cuda.synchronize(dev)
    frame_latency_ms = (time.perf_counter() - t1) * 1e3
    last_frame = (nframe[0] - 1) % nbuf

    # segment statistics (msegments_per_s): one more untimed frame with the per-pixel
    # segment counters on -- instrumentation atomics the timed frames do not carry
    step(False, count_segments=True)
    torch.cuda.synchronize(dev)
    segs_shard = int(seg_buf.to(torch.int64).sum().item())
    if use_dist:
        t = torch.tensor([segs_shard, rays_shard], dtype=torch.int64, device=coll_dev)
        dist.all_reduce(t)
        segs_total, rays_check = map(int, t.tolist())
    else:
        segs_total, rays_check = segs_shard, rays_shard

    # the reference-precision kernel on the same workload, after everything the headline
    # measures (one GPU, fp32 headline, random spheres): f64_side
    f64_side = None
    if not f64 and world_size == 1 and args.f64_side_frames > 0 and args.scene == "random":
        r64 = N.Renderer(device_index, args.seed, N.RT_PREC_F64)
        try:
            r64.upload_scene(S, M, None)
            buf64 = torch.zeros(lay.max_shard_tiles * 64 * 3, dtype=torch.float64, device=dev)
            torch.cuda.synchronize(dev)
            r64.render(cam, spp, depth, 0, 1, buf64.data_ptr(), None, sp)   # warm (module, sample buffer)
            ev = []
            for _ in range(args.f64_side_frames):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                r64.render(cam, spp, depth, 0, 1, buf64.data_ptr(), None, sp)
                b.record(stream)
                ev.append((a, b))
            torch.cuda.synchronize(dev)
            grid64 = bool(r64.scene_info().render_traversal & N.RT_TRAV_GRID)   # f64_kernel 5 (ABI 8)
            k64 = r64.tuning().f64_kernel or (5 if grid64 else 4)
            f64_side = f64_side_line(W, H, spp, [a.elapsed_time(b) for a, b in ev],
                                     f"render_kernel<double, EXACT> f64_kernel {k64} (coherent primaries"
                                     f"{', uniform sphere grid' if grid64 else ''}, reference operation order)"
                                     " + ordered reduce_kernel")
            del buf64
        finally:
            r64.close()

    if rank == 0:
        total_rays = W * H * spp
        assert rays_check == total_rays, (rays_check, total_rays)
        ms_per_step = elapsed / args.steps * 1e3
        value = total_rays * args.steps / elapsed / 1e6
        kernel_ms = per_rank_ms[slowest]
        rays_launch = per_rank_rays[slowest]
        traffic = None
        traffic_src = None
        from raytracingproject_amd.measure import pmc_workload_key
        key = pmc_workload_key(args.scene, args.mesh_level, W, H, spp, world_size)
        for pmc in map(Path, args.pmc):
            if not pmc.exists():
                continue
            d = json.loads(pmc.read_text())
            if key in d.get("per_launch_bytes", {}) and d.get("tuning") in (None, tuning_key):
                traffic = d["per_launch_bytes"][key]
                traffic_src = str(pmc.relative_to(ROOT)) if pmc.is_relative_to(ROOT) else str(pmc)
                break
        workload = {"random": f"random-spheres {W}x{H} @ {spp} spp, depth {depth} (BASELINE.json configs[2])",
                    "mesh": f"OBJ mesh ({info.num_triangles} triangles) + ground {W}x{H} @ {spp} spp, depth {depth} "
                            "(BASELINE.json configs[3])",
                    "mixed": f"485 random spheres + OBJ mesh ({info.num_triangles} triangles) {W}x{H} @ {spp} spp, "
                             f"depth {depth} (BASELINE.json configs[4])"}[args.scene]
        data = ("synthetic: the reference's random-spheres scene (main.cpp, mt19937 default seed), "
                f"per-(pixel,sample) counter RNG seed {args.seed:#x}")
        if args.scene != "random":
            data += f"; procedural blob mesh (raytracingproject_amd/meshgen.py level {args.mesh_level}) read as OBJ"
        headline = args.scene == "random" and (W, H, spp) == (1920, 1080, 256) and not f64
        out = {
            "metric": "Mrays/sec + frame time, random-spheres 1920x1080x256spp" if headline else
                      f"Mrays/sec + frame time, {args.scene} {W}x{H}x{spp}spp" + (" (fp64)" if f64 else ""),
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64" if f64 else "f32",
            "data": data,
            "config": {"workload": workload,
                       "width": W, "height": H, "spp": spp, "max_depth": depth,
                       "primary_rays_per_frame": total_rays, "parallelism": f"tiles{world_size}",
                       "tile": (f"8x8 interleaved, gather to rank 0 over RCCL ({args.gather})" if world_size > 1
                                else "8x8"),
                       **({"tuning_overrides": args.tune} if args.tune else {})},
            "roofline": sphere_roofline(f64, bool(tun.traversal & N.RT_TRAV_COH), kernel_ms, slowest, rays_launch,
                                        traffic, traffic_src),
            "cpu_baseline": cpu,
            "msegments_per_s": round(segs_total * args.steps / elapsed / 1e6, 2),
            "segments_per_primary": round(segs_total / total_rays, 4),
            "frame_latency_ms": round(frame_latency_ms, 3),
            **({"kernel_ms_per_rank": {"min": round(min(per_rank_ms), 3), "max": round(max(per_rank_ms), 3),
                                       "argmax": int(np.argmax(per_rank_ms)),
                                       "all": [round(x, 3) for x in per_rank_ms]},
                "gather_ms": round(gather_ms, 3) if gather_ms is not None else None}
               if (use_dist or capi) else {}),
            "host_frame": f"uint8 {W}x{H}x3, page-locked, copied on a second stream (inside ms_per_step)",
            "scene": {"spheres": info.num_spheres, "bvh_nodes": info.bvh_nodes, "bvh_depth": info.bvh_depth,
                      "bvh_leaves": info.bvh_leaves, "big_spheres": info.big_spheres, "lds_bytes": info.lds_bytes,
                      "triangles": info.num_triangles, "mesh_nodes": info.mesh_nodes, "mesh_depth": info.mesh_depth,
                      "mesh_leaves": info.mesh_leaves, "mesh_builder": args.mesh_builder,
                      "render_block": info.render_block, "render_traversal": info.render_traversal,
                      "render_waves_per_eu": info.render_waves_per_eu,
                      "render_mesh_lds_stack": info.render_mesh_lds_stack, "pmc_key": tuning_key,
                      "grid_res": list(info.grid_res), "grid_entries": info.grid_entries,
                      "upload_s": round(upload_s, 3), **mesh_times},
        }
        if args.scene != "random":
            # mesh configs: the triangle BVH lives in HBM (L2/MALL-cached).  The bound named
            # is HBM (north_star), achieved from the PMC-measured traffic when a profile for
            # this exact workload is on file; beside it the algorithmic work model
            # (measure.WORK_MODEL: bytes and FLOP per primary ray from the survey's probe
            # method, tests/work_model.py) as a VALU fraction, the algorithmic bytes against
            # HBM and L2 bandwidth, and traffic / algorithmic bytes (the share of the mesh
            # data a ray touches that reaches HBM; the rest is served by L2 / Infinity Cache).
            out["roofline"] = mesh_roofline(args.scene, args.mesh_level, rays_launch, kernel_ms, traffic,
                                            traffic_src, slowest)
            out["cpu_baseline"] = None
            out["cpu_baseline_note"] = "the reference has no triangle primitive (SURVEY.md §8(f)1): no CPU path to time"
        if f64_side:
            out["f64_side"] = f64_side
        if cpu:
            out["speedup_vs_cpu"] = round(value / cpu["value"], 1)
        if args.gather == "host":
            out["note"] = "host-staged gather (test mode): not a reportable number"
        if gather_note:
            out["gather_note"] = gather_note
        if args.dump:
            np.save(args.dump, host8[last_frame].numpy().reshape(H, W, 3))
        print(json.dumps(out), flush=True)
    if capi:
        r.comm_destroy()
    r.close()
    if use_dist:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())

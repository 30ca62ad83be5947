"""Host-bound frames and the RCCL gather behind the C ABI, on one MI355X.

* rt_finish_frame_u8 / rt_render_frame_u8 (8-bit frame, the D2H path bench.py times)
  equal rt_quantize's int32 write_color values byte for byte, for any shard count;
* the C-ABI communicator: a single-rank ncclCommInitAll / ncclCommInitRank and
  ncclGather through rt_gather_shards move a shard exactly; two contexts on ONE GPU are
  refused by RCCL with a clean RT_ERR_COMM (the real N>1 run needs one GPU per rank);
* bench.py's default N>1 path (--gather capi: gloo bootstrap + C-ABI RCCL) run as one
  rank with the communicator forced on gives the same frame as the plain N=1 run.
"""
import json
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

from raytracingproject_amd import _native as N
from raytracingproject_amd import api, rtweekend, scenes

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]
SEED = 0x5EED


def random_arrays():
    rtweekend.reset_stream()
    return api.flatten(scenes.random_spheres())


def camera(width, spp):
    cam = scenes.main_camera()
    cam.image_width, cam.samples_per_pixel = width, spp
    return cam.native


def test_u8_frame_equals_write_color():
    import torch
    cam = camera(203, 5)   # ragged edge tiles
    W, H = cam.image_width, cam.image_height
    r = N.Renderer(0, SEED, N.RT_PREC_F32)
    try:
        r.upload_scene(*random_arrays())
        sums, rgb, _ = r.render_frame(cam, 5, 50)
        u8 = r.render_frame_u8(cam, 5, 50)
        assert rgb.min() >= 0 and rgb.max() <= 255
        assert np.array_equal(u8, rgb.astype(np.uint8))
        pinned = N.host_alloc(W * H * 3)   # the direct-copy branch (page-locked caller memory)
        try:
            got = r.render_frame_u8(cam, 5, 50, out=pinned)
            assert np.array_equal(got, u8)
        finally:
            N.host_free(pinned)
        # finish_u8 from 3 stacked shards == the same frame
        n = 3
        lay = N.shard_layout(W, H, 0, n)
        per = lay.max_shard_tiles * 64 * 3
        g = torch.zeros(n * per, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        for sh in range(n):
            r.render(cam, 5, 50, sh, n, g.data_ptr() + sh * per * 4)
        out = torch.zeros(W * H * 3, dtype=torch.uint8, device="cuda")
        r.finish_u8(g.data_ptr(), W, H, n, 5, out.data_ptr())
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy().reshape(H, W, 3), u8)
    finally:
        r.close()


def test_comm_single_rank_gather():
    import torch
    W, H = 64, 40
    lay = N.shard_layout(W, H, 0, 1)
    per = lay.max_shard_tiles * 64 * 3
    shard = torch.arange(per, dtype=torch.float32, device="cuda") * 0.5
    for how in ("all", "rank"):
        r = N.Renderer(0, SEED, N.RT_PREC_F32)
        try:
            if how == "all":
                N.comm_init_all([r])
            else:
                r.comm_init_rank(1, 0, N.comm_unique_id())
            assert r.comm_rank() == (0, 1)
            with pytest.raises(N.RtError):
                N.comm_init_all([r])        # already has one
            got = torch.full((per,), -1.0, dtype=torch.float32, device="cuda")
            torch.cuda.synchronize()
            r.gather_shards(shard.data_ptr(), got.data_ptr(), W, H)
            with pytest.raises(N.RtError):
                r.gather_shards(shard.data_ptr(), None, W, H)   # rank 0 needs a receive buffer
            torch.cuda.synchronize()
            assert torch.equal(got, shard), how
            r.comm_destroy()
            with pytest.raises(N.RtError):
                r.comm_rank()
        finally:
            r.close()


_DUP = r"""
import sys
sys.path.insert(0, %r)
from raytracingproject_amd import _native as N
a, b = N.Renderer(0), N.Renderer(0)
try:
    N.comm_init_all([a, b])
    print("ACCEPTED")
except N.RtError as e:
    print("REFUSED", e)
a.close(); b.close()
"""


def test_comm_two_contexts_on_one_gpu_refused():
    """RCCL needs distinct devices per rank: on a 1-GPU box, a 2-rank ncclCommInitAll over
    device 0 twice must come back as a clean error, not a hang or a crash."""
    r = subprocess.run([sys.executable, "-c", _DUP % str(ROOT)], capture_output=True, text=True, timeout=120,
                       cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    out = r.stdout.strip().splitlines()[-1]
    assert out.startswith("REFUSED") and "RCCL" in out, out


def _bench(extra, out, port=None):
    base = [str(ROOT / "bench.py"), "--steps", "1", "--warmup", "0", "--width", "264", "--spp", "3",
            "--no-cpu-baseline", "--dump", str(out)]
    if port is None:
        cmd = [sys.executable] + base + extra
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr",
               "127.0.0.1", "--master-port", str(port)] + base + extra
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


def test_bench_capi_rccl_path_one_rank(tmp_path):
    _bench([], tmp_path / "plain.npy")
    out = _bench(["--gather", "capi", "--comm-at-1"], tmp_path / "capi.npy", port=29531)
    a, b = np.load(tmp_path / "plain.npy"), np.load(tmp_path / "capi.npy")
    line = json.loads(out.strip().splitlines()[-1])
    # the multi-GPU diagnostics: every rank's kernel time and the gather's own time
    assert line["kernel_ms_per_rank"]["argmax"] == 0 and len(line["kernel_ms_per_rank"]["all"]) == 1
    assert line["gather_ms"] is not None and line["gather_ms"] >= 0
    assert a.dtype == np.uint8 and a.shape == (148, 264, 3)
    assert np.array_equal(a, b)
    # a communicator that fails to come up: the run falls back to torch.distributed's
    # RCCL gather and still produces the same frame
    out = _bench(["--gather", "capi", "--comm-at-1", "--test-comm-failure"], tmp_path / "fallback.npy", port=29533)
    assert np.array_equal(a, np.load(tmp_path / "fallback.npy"))
    assert "gather_note" in out


def test_bench_self_launches_ranks(tmp_path):
    """`python bench.py --gpus 2` with no launcher (the way the driver runs BENCH) starts
    torch.distributed.run itself; two ranks (sharing this box's one GPU through the
    host-staged gather) give the N = 1 frame, and the line carries both ranks' kernel
    times with the roofline taken on the slower one."""
    _bench([], tmp_path / "plain.npy")
    out = _bench(["--gpus", "2", "--gather", "host"], tmp_path / "two.npy")
    line = json.loads(out.strip().splitlines()[-1])
    assert line["n_gpus"] == 2
    per = line["kernel_ms_per_rank"]
    assert len(per["all"]) == 2 and line["roofline"]["kernel_rank"] == per["argmax"]
    assert line["roofline"]["kernel_ms"] == per["max"]
    assert np.array_equal(np.load(tmp_path / "plain.npy"), np.load(tmp_path / "two.npy"))


def test_comm_init_times_out_when_peers_never_join():
    """A rank whose peers never reach the init (one failed before it) gets RT_ERR_COMM
    after the timeout instead of blocking forever (non-blocking ncclCommInitRankConfig,
    polled, then aborted); the context stays usable for a fresh single-rank communicator."""
    import time
    r = N.Renderer(0, SEED, N.RT_PREC_F32)
    try:
        t0 = time.time()
        with pytest.raises(N.RtError, match="timed out|RCCL"):
            r.comm_init_rank(2, 0, N.comm_unique_id(), timeout_ms=3000)
        assert time.time() - t0 < 60
        with pytest.raises(N.RtError):
            r.comm_rank()                     # nothing was kept
        r.comm_init_rank(1, 0, N.comm_unique_id())
        assert r.comm_rank() == (0, 1)
        r.comm_destroy()
    finally:
        r.close()

"""The N>1 bench path on ONE GPU: 2 and 3 ranks (torch.distributed.run) render their
interleaved tile shards on cuda:0, gather them (host-staged gloo instead of RCCL, the
only difference from the 8-GPU run) and rank 0 un-interleaves and quantises: the frame
must equal the 1-rank frame bit for bit."""
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.gpu


def run(n, out, port):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(ROOT / "bench.py"), "--gpus", str(n),
           "--gather", "host", "--steps", "1", "--warmup", "0", "--width", "264", "--spp", "3",
           "--no-cpu-baseline", "--dump", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]


def test_multirank_frame_equals_single_rank(tmp_path):
    run(1, tmp_path / "n1.npy", 29511)
    ref = np.load(tmp_path / "n1.npy")
    for n, port in ((2, 29512), (3, 29513)):
        run(n, tmp_path / f"n{n}.npy", port)
        assert np.array_equal(np.load(tmp_path / f"n{n}.npy"), ref), n

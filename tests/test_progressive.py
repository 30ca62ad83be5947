"""Progressive rendering with snapshots (raytracingproject_amd/progressive.py):
every snapshot is the frame of the samples accumulated so far -- checked against the
oracle's frame of that many samples (samples are keyed per (pixel, sample), so the first
k samples of a progressive run are the k-spp frame of camera.h:40-44): fp64 bit for bit,
fp32 within the F32_* tolerance of test_gpu_parity -- and the last one equals a single
launch of all samples bit for bit."""
import json
import subprocess
import sys

import numpy as np
import pytest

import oracle_bind as O
from raytracingproject_amd import _native as N
from raytracingproject_amd import ppm, progressive, scenes

ROOT = progressive.Path(__file__).resolve().parents[1]


def test_cli_help_without_gpu():
    r = subprocess.run([sys.executable, "-m", "raytracingproject_amd.progressive", "--help"], cwd=ROOT,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "--every" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("precision", [N.RT_PREC_F32, N.RT_PREC_F64])
def test_progressive_snapshots_match_one_launch(tmp_path, precision):
    W, spp, every = 96, 10, 3
    cam = scenes.main_camera()
    cam.image_width = W
    seen, snaps = [], []

    def cb(k, n, im, fs):
        seen.append(n)
        snaps.append((n, im.copy(), fs.copy()))

    img, sums = progressive.render_progressive(progressive.world_for("random", 0), cam, spp, every,
                                               str(tmp_path / "f_%02d.ppm"), precision=precision, callback=cb,
                                               callback_sums=True)
    assert seen == [3, 6, 9, 10]
    from test_gpu_parity import F32_BIAS_LSB, F32_EXACT_FRAC, F32_MAX_LSB, F32_MEAN_LSB, f32_stats
    osc = O.OracleScene("random")
    for n, im, fs in snaps:
        osums, orgb, _ = O.render_counter_full(osc, O.camera(W, n), 0x5EED)
        if precision == N.RT_PREC_F64:
            assert np.array_equal(fs, osums), f"snapshot of {n} samples: sums differ from the oracle"
            assert np.array_equal(im, orgb), f"snapshot of {n} samples: 8-bit image differs from the oracle"
        else:
            st = f32_stats(im, orgb)
            print(n, "samples vs oracle", json.dumps(st))
            assert st["max"] <= F32_MAX_LSB and st["exact"] >= F32_EXACT_FRAC
            assert st["mean_abs"] <= F32_MEAN_LSB and abs(st["bias"]) <= F32_BIAS_LSB
    files = sorted(tmp_path.glob("f_*.ppm"))
    assert len(files) == 4
    assert np.array_equal(ppm.read_ppm(files[-1].read_bytes()), img)
    with N.Renderer(0, 0x5EED, precision) as r:
        from raytracingproject_amd import api, rtweekend
        rtweekend.reset_stream()
        r.upload_scene(*api.flatten(scenes.random_spheres()))
        cam2 = scenes.main_camera()
        cam2.image_width, cam2.samples_per_pixel = W, spp
        ref_sums, ref_rgb, _ = r.render_frame(cam2.native, spp, 50)
    assert np.array_equal(sums, ref_sums) and np.array_equal(img, ref_rgb)


@pytest.mark.gpu
def test_progressive_three_argument_callback():
    """the default callback keeps the three-argument form (k, samples, image);
    the sums come only with callback_sums=True."""
    cam = scenes.main_camera()
    cam.image_width = 32
    seen = []
    img, _ = progressive.render_progressive(progressive.world_for("four", 0), cam, 4, 2,
                                            callback=lambda k, n, im: seen.append((k, n, im.shape)))
    assert seen == [(0, 2, img.shape), (1, 4, img.shape)]

"""Time-binned sphere trees (RT_TRAV_TBIN, rt_bvh.cpp refit_time_bins), on the CPU: the
refitted copies keep the tree's refs and stay conservative -- at every ray time of a bin,
each sphere (placed as the fp32 kernel places it) is inside every child box on its path
(tests/cpp/refit_check.cpp, built here with g++)."""
import subprocess
from pathlib import Path

import numpy as np
import pytest

from raytracingproject_amd import api, rtweekend, scenes

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    out = tmp_path_factory.mktemp("refit") / "refit_check"
    subprocess.run(["g++", "-std=c++17", "-O1", f"-I{ROOT / 'include'}", str(ROOT / "tests/cpp/refit_check.cpp"),
                    str(ROOT / "raytracingproject_amd/csrc/rt_bvh.cpp"), "-o", str(out)], check=True)
    return out


@pytest.mark.parametrize("params", [(6, 1.0, 0.25), (2, 1.0, 1.0), (16, 1.0, 0.1)])
def test_time_bins_are_conservative(checker, tmp_path, params):
    rtweekend.reset_stream()
    spheres, _ = api.flatten(scenes.random_spheres())
    assert int(spheres["moving"].sum()) > 300   # the scene this flag is for: most spheres move
    f = tmp_path / "spheres.bin"
    f.write_bytes(np.ascontiguousarray(spheres).tobytes())
    res = subprocess.run([str(checker), str(f), *map(str, params)], capture_output=True, text=True, check=True)
    words = res.stdout.split()
    assert words[0] == "violations" and int(words[1]) == 0, res.stdout
    assert int(words[3]) > 10
    assert int(words[5]) > int(words[3])   # most child boxes shrink (the spheres move up to 0.5)


def test_time_bins_single_leaf(checker, tmp_path):
    """A scene small enough for one leaf (root with an empty second child)."""
    s = np.zeros(2, dtype=api.flatten(scenes.four_spheres())[0].dtype)
    s["radius"] = 0.5
    s["center"][1] = (2.0, 0.0, 0.0)
    s["center_vec"][0] = (0.0, 0.5, 0.0)
    s["moving"][0] = 1
    f = tmp_path / "spheres.bin"
    f.write_bytes(s.tobytes())
    res = subprocess.run([str(checker), str(f), "6", "1.0", "0.25"], capture_output=True, text=True, check=True)
    words = res.stdout.split()
    assert words[:2] == ["violations", "0"] and int(words[5]) >= 1, res.stdout

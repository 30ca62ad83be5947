"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU; SURVEY.md §5
"Sanitizers" -- the reference's own ASan flags are commented out, CMakeLists.txt:18-23).

`python -m raytracingproject_amd.build --sanitize` builds tests/cpp/sanitize_driver.cpp
with the product's host sources that read untrusted input or build trees (csrc/rt_obj.cpp,
csrc/rt_bvh.cpp) and the oracle (oracle/rt_oracle.c), all -fsanitize=address,undefined
-fno-sanitize-recover=all: any report aborts the driver.  Run here over

* the malformed-OBJ corpus tests/golden/obj_malformed/ (expected.json: the status and
  counts rt_obj_load must give, and how tinyobjloader reads the same file), the three
  parse fixtures, and generated 4,096- and 100,000-corner polygons;
* a mutation fuzzer over those files (byte flips, token splices, truncation, duplicated
  lines, number edge cases), every mutant loaded and, when it loads, its BVHs built and
  checked;
* the random-spheres scene through build_bvh (leaf sizes, front lists) and adversarial
  variants (coincident centres; 1e300 / -1e31 / NaN / inf coordinates must be refused),
  then the oracle's counter- and mt-mode renders.

The corpus is also pinned against the reference's vendored tinyobjloader
(oracle/_ref/obj_dump) where the two agree by design, and run through the shipped
(non-sanitized) librt_hip.so.
"""
import json
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle_bind as O
from raytracingproject_amd import _native as N
from raytracingproject_amd import api, rtweekend, scenes

ROOT = Path(__file__).resolve().parents[1]
CORPUS = ROOT / "tests" / "golden" / "obj_malformed"
EXPECTED = json.loads((CORPUS / "expected.json").read_text()) if (CORPUS / "expected.json").exists() else {}
OBJ_DUMP = O.ORACLE_DIR / "_ref" / "obj_dump"
LOG = ROOT / "raytracingproject_amd" / "build" / "san" / "sanitize.log"   # copied to profiles/ per round


@pytest.fixture(scope="module")
def driver():
    from raytracingproject_amd.build import build_sanitize
    return build_sanitize()


def _run(driver, *args, timeout=600):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(driver), *map(str, args)], capture_output=True, text=True, timeout=timeout, env=env)
    report = "AddressSanitizer" in r.stderr or "runtime error" in r.stderr or "LeakSanitizer" in r.stderr
    with open(LOG, "a") as f:
        f.write(f"$ san_driver {' '.join(Path(str(a)).name for a in args)[:300]}\nrc={r.returncode}\n{r.stdout}"
                f"{r.stderr}\n")
    assert r.returncode == 0 and not report, r.stdout[-3000:] + r.stderr[-5000:]
    return r.stdout


def _polygon(path, n):
    ang = np.linspace(0, 2 * np.pi, n, endpoint=False)
    with open(path, "w") as f:
        for a in ang:
            f.write(f"v {np.cos(a)!r} {np.sin(a)!r} 0\n")
        f.write("f " + " ".join(str(k + 1) for k in range(n)) + "\n")


def test_obj_corpus_under_sanitizers(driver, tmp_path):
    LOG.parent.mkdir(parents=True, exist_ok=True)
    LOG.write_text("# tests/test_sanitize.py: host ASan+UBSan driver (raytracingproject_amd/build.py "
                   "build_sanitize)\n")
    files = sorted(CORPUS.glob("*.obj"))
    assert {f.name for f in files} == set(EXPECTED)
    big4k, big100k = tmp_path / "ngon4096.obj", tmp_path / "ngon100000.obj"
    _polygon(big4k, 4096)
    _polygon(big100k, 100_000)
    fixtures = sorted((ROOT / "tests" / "golden" / "obj").glob("*.obj"))
    out = _run(driver, "obj", *files, *fixtures, big4k, big100k)
    got = {}
    for line in out.splitlines():
        w = line.split()
        if len(w) == 5:
            got[Path(w[0]).name] = list(map(int, w[1:]))
    for name, exp in EXPECTED.items():
        assert got[name] == exp[:4], (name, got[name], exp)
    assert got["ngon4096.obj"] == [N.RT_OK, 4096, 1, 4094]
    assert got["ngon100000.obj"][0] == -4     # RT_ERR_LIMIT: more than RT_OBJ_MAX_FACE_VERTICES corners
    for f in fixtures:
        assert got[f.name][0] == N.RT_OK
    assert "checks failed 0" in out


def test_obj_fuzz_under_sanitizers(driver):
    seeds = sorted(CORPUS.glob("*.obj"))
    seeds = [f for f in seeds if f.stat().st_size < 4096] + sorted((ROOT / "tests" / "golden" / "obj").glob("*.obj"))
    out = _run(driver, "fuzz", "0x5EED", 4000, *seeds)
    w = out.split()
    assert w[:3] == ["fuzz", "iterations", "4000"] and int(w[4]) > 100   # many mutants still load
    assert "checks failed 0" in out


def test_sphere_bvh_and_oracle_under_sanitizers(driver, tmp_path):
    rtweekend.reset_stream()
    S, _ = api.flatten(scenes.random_spheres())
    f = tmp_path / "spheres.bin"
    f.write_bytes(np.ascontiguousarray(S).tobytes())
    out = _run(driver, "spheres", f)
    w = out.split()
    assert w[0] == "spheres" and int(w[1]) == 485 and int(w[3]) == 13 and int(w[5]) == 8
    # uniform sphere grids over every successful tree's order at 3 densities and 1 / 16 time
    # slabs (64 of 78 built: the coincident-centre variant and some grids over the R = 1
    # spheres -- front list off -- are refused), each walked by 2000 random rays (times at
    # slab edges among them) as the kernel walks it, clipped to the ray's slab box, and
    # checked against brute force; every slab box checked to hold its spheres across its slab
    assert int(w[w.index("grids") + 1]) >= 48
    # r06: a quarter of the rays start 10 .. 10^9 cells from the box.  Those within
    # GridHdr::far_o (the only origins a launch that walks the grid can have: rt_abi.cpp
    # grid_reach_ok) walk exactly, in at most res_x + res_y + res_z + 2 steps, never past the
    # pad layers; those beyond are walked too, under a guard, and some of those walks fail --
    # what the bound is for
    walked, beyond, bad = (int(w[w.index(k) + 1]) for k in ("walked", "beyond", "beyond_bad"))
    assert walked > 30000 and beyond > 5000 and bad > 0, (walked, beyond, bad)
    # r06: grids one cell tall in y (main.cpp's field at these densities) are walked the flat
    # way too (TRAV_GFLAT: x and z steps only), equally exact
    assert int(w[w.index("walked_flat") + 1]) > 10000
    assert "checks failed 0" in out


def test_corpus_through_shipped_library():
    """The same statuses and counts through the product's (non-sanitized) librt_hip.so."""
    for name, (st, nv, nf, nt, _) in EXPECTED.items():
        if st != N.RT_OK:
            with pytest.raises(N.RtError):
                N.obj_load(CORPUS / name)
            continue
        V, F, faces = N.obj_load(CORPUS / name)
        assert (len(V), faces, len(F)) == (nv, nf, nt), name
        assert np.isfinite(V).all() and (F >= 0).all() and (F < max(nv, 1)).all()


@pytest.mark.skipif(not OBJ_DUMP.exists(), reason="oracle/_ref/obj_dump not built (needs /root/reference)")
def test_corpus_against_tinyobjloader():
    """Where expected.json says "same", tinyobjloader (the reference's vendored copy, built
    unmodified into oracle/_ref/obj_dump) reads the file identically; the documented
    divergences are checked to be what they say."""
    from test_mesh import assert_same_parse
    for name, (st, *_, how) in EXPECTED.items():
        r = subprocess.run([str(OBJ_DUMP), str(CORPUS / name)], capture_output=True, text=True)
        if how == "same":
            assert r.returncode == 0, name
            assert_same_parse(CORPUS / name, r.stdout)
        elif how == "fails" or how.startswith("fails on"):
            assert r.returncode != 0, name
        else:   # tinyobjloader accepts what rt_obj_load refuses
            assert r.returncode == 0 and st != N.RT_OK, name

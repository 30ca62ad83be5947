"""Mesh path (BASELINE.json configs 4/5): OBJ ingestion, the procedural
mesh, the oracle's triangle restatement, and (GPU) the HIP mesh BVH against the oracle.

Parity status: the reference has no triangle primitive and no OBJ call site, so rendering
parity for meshes is "unpinned" against the reference: the GPU is checked against the
oracle's documented restatement (oracle/rt_oracle.c tri_hit: two-sided Moller-Trumbore,
the sphere path's (0.001, inf) interval).  The OBJ PARSE is pinned against the
reference's vendored tinyobjloader (committed dumps under tests/golden/obj/, plus a live
fuzz against oracle/_ref/obj_dump where it was built).

Tolerances (GPU):
  fp64 -- bit-exact vs the oracle (sums, 8-bit, world.hit counts).
  fp32 -- the sphere path's bounds (test_gpu_parity.F32_*), except that a pixel may differ by
          up to MESH_F32_MAX_LSB where a path grazes a triangle edge: fp32 and fp64 then take
          different branches of the whole path (silhouettes of 1,280 flat facets).
"""
from __future__ import annotations

import subprocess

import numpy as np
import pytest

import oracle_bind as O
from raytracingproject_amd import _native as N
from raytracingproject_amd import api, meshgen, rtweekend, scenes

GOLDEN_OBJ = O.GOLDEN / "obj"
OBJ_DUMP = O.ORACLE_DIR / "_ref" / "obj_dump"
SEED = 0x5EED
MESH_F32_MAX_LSB = 8
MESH_F32_EXACT_FRAC = 0.99
MESH_F32_MEAN_LSB = 0.05


def read_tinyobj_dump(text: str):
    lines = text.splitlines()
    nv = int(lines[0].split()[1])
    V = np.array([[float(x) for x in l.split()] for l in lines[1:1 + nv]], dtype=np.float32).reshape(-1, 3)
    nt = int(lines[1 + nv].split()[1])
    F = np.array([[int(x) for x in l.split()] for l in lines[2 + nv:2 + nv + nt]], dtype=np.int32).reshape(-1, 3)
    return V, F


def assert_same_parse(path, dump_text):
    V, F, _ = N.obj_load(path)
    tv, tf = read_tinyobj_dump(dump_text)
    # tinyobjloader keeps float (real_t); rt_obj_load keeps the file's doubles
    with np.errstate(over="ignore"):   # 1e300 is inf as a float there too
        assert np.array_equal(V.astype(np.float32), tv)
    assert np.array_equal(F, tf)


# ---- OBJ parse vs tinyobjloader ----------------------------------------------------
@pytest.mark.parametrize("case", ["quads", "polygons", "blob2"])
def test_obj_load_matches_tinyobjloader_fixture(case):
    assert_same_parse(GOLDEN_OBJ / f"{case}.obj", (GOLDEN_OBJ / f"{case}.tinyobj.txt").read_text())


def _random_polygon_obj(rng, path):
    """Random soup: star-shaped n-gons (3..9 vertices, convex and concave), random index
    forms, relative indices, CRLF on some lines."""
    lines, nv = [], 0
    for _ in range(40):
        n = int(rng.integers(3, 10))
        c = rng.normal(size=3) * 3
        u, w = rng.normal(size=3), rng.normal(size=3)
        ang = np.sort(rng.uniform(0, 2 * np.pi, n))
        rad = rng.uniform(0.3, 1.0, n)
        tilt = rng.uniform(-0.2, 0.2, n)
        for a, r, t in zip(ang, rad, tilt):
            p = c + r * np.cos(a) * u + r * np.sin(a) * w + t * np.cross(u, w)
            lines.append("v " + " ".join(repr(float(x)) for x in p))
        idx = list(range(nv + 1, nv + n + 1))
        nv += n
        form = rng.integers(0, 4)
        toks = [str(k) if form == 0 else f"{k}/{k}" if form == 1 else f"{k}//1" if form == 2 else str(k - nv - 1)
                for k in idx]
        lines.append("f " + " ".join(toks))
    return "\n".join(l + ("\r" if rng.uniform() < 0.3 else "") for l in lines) + "\n"


@pytest.mark.skipif(not OBJ_DUMP.exists(), reason="oracle/_ref/obj_dump not built (needs /root/reference)")
@pytest.mark.parametrize("seed", range(6))
def test_obj_load_matches_tinyobjloader_live(tmp_path, seed):
    rng = np.random.default_rng(seed)
    p = tmp_path / "soup.obj"
    p.write_text(_random_polygon_obj(rng, p))
    dump = subprocess.run([str(OBJ_DUMP), str(p)], check=True, capture_output=True, text=True).stdout
    assert_same_parse(p, dump)


def test_obj_load_errors(tmp_path):
    with pytest.raises(N.RtError):
        N.obj_load(tmp_path / "missing.obj")
    for bad in ("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 4\n", "v 0 0 0\nf 0 1 1\n", "v 1e999 0 0\n"):
        p = tmp_path / "bad.obj"
        p.write_text(bad)
        with pytest.raises(N.RtError):
            N.obj_load(p)
    p = tmp_path / "empty.obj"
    p.write_text("# nothing\n")
    V, F, nf = N.obj_load(p)
    assert V.shape == (0, 3) and F.shape == (0, 3) and nf == 0
    # a truncated vertex line takes tinyobjloader's defaults (parseV: missing -> 0)
    p.write_text("v 1 2\nv 0 1 0\nv 1 1\nf 1 2 3\n")
    V, F, nf = N.obj_load(p)
    assert V.tolist() == [[1, 2, 0], [0, 1, 0], [1, 1, 0]] and F.tolist() == [[0, 1, 2]]


def test_obj_roundtrip_is_exact(tmp_path):
    V, F = meshgen.blob(3, center=meshgen.MESH_CENTER)
    p = tmp_path / "blob3.obj"
    meshgen.write_obj(p, V, F)
    V2, F2, nf = N.obj_load(p)
    assert nf == len(F) and np.array_equal(V, V2) and np.array_equal(F, F2)


# ---- the procedural mesh -------------------------------------------------------------
@pytest.mark.parametrize("level", [0, 2, 4])
def test_meshgen_blob_is_closed_and_outward(level):
    V, F = meshgen.blob(level, center=(1.0, 2.0, 3.0))
    assert len(F) == 20 * 4 ** level and len(V) == 10 * 4 ** level + 2
    e = np.sort(np.concatenate([F[:, [0, 1]], F[:, [1, 2]], F[:, [2, 0]]]), axis=1)
    _, counts = np.unique(e, axis=0, return_counts=True)
    assert (counts == 2).all(), "every edge shared by exactly two triangles"
    n = np.cross(V[F[:, 1]] - V[F[:, 0]], V[F[:, 2]] - V[F[:, 0]])
    cen = V[F].mean(axis=1) - np.array([1.0, 2.0, 3.0])
    assert ((n * cen).sum(axis=1) > 0).all(), "counter-clockwise seen from outside"


def test_meshgen_is_deterministic():
    a = meshgen.blob(5)
    b = meshgen.blob(5)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_flatten_scene_with_mesh():
    world = scenes.mesh_only(level=2)
    S, M, T = api.flatten_scene(world)
    assert len(S) == 1 and len(T) == 320 and len(M) == 2
    assert (T["mat"] == 1).all() and M[1]["type"] == N.RT_LAMBERTIAN
    with pytest.raises(TypeError):
        api.flatten(world)


# ---- the oracle's triangle restatement (known answers) ------------------------------
def _one_triangle_scene():
    T = np.zeros(1, N.TRIANGLE_DTYPE)
    T[0]["v0"], T[0]["v1"], T[0]["v2"] = (0, 0, 0), (2, 0, 0), (0, 2, 0)
    M = np.zeros(1, N.MATERIAL_DTYPE)
    M[0]["type"], M[0]["albedo"] = N.RT_LAMBERTIAN, (0.5, 0.5, 0.5)
    return np.zeros(0, N.SPHERE_DTYPE), M, T


def _sky(d):
    d = np.asarray(d, float) / np.linalg.norm(d)
    a = 0.5 * (d[1] + 1.0)
    return (1.0 - a) * np.ones(3) + a * np.array([0.5, 0.7, 1.0])


@pytest.mark.parametrize("xy,hit", [((0.5, 0.5), True), ((1.0, 1.0), True), ((0.0, 1.0), True), ((1.5, 0.6), False),
                                    ((-0.01, 0.5), False), ((0.5, -0.01), False)])
@pytest.mark.parametrize("side", [1.0, -1.0])
def test_oracle_triangle_hit_and_miss(xy, hit, side):
    """depth 1: a hit returns black (attenuation * ray_color(depth 0)), a miss the sky."""
    sc = O.OracleScene.from_arrays(*_one_triangle_scene())
    d = (0.0, 0.0, -side)
    ray = [xy[0], xy[1], 3.0 * side, *d, 0.0]
    col, used = O.trace_tape(sc, ray, 1, np.full(16, 0.25))
    if hit:
        assert col == [0.0, 0.0, 0.0] and used == 3   # lambertian: one random_in_unit_sphere try
    else:
        assert np.allclose(col, _sky(d), rtol=0, atol=1e-15) and used == 0


def test_oracle_triangle_tmin_and_normal():
    """A ray starting 0.0005 above the plane misses it (t < 0.001); the bounce off the
    triangle goes along the normal on the side the ray came from."""
    sc = O.OracleScene.from_arrays(*_one_triangle_scene())
    col, used = O.trace_tape(sc, [0.5, 0.5, 0.0005, 0, 0, -1, 0], 1, np.full(16, 0.25))
    assert used == 0
    # depth 2 from below (back face): lambertian bounce = normal(0,0,-1) + unit(p); the
    # tape's point p = (-0.5,-0.5,-0.5) (0.25 -> -0.5), so the bounce heads down-left;
    # its sky colour times the albedo 0.5 is the answer.
    col, used = O.trace_tape(sc, [0.5, 0.5, -2.0, 0, 0, 1, 0], 2, np.full(16, 0.25))
    p = np.array([-0.5, -0.5, -0.5]) / np.sqrt(0.75)
    expect = 0.5 * _sky(np.array([0, 0, -1.0]) + p)
    assert used == 3 and np.allclose(col, expect, rtol=0, atol=1e-12)


# ---- GPU: HIP mesh BVH vs the oracle --------------------------------------------------
MESH_LEVEL_PARITY = 3   # 1,280 triangles: the linear-scan oracle finishes in seconds


def mesh_world(kind: str, level: int = MESH_LEVEL_PARITY):
    if kind == "mesh":
        return scenes.mesh_only(level)
    rtweekend.reset_stream()
    return scenes.mixed(level)


_ARRAYS = {}


def mesh_arrays(kind: str, level: int = MESH_LEVEL_PARITY):
    key = (kind, level)
    if key not in _ARRAYS:
        _ARRAYS[key] = api.flatten_scene(mesh_world(kind, level))
    return _ARRAYS[key]


def main_cam(width, spp, depth=50):
    cam = scenes.main_camera()
    cam.image_width, cam.samples_per_pixel, cam.max_depth = width, spp, depth
    return cam.native


def _render(precision, kind, W, spp, depth=50, level=MESH_LEVEL_PARITY):
    with N.Renderer(0, SEED, precision) as r:
        r.upload_scene(*mesh_arrays(kind, level))
        return r.render_frame(main_cam(W, spp, depth), spp, depth), r.scene_info()


def _oracle(kind, W, spp, stride, depth=50):
    cam = O.camera(W, spp, depth)
    sc = O.OracleScene.from_arrays(*mesh_arrays(kind))
    H = cam.image_height
    k = np.arange(0, W * H, stride)
    ij = np.stack([k % W, k // W], axis=1)
    sums, rgb, segs = O.render_counter(sc, cam, SEED, ij)
    return ij, sums, rgb, segs


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["mesh", "mixed"])
def test_mesh_f64_bit_exact_vs_oracle(kind):
    W, spp = 96, 4
    (sums, rgb, segs), info = _render(N.RT_PREC_F64, kind, W, spp)
    assert info.num_triangles == 20 * 4 ** MESH_LEVEL_PARITY and 0 < info.mesh_depth <= 64
    ij, osums, orgb, osegs = _oracle(kind, W, spp, 5)
    i, j = ij[:, 0], ij[:, 1]
    assert np.array_equal(segs[j, i].astype(np.int64), osegs.astype(np.int64)), "path structure differs"
    bad = ~(sums[j, i] == osums).all(axis=1)
    assert not bad.any(), f"{bad.sum()} of {len(bad)} pixels differ"
    assert np.array_equal(rgb[j, i], orgb)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["mesh", "mixed"])
def test_mesh_f32_within_tolerance_vs_oracle(kind):
    W, spp = 96, 16
    (sums, rgb, segs), _ = _render(N.RT_PREC_F32, kind, W, spp)
    ij, osums, orgb, osegs = _oracle(kind, W, spp, 3)
    i, j = ij[:, 0], ij[:, 1]
    d = rgb[j, i].astype(np.int64) - orgb.astype(np.int64)
    st = {"max": int(np.abs(d).max()), "exact": float((d == 0).mean()), "mean_abs": float(np.abs(d).mean()),
          "bias": float(d.mean())}
    print(kind, st)
    assert st["max"] <= MESH_F32_MAX_LSB and st["exact"] >= MESH_F32_EXACT_FRAC
    assert st["mean_abs"] <= MESH_F32_MEAN_LSB


@pytest.mark.gpu
def test_mesh_trace_tape_vs_oracle():
    """Random rays aimed at the blob (and around it) on explicit tapes, fp64."""
    rng = np.random.default_rng(11)
    S, M, T = mesh_arrays("mixed")
    sc = O.OracleScene.from_arrays(S, M, T)
    c = np.array(meshgen.MESH_CENTER)
    with N.Renderer(0, SEED, N.RT_PREC_F64) as r:
        r.upload_scene(S, M, T)
        for _ in range(48):
            o = c + rng.normal(size=3) * 4 + [0, 2, 0]
            d = (c + rng.normal(size=3) * 0.8) - o
            ray = [*o, *d, rng.uniform()]
            tape = rng.uniform(size=400)
            col, used = r.trace_tape(ray, 50, tape)
            ocol, oused = O.trace_tape(sc, ray, 50, tape)
            assert used == oused and list(col) == ocol


def _inside_cameras(center, W):
    """Six 90-degree cube-face cameras at `center` (covering every direction)."""
    dirs = [(1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1)]
    ups = [(0, 1, 0)] * 2 + [(0, 0, 1)] * 2 + [(0, 1, 0)] * 2
    for d, up in zip(dirs, ups):
        cam = api.camera()
        cam.aspect_ratio, cam.image_width, cam.vfov = 1.0, W, 90.0
        cam.lookfrom = tuple(center)
        cam.lookat = tuple(np.add(center, d))
        cam.vup, cam.defocus_angle, cam.focus_dist = up, 0.0, 1.0
        yield cam.native


@pytest.mark.gpu
@pytest.mark.parametrize("precision", [N.RT_PREC_F64, N.RT_PREC_F32])
def test_mesh_is_watertight_at_full_size(precision):
    """Config-4 mesh (327,680 triangles): every ray from inside the closed blob hits it
    (depth 1 -> black); a sky-coloured pixel is a ray that leaked between triangles."""
    S, M, T = mesh_arrays("mesh", scenes.MESH_LEVEL)
    W = 256
    leaks = 0
    with N.Renderer(0, SEED, precision) as r:
        r.upload_scene(S, M, T)
        info = r.scene_info()
        assert info.num_triangles == 327680 and info.mesh_depth <= 64
        for cam in _inside_cameras((0.0, 1.0, 0.0), W):
            _, rgb, _ = r.render_frame(cam, 4, 1)
            leaks += int((rgb.reshape(-1, 3).sum(axis=1) > 0).sum())
    print("leaked pixels", leaks, "of", 6 * W * W)
    assert leaks == 0   # fp32 too since r05: the watertight edge-function test (rt_device.h tri_wt)


def _edge_rays(V, F, n, spread, seed):
    """Rays from around the blob's centre aimed at random points ON shared edges (the
    worst case for a non-watertight test): (o, d) in fp32, the two triangles of each edge,
    and every triangle around either end of the edge (a point near a vertex may, after
    rounding, lie in another triangle of the vertex's fan), -1 padded."""
    E = np.concatenate([F[:, [0, 1]], F[:, [1, 2]], F[:, [2, 0]]])
    T = np.concatenate([np.arange(len(F))] * 3)
    key = np.sort(E, axis=1)
    order = np.lexsort((key[:, 1], key[:, 0]))
    pair_e, pair_t = key[order][::2], T[order].reshape(-1, 2)
    fan = np.full((len(V), 8), -1, np.int64)
    fill = np.zeros(len(V), np.int64)
    for k, tri in enumerate(F):
        for v in tri:
            fan[v, fill[v]] = k
            fill[v] += 1
    rng = np.random.default_rng(seed)
    sel = rng.integers(0, len(pair_e), n)
    s = rng.uniform(0, 1, n)[:, None]
    p = V[pair_e[sel, 0]] + s * (V[pair_e[sel, 1]] - V[pair_e[sel, 0]])
    o = np.array([0.0, 1.0, 0.0]) + rng.uniform(-spread, spread, (n, 3))
    near = np.concatenate([fan[pair_e[sel, 0]], fan[pair_e[sel, 1]]], axis=1)
    return o.astype(np.float32), (p - o).astype(np.float32), pair_t[sel], near


def _tri_wt_f32(V32, F, tri, o, d):
    """numpy restatement of the fp32 watertight test's inside decision (rt_device.h tri_wt:
    the edge values in unfused fp32 products and differences, as the device computes them;
    inside = every edge value has the sign of d . n, n the facet's normal, or is 0)."""
    P = [V32[F[tri, j]] for j in range(3)]
    A, B, C = (p - o for p in P)

    def cross(u, v):
        return np.stack([u[:, 1] * v[:, 2] - u[:, 2] * v[:, 1], u[:, 2] * v[:, 0] - u[:, 0] * v[:, 2],
                         u[:, 0] * v[:, 1] - u[:, 1] * v[:, 0]], 1)

    def dot(a, b):
        return (a[:, 0] * b[:, 0] + a[:, 1] * b[:, 1]) + a[:, 2] * b[:, 2]
    ea, eb, ec = dot(d, cross(B, C)), dot(d, cross(C, A)), dot(d, cross(A, B))
    V = [V32[F[tri, j]].astype(np.float64) for j in range(3)]
    nd = dot(np.cross(V[1] - V[0], V[2] - V[0]).astype(np.float32), d)   # TriF::n: fp64, rounded
    s = np.sign(nd)[:, None]
    return (np.stack([ea, eb, ec], 1) * s >= 0).all(1) & (nd != 0)


@pytest.mark.parametrize("spread", [0.0, 0.3, 1.0])
def test_fp32_edge_test_leaves_no_gap(spread):
    """CPU: rays through points on the shared edges of the config-4 blob (level 5 here) --
    where fp32 Moller-Trumbore with the old 2^-20 widening missed both triangles for ~8 %
    of such rays -- hit at least one of the two triangles with the watertight test: each
    edge's value is computed identically (up to sign) by both, so no point falls between."""
    V, F = meshgen.blob(5, radius=1.6, center=(0.0, 1.0, 0.0))
    V32 = V.astype(np.float32)
    o, d, tt, near = _edge_rays(V, F, 200_000, spread, seed=int(spread * 10))
    # a ray through a silhouette edge (the two triangles facing it from opposite sides:
    # origins outside the blob, spread 1.0) may rightly touch neither; the others cross
    # the surface at the edge and must hit one of the triangles around it
    n = [np.cross(V[F[tt[:, j], 1]] - V[F[tt[:, j], 0]], V[F[tt[:, j], 2]] - V[F[tt[:, j], 0]]) for j in (0, 1)]
    crossing = np.sign((n[0] * d).sum(1)) == np.sign((n[1] * d).sum(1))
    h = np.zeros(len(o), bool)
    with np.errstate(all="ignore"):
        for j in range(near.shape[1]):
            k = near[:, j]
            h |= (k >= 0) & _tri_wt_f32(V32, F, np.maximum(k, 0), o, d)
    assert crossing.mean() > 0.99
    bad = crossing & ~h
    assert not bad.any(), f"{bad.sum()} of {crossing.sum()} edge rays fall between two triangles"


@pytest.mark.gpu
@pytest.mark.parametrize("builder", [N.RT_MESH_BUILD_HOST, N.RT_MESH_BUILD_GPU, N.RT_MESH_BUILD_GPU_LBVH])
def test_fp32_trace_rays_watertight(builder):
    """8M random rays from inside the closed config-4 blob through rt_trace_rays in fp32:
    every one hits (the blob, or the ground where it cuts the blob).  r04's Moller-Trumbore
    leaked 39 of 33.5M such rays with either tree (tools/leak_probe.py, r05a)."""
    S, M, T = mesh_arrays("mesh", scenes.MESH_LEVEL)
    rng = np.random.default_rng(7)
    misses = 0
    with N.Renderer(0, SEED, N.RT_PREC_F32) as r:
        r.set_tuning(mesh_builder=builder)
        r.upload_scene(S, M, T)
        for _ in range(4):
            n = 1 << 21
            dd = rng.normal(size=(n, 3))
            o = np.array([0.0, 1.0, 0.0]) + rng.uniform(-0.3, 0.3, (n, 3))
            rays = np.concatenate([o, dd, np.zeros((n, 1))], axis=1).astype(np.float32)
            misses += int((r.trace_rays_host(rays)["id"] == -1).sum())
    assert misses == 0


@pytest.mark.gpu
def test_mesh_tuning_variants_are_identical():
    S, M, T = mesh_arrays("mixed")
    cam = main_cam(128, 4)
    frames = []
    with N.Renderer(0, SEED, N.RT_PREC_F32) as r:
        r.upload_scene(S, M, T)
        # (mesh block, mesh_waves_per_eu, traversal): 600 = the default flags (the if-if loop
        # is added: 8792 with LDS item sums, or 8920 where they would cost occupancy), 728
        # forces no sums, 8 one path per lane, + 16384 the while-while loop of rounds 1-3;
        # mesh_waves_per_eu 6 = the <= 80-VGPR kernels, 0 = the compiler's budget, -1 = auto
        W = N.RT_TRAV_MWHILE
        cases = [(512, 0, 8), (256, 6, 600), (512, 6, 600), (768, 6, 600), (256, 6, 728), (512, 6, 728),
                 (768, 6, 728), (256, 0, 600), (512, 0, 728 | W), (512, 0, 600 | W), (256, 6, 600 | 8192),
                 (0, -1, 600),
                 # the sphere grid (r05), with its flat walk (the default on this field, r06) or its 3-D one
                 (768, 6, N.RT_TRAV_DEFAULT), (768, 6, N.RT_TRAV_DEFAULT | N.RT_TRAV_G3D),
                 (512, 6, N.RT_TRAV_DEFAULT), (512, 6, N.RT_TRAV_DEFAULT | N.RT_TRAV_G3D)]
        for block, wpe, trav in cases:
            r.set_tuning(block=512 if trav == 8 else 1024, waves_per_eu=8, mesh_block=block,
                         mesh_waves_per_eu=wpe, traversal=trav)   # (block: a sphere kernel must exist too)
            info = r.scene_info()
            assert (block == 0 or info.render_block == block) and (wpe < 0 or info.render_waves_per_eu == wpe)
            assert bool(info.render_traversal & N.RT_TRAV_MIFIF) == (trav not in (8, 728 | W, 600 | W))
            # (the flat walk wherever the plan walks this field's grid and the 3-D walk is not
            # asked for; at 512 threads the plan prefers the sphere tree)
            grid = bool(info.render_traversal & N.RT_TRAV_GRID)
            assert grid or block != 768 or trav & N.RT_TRAV_GRID == 0, (block, trav)
            assert bool(info.render_traversal & N.RT_TRAV_GFLAT) == (grid and not trav & N.RT_TRAV_G3D), (block, trav)
            frames.append(r.render_frame(cam, 4, 50)[0])
        for mst in (0, 1, 5, 40, -1):                          # LDS / scratch stack split (-1: auto)
            r.set_tuning(block=512, mesh_block=512, mesh_waves_per_eu=0, traversal=8, mesh_lds_stack=mst)
            assert mst < 0 or r.scene_info().render_mesh_lds_stack == mst
            frames.append(r.render_frame(cam, 4, 50)[0])
        r.set_tuning(mesh_lds_stack=12)
        r.set_tuning(mesh_block=256, block=1024, waves_per_eu=8, traversal=88)   # no such mesh kernel
        with pytest.raises(N.RtError):
            r.render_frame(cam, 4, 50)
        # 512 threads at the compiler's budget has only the while-while kernel: without 16384
        # that is refused, not run in place of the if-if loop
        r.set_tuning(mesh_block=512, mesh_waves_per_eu=0, traversal=600)
        with pytest.raises(N.RtError):
            r.render_frame(cam, 4, 50)
        r.set_tuning(traversal=600 | W)
        assert r.scene_info().render_traversal == 728
        r.render_frame(cam, 4, 50)
        with pytest.raises(N.RtError):
            r.set_tuning(mesh_waves_per_eu=5)   # only -1 (auto), 0 and 6
        with pytest.raises(N.RtError):
            r.set_tuning(mesh_lds_stack=-2)
        with pytest.raises(N.RtError):   # quantised mesh nodes: measured slower in r05, removed
            r.set_tuning(traversal=600 | N.RT_TRAV_MQ)
    for f in frames[1:]:
        assert np.array_equal(f, frames[0])


@pytest.mark.gpu
def test_mesh_six_wave_kernel_is_identical():
    """The 6-wave mesh kernel (mesh_waves_per_eu = 6: <= 80 VGPRs, 256-thread if-if
    kernel; the auto default picks it) renders the mesh-only scene bit for bit like the
    5-wave one of rounds 1-3, and the plan really runs each (scene_info)."""
    S, M, T = mesh_arrays("mesh")
    cam = main_cam(128, 4)
    out = []
    with N.Renderer(0, SEED, N.RT_PREC_F32) as r:
        r.upload_scene(S, M, T)
        for wpe in (0, 6, 0, -1):
            r.set_tuning(mesh_waves_per_eu=wpe, mesh_block=256)
            info = r.scene_info()
            assert info.render_block == 256 and info.render_waves_per_eu == (wpe if wpe >= 0 else 6)
            out.append(r.render_frame(cam, 4, 50))
    for f in out[1:]:
        assert np.array_equal(f[0], out[0][0]) and np.array_equal(f[2], out[0][2])


@pytest.mark.gpu
def test_mesh_auto_plan_matches_the_measured_best():
    """The default plan (mesh_block, mesh_waves_per_eu and mesh_lds_stack all auto) runs
    the kernels the A/Bs measured fastest: C4's mesh-only scene the 6-wave 256-thread
    kernel with LDS item sums and all 12 stack entries in LDS (six workgroups per CU), the
    mixed scene (C5 geometry: the sphere scene shares LDS) the 6-wave 768-thread kernel
    with the LDS item sums and, its spheres in the uniform grid (no sphere traversal stack),
    two workgroups per CU (the same 24 waves as r04's three 512-thread workgroups without
    either; r05: 59.0 -> 53.4 ms at 4K @ 32 with the grid) and, since r06, its mesh stack all
    in scratch (1,568 -> 1,526 ms at 4K @ 1024 against the 5 LDS entries of r05) and the
    grid's flat walk (74328 + 131072: the grid is one cell tall in y; C5 geometry -1.8 %)."""
    for kind, want in (("mesh", (256, 8792, 6, 12)), ("mixed", (768, 74328 | N.RT_TRAV_GFLAT, 6, 0))):
        S, M, T = mesh_arrays(kind)
        with N.Renderer(0, SEED, N.RT_PREC_F32) as r:
            r.upload_scene(S, M, T)
            i = r.scene_info()
            got = (i.render_block, i.render_traversal, i.render_waves_per_eu, i.render_mesh_lds_stack)
            assert got == want, (kind, got, i.lds_bytes)


@pytest.mark.gpu
def test_mesh_kernel_plan_picks_if_if_loop():
    """fp32 mesh scenes run the if-if mesh loop (8192 added to the tuning's flags) unless
    the while-while loop (16384) is asked for; sphere scenes and the fp64 path never carry
    the mesh flags; 8192 with 16384 and the removed LDS tree top (4096) are refused."""
    S, M, T = mesh_arrays("mixed")
    with N.Renderer(0, SEED, N.RT_PREC_F32) as r:
        r.upload_scene(S, M, T)
        assert r.scene_info().render_traversal & N.RT_TRAV_MIFIF
        r.set_tuning(traversal=N.RT_TRAV_DEFAULT | N.RT_TRAV_MWHILE)
        t = r.scene_info().render_traversal
        assert not t & (N.RT_TRAV_MIFIF | N.RT_TRAV_MWHILE)
        with pytest.raises(N.RtError):
            r.set_tuning(traversal=N.RT_TRAV_DEFAULT | N.RT_TRAV_MTOP)
        with pytest.raises(N.RtError):
            r.set_tuning(traversal=N.RT_TRAV_DEFAULT | N.RT_TRAV_MIFIF | N.RT_TRAV_MWHILE)
    with N.Renderer(0, SEED, N.RT_PREC_F32) as r:   # the same spheres without the mesh
        r.set_tuning(traversal=N.RT_TRAV_DEFAULT | N.RT_TRAV_MIFIF)
        r.upload_scene(S, M)
        # (the field's grid is one cell tall in y: the flat walk is added, r06)
        assert r.scene_info().render_traversal == N.RT_TRAV_DEFAULT | N.RT_TRAV_GFLAT
    with N.Renderer(0, SEED, N.RT_PREC_F64) as r:
        r.upload_scene(S, M, T)
        assert not r.scene_info().render_traversal & (N.RT_TRAV_MIFIF | N.RT_TRAV_MWHILE)


@pytest.mark.gpu
def test_mesh_full_size_fp32_tracks_fp64():
    """Config-5 geometry (485 spheres + 327,680 triangles) at reduced resolution: the fp32
    frame is deterministic and within the 8-bit tolerance of the fp64 frame."""
    W, spp = 160, 8
    (s32, rgb32, _), _ = _render(N.RT_PREC_F32, "mixed", W, spp, level=scenes.MESH_LEVEL)
    (s32b, _, _), _ = _render(N.RT_PREC_F32, "mixed", W, spp, level=scenes.MESH_LEVEL)
    (_, rgb64, _), _ = _render(N.RT_PREC_F64, "mixed", W, spp, level=scenes.MESH_LEVEL)
    assert np.array_equal(s32, s32b)
    d = rgb32.astype(np.int64) - rgb64.astype(np.int64)
    print("f32 vs f64", int(np.abs(d).max()), float((d == 0).mean()), float(np.abs(d).mean()))
    assert float(np.abs(d).mean()) <= 4 * MESH_F32_MEAN_LSB and abs(float(d.mean())) <= 0.05


# ---- GPU (LBVH) mesh BVH build -------------------------------------------------------
def _render_with(builder, precision, arrays, W, spp, depth=50):
    with N.Renderer(0, SEED, precision) as r:
        r.set_tuning(mesh_builder=builder)
        r.upload_scene(*arrays)
        return r.render_frame(main_cam(W, spp, depth), spp, depth), r.scene_info()


GPU_BUILDERS = [N.RT_MESH_BUILD_GPU, N.RT_MESH_BUILD_GPU_LBVH]   # (treelet-restructured, plain LBVH)


@pytest.mark.gpu
@pytest.mark.parametrize("builder", GPU_BUILDERS)
@pytest.mark.parametrize("kind", ["mesh", "mixed"])
@pytest.mark.parametrize("precision", [N.RT_PREC_F64, N.RT_PREC_F32])
def test_gpu_bvh_build_renders_like_host_build(kind, precision, builder):
    """The GPU trees (r06: the LBVH restructured by treelets, and the plain LBVH) differ from
    the host SAH tree, the closest hits do not: in fp64 the frames and world.hit counts are
    identical.  In fp32 two triangles sharing an edge can return the same rounded t for a ray
    through that edge, and then the one visited first wins (strict t < t_max, as
    hittable_list::hit); the frames agree within the mesh fp32 tolerance."""
    arrays = mesh_arrays(kind)
    (s_h, rgb_h, g_h), info_h = _render_with(N.RT_MESH_BUILD_HOST, precision, arrays, 96, 4)
    (s_g, rgb_g, g_g), info_g = _render_with(builder, precision, arrays, 96, 4)
    assert info_g.num_triangles == info_h.num_triangles and info_g.mesh_nodes > 0
    if precision == N.RT_PREC_F64:
        assert np.array_equal(g_h, g_g) and np.array_equal(s_h, s_g)
    else:
        d = rgb_h.astype(np.int64) - rgb_g.astype(np.int64)
        print(kind, "host vs GPU tree, fp32:", int(np.abs(d).max()), float((d == 0).mean()))
        assert np.abs(d).max() <= MESH_F32_MAX_LSB and (d == 0).mean() >= MESH_F32_EXACT_FRAC


@pytest.mark.gpu
@pytest.mark.parametrize("builder", GPU_BUILDERS)
@pytest.mark.parametrize("n_tris", [1, 2, 3, 5, 17])
def test_gpu_bvh_build_small_and_degenerate(n_tris, builder):
    """Tiny meshes (single-leaf roots) and coincident centroids (equal Morton codes): fp64
    GPU-built render vs the oracle, bit-exact."""
    rng = np.random.default_rng(n_tris)
    T = np.zeros(n_tris, N.TRIANGLE_DTYPE)
    base = np.array([0.0, 1.0, 0.0])
    for k in range(n_tris):
        # half of them share one centroid (same Morton code), the rest are scattered
        off = np.zeros(3) if k % 2 == 0 else rng.normal(size=3) * 0.5
        a = rng.normal(size=3) * 0.6
        b = rng.normal(size=3) * 0.6
        T[k]["v0"], T[k]["v1"], T[k]["v2"] = base + off + a, base + off + b, base + off - a - b
    T["mat"] = 1
    S = np.zeros(1, N.SPHERE_DTYPE)
    S[0]["center"], S[0]["radius"], S[0]["mat"] = (0, -1000, 0), 1000, 0
    M = np.zeros(2, N.MATERIAL_DTYPE)
    M[0]["type"], M[0]["albedo"] = N.RT_LAMBERTIAN, (0.5, 0.5, 0.5)
    M[1]["type"], M[1]["albedo"], M[1]["fuzz"] = N.RT_METAL, (0.8, 0.7, 0.6), 0.1
    W, spp = 48, 2
    (sums, _, segs), info = _render_with(builder, N.RT_PREC_F64, (S, M, T), W, spp)
    assert info.num_triangles == n_tris
    cam = O.camera(W, spp)
    H = cam.image_height
    k = np.arange(0, W * H, 3)
    ij = np.stack([k % W, k // W], axis=1)
    osums, _, osegs = O.render_counter(O.OracleScene.from_arrays(S, M, T), cam, SEED, ij)
    assert np.array_equal(segs[ij[:, 1], ij[:, 0]].astype(np.int64), osegs.astype(np.int64))
    assert np.array_equal(sums[ij[:, 1], ij[:, 0]], osums)


@pytest.mark.gpu
@pytest.mark.parametrize("builder", [N.RT_MESH_BUILD_HOST] + GPU_BUILDERS)
@pytest.mark.parametrize("n_tris", [1, 2, 3, 17])
def test_if_if_mesh_loop_small_meshes(n_tris, builder):
    """fp32 tiny meshes (a root holding one leaf, empty child slots in the mesh box union,
    coincident centroids): the if-if loop with its mesh-box pre-test renders the
    while-while loop's frame and segment counts bit for bit, with either builder."""
    rng = np.random.default_rng(100 + n_tris)
    T = np.zeros(n_tris, N.TRIANGLE_DTYPE)
    for k in range(n_tris):
        off = np.zeros(3) if k % 2 == 0 else rng.normal(size=3) * 0.5
        a, b = rng.normal(size=3) * 0.6, rng.normal(size=3) * 0.6
        c = np.array([0.0, 1.0, 0.0]) + off
        T[k]["v0"], T[k]["v1"], T[k]["v2"] = c + a, c + b, c - a - b
    T["mat"] = 1
    S = np.zeros(1, N.SPHERE_DTYPE)
    S[0]["center"], S[0]["radius"], S[0]["mat"] = (0, -1000, 0), 1000, 0
    M = np.zeros(2, N.MATERIAL_DTYPE)
    M[0]["type"], M[0]["albedo"] = N.RT_LAMBERTIAN, (0.5, 0.5, 0.5)
    M[1]["type"], M[1]["albedo"], M[1]["fuzz"] = N.RT_METAL, (0.8, 0.7, 0.6), 0.1
    out = []
    for trav in (N.RT_TRAV_DEFAULT, N.RT_TRAV_DEFAULT | N.RT_TRAV_MWHILE):
        with N.Renderer(0, SEED, N.RT_PREC_F32) as r:
            r.set_tuning(mesh_builder=builder, traversal=trav)
            r.upload_scene(S, M, T)
            assert bool(r.scene_info().render_traversal & N.RT_TRAV_MIFIF) == (trav == N.RT_TRAV_DEFAULT)
            sums, _, segs = r.render_frame(main_cam(48, 4), 4, 50)
            out.append((sums, segs))
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])


@pytest.mark.gpu
@pytest.mark.parametrize("precision", [N.RT_PREC_F64, N.RT_PREC_F32])
def test_gpu_bvh_build_full_size_watertight(precision):
    """Config-4 mesh (327,680 triangles) built on the GPU: every ray from inside hits."""
    import time
    S, M, T = mesh_arrays("mesh", scenes.MESH_LEVEL)
    W = 256
    leaks = 0
    with N.Renderer(0, SEED, precision) as r:
        r.set_tuning(mesh_builder=N.RT_MESH_BUILD_GPU)
        r.upload_scene(S, M, T)          # warm (module load, scratch)
        t0 = time.perf_counter()
        r.upload_scene(S, M, T)
        t_gpu = time.perf_counter() - t0
        info = r.scene_info()
        for cam in _inside_cameras((0.0, 1.0, 0.0), W):
            _, rgb, _ = r.render_frame(cam, 4, 1)
            leaks += int((rgb.reshape(-1, 3).sum(axis=1) > 0).sum())
        r.set_tuning(mesh_builder=N.RT_MESH_BUILD_HOST)
        t0 = time.perf_counter()
        r.upload_scene(S, M, T)
        t_host = time.perf_counter() - t0
    print(f"upload+build: GPU (LBVH + treelets) {t_gpu * 1e3:.1f} ms ({info.mesh_nodes} nodes, depth "
          f"{info.mesh_depth}), host SAH {t_host * 1e3:.1f} ms; leaked {leaks}")
    assert info.num_triangles == 327680 and 0 < info.mesh_depth <= 21
    assert leaks == 0
    assert t_gpu < 0.05   # (the build within 20 ms; upload of the arrays included)


@pytest.mark.gpu
def test_triangles_only_scene_and_shards():
    """No spheres at all (empty sphere BVH and big-sphere list), only a mesh: fp64 matches
    the oracle, and a 3-way shard split rendered as accumulated sample ranges equals the
    one-shard frame (fp32)."""
    import torch
    S0, M, T = mesh_arrays("mesh")
    S = np.zeros(0, N.SPHERE_DTYPE)
    W, spp = 64, 4
    (sums, _, segs), info = _render_with(N.RT_MESH_BUILD_HOST, N.RT_PREC_F64, (S, M, T), W, spp)
    assert info.num_spheres == 0 and info.big_spheres == 0 and info.num_triangles == len(T)
    cam = O.camera(W, spp)
    H = cam.image_height
    k = np.arange(0, W * H, 4)
    ij = np.stack([k % W, k // W], axis=1)
    osums, _, osegs = O.render_counter(O.OracleScene.from_arrays(S, M, T), cam, SEED, ij)
    assert np.array_equal(sums[ij[:, 1], ij[:, 0]], osums)
    with N.Renderer(0, SEED, N.RT_PREC_F32) as r:
        r.upload_scene(S, M, T)
        ncam = main_cam(W, spp)
        ref, _, ref_segs = r.render_frame(ncam, spp, 50)
        lay = N.shard_layout(W, ncam.image_height, 0, 3)
        per = lay.max_shard_tiles * 64
        buf = torch.zeros(3 * per * 3, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        for sh in range(3):
            for i, (b, n) in enumerate([(0, 1), (1, 3)]):
                r.render_range(ncam, b, n, 50, sh, 3, i > 0, buf.data_ptr() + sh * per * 3 * 4)
        frame = torch.empty(ncam.image_height * W * 3, dtype=torch.float32, device="cuda")
        r.unshard(buf.data_ptr(), W, ncam.image_height, 3, frame.data_ptr())
        torch.cuda.synchronize()
        assert np.array_equal(frame.cpu().numpy().reshape(ref.shape), ref)


# ---- configs 4 and 5 at their own frame sizes --------------------------------------
FULL_CONFIGS = {
    # BASELINE.json configs[3]: OBJ mesh (327,680 triangles) + ground, 1920x1080 @ 128 spp
    "mesh": (1920, 128),
    # BASELINE.json configs[4]: 485 random spheres + the mesh, 3840x2160 @ 1024 spp, depth 50
    "mixed": (3840, 1024),
}


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["mesh", "mixed"])
def test_full_frame_config(kind):
    """C4 / C5 rendered at full frame size and spp through the fp32 kernel (C5 is the
    workload the 8-GPU split targets; one GPU renders it in a few seconds):
      * every pixel finite, and a second render identical bit for bit (sums, world.hit);
      * the 8-shard split (tiles t -> shard t % 8, as the 8-GPU run deals them), rendered
        shard by shard and un-interleaved, equals the 1-shard frame bit for bit;
      * segments per primary within 2 % of the fp64 kernel's on the tiles below;
      * 16 tiles (1,024 pixels) rendered by the fp64 kernel -- shard t of num_tiles is
        exactly tile t -- agree with the fp32 frame within the mesh fp32 tolerance."""
    import torch
    W, spp = FULL_CONFIGS[kind]
    S, M, T = mesh_arrays(kind, scenes.MESH_LEVEL)
    cam = main_cam(W, spp)
    H = cam.image_height
    lay1, lay8 = N.shard_layout(W, H, 0, 1), N.shard_layout(W, H, 0, 8)
    n1, n8 = lay1.max_shard_tiles * 64, lay8.max_shard_tiles * 64
    with N.Renderer(0, SEED, N.RT_PREC_F32) as r:
        r.upload_scene(S, M, T)
        assert r.scene_info().num_triangles == 327680
        a = torch.zeros(n1 * 3, dtype=torch.float32, device="cuda")
        b = torch.zeros_like(a)
        sa = torch.zeros(n1, dtype=torch.int32, device="cuda")
        sb = torch.zeros_like(sa)
        g = torch.zeros(8 * n8 * 3, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        r.render(cam, spp, 50, 0, 1, a.data_ptr(), sa.data_ptr())
        ms = r.last_kernel_ms()
        r.render(cam, spp, 50, 0, 1, b.data_ptr(), sb.data_ptr())
        for sh in range(8):
            r.render(cam, spp, 50, sh, 8, g.data_ptr() + sh * n8 * 3 * 4)
        f1 = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
        f8 = torch.zeros_like(f1)
        r.unshard(a.data_ptr(), W, H, 1, f1.data_ptr())
        r.unshard(g.data_ptr(), W, H, 8, f8.data_ptr())
        rgb = torch.zeros(W * H * 3, dtype=torch.int32, device="cuda")
        r.quantize(f1.data_ptr(), W, H, spp, rgb.data_ptr())
        torch.cuda.synchronize()
        assert torch.isfinite(a).all()
        assert torch.equal(a, b) and torch.equal(sa, sb), "fp32 frame not deterministic"
        assert torch.equal(f1, f8), f"8-shard split differs at {(f1 != f8).sum().item()} values"
        frame = f1.cpu().numpy().reshape(H, W, 3)
        rgb32 = rgb.cpu().numpy().reshape(H, W, 3)
        segs32 = sa.cpu().numpy().astype(np.int64)
    print(f"{kind} {W}x{H}@{spp}: fp32 kernel {ms:.1f} ms, {W * H * spp / ms / 1e3:.0f} Mrays/s")

    # fp64 on 16 tiles spread over the frame (rows of tiles across the image)
    num_tiles = lay1.num_tiles
    tiles = np.linspace(num_tiles // 17, num_tiles - 1 - num_tiles // 17, 16).astype(int)
    with N.Renderer(0, SEED, N.RT_PREC_F64) as r:
        r.upload_scene(S, M, T)
        buf = torch.zeros(64 * 3, dtype=torch.float64, device="cuda")
        segs = torch.zeros(64, dtype=torch.int32, device="cuda")
        sums64, seg64, seg32 = [], 0, 0
        for t in tiles:
            torch.cuda.synchronize()
            r.render(cam, spp, 50, int(t), num_tiles, buf.data_ptr(), segs.data_ptr())
            torch.cuda.synchronize()
            sums64.append(buf.cpu().numpy().reshape(64, 3).copy())
            seg64 += int(segs.sum().item())
            seg32 += int(segs32[t * 64:(t + 1) * 64].sum())
    tx, ty = tiles % lay1.tiles_x, tiles // lay1.tiles_x
    lane = np.arange(64)
    xs = (tx[:, None] * 8 + lane % 8).ravel()
    ys = (ty[:, None] * 8 + lane // 8).ravel()
    s64 = np.concatenate(sums64)
    ok = (xs < W) & (ys < H)
    x = np.sqrt(s64[ok] / spp)
    q64 = (256 * np.clip(x, 0.0, 0.999)).astype(np.int64)
    d = rgb32[ys[ok], xs[ok]].astype(np.int64) - q64
    st = {"max": int(np.abs(d).max()), "exact": float((d == 0).mean()), "mean_abs": float(np.abs(d).mean())}
    print(kind, "fp32 vs fp64 tiles", st, "segments/primary fp32", seg32 / (64 * len(tiles) * spp),
          "fp64", seg64 / (64 * len(tiles) * spp))
    assert abs(seg32 / seg64 - 1) <= 0.02
    assert st["max"] <= MESH_F32_MAX_LSB and st["exact"] >= MESH_F32_EXACT_FRAC
    assert st["mean_abs"] <= MESH_F32_MEAN_LSB
    assert np.isfinite(frame).all()

"""Generate the golden fixtures in tests/golden/ from the REFERENCE ITSELF.

Run in the build container (where /root/reference exists):
    make -C oracle ref && python tests/golden/make_golden.py

Every vector here comes out of oracle/_ref/ref_golden, i.e. the unmodified reference
sources compiled with g++ (oracle/ref_golden.cpp explains the two hooks: RNG injection
and scene capture).  Nothing in this directory is produced by the C restatement or by
the GPU code it is used to check.

Fixtures
  image_ref.json           sha256 + spot pixels of /root/reference/image.ppm (decoded
                           from its UTF-16LE/CRLF form to the LF ASCII the binary prints)
  image_ref_p6.ppm.gz      the same image as binary P6 (for statistical comparisons)
  pixelmatch.json          tests/tests.cpp PixelMatch: ray_color of the centre ray on the
                           ground-only scene + the first random_double() values
  scene_random.txt         the 485 spheres main.cpp builds (center, center_vec, radius,
                           material), %.17g
  counter_*.npz            per-pixel fp64 sums / 8-bit / world.hit counts under the
                           RT-CRNG-1 counter RNG (oracle/rt_rng_spec.h), seed 0x5EED
"""
from __future__ import annotations

import gzip
import hashlib
import json
import subprocess
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
REF = ROOT / "oracle" / "_ref" / "ref_golden"
SEED = "0x5EED"

# name -> (ref_golden render args, pixel selection)
COUNTER_CASES = {
    # config 1: ground + 3 big spheres, 400x225 @ 10 spp (BASELINE.json configs[0])
    "counter_c1_four_400x225_10spp": (["--scene", "four", "--width", "400", "--spp", "10"], "stride:13"),
    # config 2: random spheres 1280x720 @ 64 spp, 2048 random pixels
    "counter_c2_random_1280x720_64spp": (["--scene", "random", "--width", "1280", "--spp", "64"], ("rand", 2048, 1)),
    # config 3: random spheres 1920x1080 @ 256 spp, 512 random pixels
    "counter_c3_random_1920x1080_256spp": (["--scene", "random", "--width", "1920", "--spp", "256"],
                                           ("rand", 512, 2)),
    # depth cut-off (camera_cpu.h:12-13) on a short depth
    "counter_depth3_random_320x180_8spp": (["--scene", "random", "--width", "320", "--spp", "8", "--depth", "3"],
                                           "stride:13"),
    # camera without defocus (camera.h:94 branch), other aspect / vfov
    "counter_nodefocus_four_240x160_6spp": (["--scene", "four", "--width", "240", "--spp", "6", "--aspect", "1.5",
                                             "--vfov", "40", "--defocus-angle", "0"], "stride:5"),
    # PixelMatch scene, whole small frame
    "counter_ground_200x112_4spp": (["--scene", "ground", "--width", "200", "--spp", "4"], "stride:3"),
}


def run(args: list[str]) -> str:
    return subprocess.run([str(REF), *args], check=True, capture_output=True, text=True).stdout


def parse_render(text: str):
    rows = [l.split() for l in text.splitlines() if l and not l.startswith("#")]
    a = np.array(rows, dtype=object)
    ij = a[:, 0:2].astype(np.int32)
    sums = np.array([[float(x) for x in r[2:5]] for r in rows], dtype=np.float64)
    rgb = a[:, 5:8].astype(np.int32)
    segs = a[:, 8].astype(np.int64)
    draws = a[:, 9].astype(np.int64)
    header = [l for l in text.splitlines() if l.startswith("# W ")][0].split()
    meta = dict(zip(header[1::2], header[2::2]))
    return ij, sums, rgb, segs, draws, meta


def main() -> int:
    if not REF.exists():
        print(f"{REF} missing: run `make -C oracle ref` first", file=sys.stderr)
        return 1

    # -- image.ppm (UTF-16LE with CRLF in the reference tree) -------------------------
    raw = Path("/root/reference/image.ppm").read_bytes()
    text = raw.decode("utf-16").replace("\r\n", "\n")
    sha = hashlib.sha256(text.encode("ascii")).hexdigest()
    lines = text.split("\n")
    W, H = map(int, lines[1].split())
    px = np.array([list(map(int, l.split())) for l in lines[3:3 + W * H]], dtype=np.uint8).reshape(H, W, 3)
    p = subprocess.run([str(REF), "main"], check=True, capture_output=True, text=True)
    main_out = p.stdout
    assert hashlib.sha256(main_out.encode()).hexdigest() == sha, "reference binary does not reproduce image.ppm"
    stats = p.stderr.strip().splitlines()[-1].split()   # "# scene_draws S render_draws R segments G"
    (HERE / "image_ref.json").write_text(json.dumps({
        "source": "/root/reference/image.ppm (UTF-16LE, CRLF) decoded to LF ASCII",
        "sha256_lf_ascii": sha, "width": W, "height": H, "spp": 30, "max_depth": 50,
        "spot": {"0,0": px[0, 0].tolist(), "200,112": px[112, 200].tolist(), "399,224": px[224, 399].tolist()},
        "stream_counts_source": "oracle/_ref/ref_golden main (the unmodified reference; world wrapped in a "
                                "world.hit counter): mt19937 draws for the scene and the render, world.hit calls",
        "scene_draws": int(stats[2]), "render_draws": int(stats[4]), "segments": int(stats[6]),
    }, indent=1) + "\n")
    with open(HERE / "image_ref_p6.ppm.gz", "wb") as raw_f:
        with gzip.GzipFile(fileobj=raw_f, mode="wb", compresslevel=9, mtime=0) as f:
            f.write(f"P6\n{W} {H}\n255\n".encode() + px.tobytes())

    # -- PixelMatch + first draws --------------------------------------------------
    pm = run(["pixelmatch"]).split()
    draws = [float(x) for x in run(["draws", "16"]).split()]
    (HERE / "pixelmatch.json").write_text(json.dumps({
        "source": "tests/tests.cpp:35-45 (RayTracingFixture.PixelMatch) run on the reference",
        "expected_similar_to": [0.253, 0.3518, 0.5], "tolerance": 1e-3,
        "ray_color": [float(x) for x in pm[:3]], "draws_before_ray_color": int(pm[3]),
        "draws_in_ray_color": int(pm[4]), "first_random_doubles": draws,
    }, indent=1) + "\n")

    # -- camera::initialize for the configs ---------------------------------------------
    cams = {}
    for scene, w in (("random", 400), ("random", 1280), ("random", 1920), ("four", 401)):
        lines_ = run(["camera", "--scene", scene, "--width", str(w)]).splitlines()
        d = {l.split()[0]: [float(x) for x in l.split()[1:]] for l in lines_}
        d["image_height"] = int(d["image_height"][0])
        cams[f"{scene}_{w}"] = d
    (HERE / "camera_init.json").write_text(json.dumps(cams, indent=1) + "\n")

    # -- the random-spheres scene ----------------------------------------------------
    (HERE / "scene_random.txt").write_text(run(["scene"]))

    # -- counter-RNG goldens -------------------------------------------------------------
    for name, (args, sel) in COUNTER_CASES.items():
        if isinstance(sel, tuple):
            _, n, rs = sel
            scene, w = args[args.index("--scene") + 1], int(args[args.index("--width") + 1])
            h = int(run(["camera", "--scene", scene, "--width", str(w)]).split()[1])
            rng = np.random.default_rng(rs)
            flat = rng.choice(w * h, size=n, replace=False)
            flat.sort()
            lst = HERE / f".{name}.pixels"
            lst.write_text("".join(f"{p % w} {p // w}\n" for p in flat))
            pixarg = f"list:{lst}"
        else:
            pixarg = sel
        out = run(["render", *args, "--seed", SEED, "--rng", "counter", "--pixels", pixarg])
        if isinstance(sel, tuple):
            lst.unlink()
        ij, sums, rgb, segs, nd, meta = parse_render(out)
        np.savez_compressed(HERE / f"{name}.npz", ij=ij, sums=sums, rgb=rgb, segments=segs, draws=nd,
                            meta=json.dumps({"args": args, "seed": SEED, "pixels": str(sel), **meta}))
        print(name, len(ij), "pixels", f"W={meta['W']} H={meta['H']}")
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""Make the OBJ parse fixtures: tests/golden/obj/<case>.obj (inputs) and
<case>.tinyobj.txt, the dump of the reference's vendored tinyobjloader
(dependencies/tinyobjloader, LoadObj at tiny_obj_loader.h:605) over the same file, made
by oracle/_ref/obj_dump (built from the reference's sources by oracle/Makefile).

Run here (where /root/reference exists):  python tests/golden/make_obj_golden.py
"""
from __future__ import annotations

import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
OUT = Path(__file__).resolve().parent / "obj"
sys.path.insert(0, str(ROOT))


def quads() -> str:
    # irregular, non-planar 6x5 grid of quads: both diagonal choices occur
    rng = np.random.default_rng(7)
    nx, ny = 7, 6
    lines = ["# quad grid"]
    for j in range(ny):
        for i in range(nx):
            x, y, z = i + rng.uniform(-0.3, 0.3), rng.uniform(-0.5, 0.5), j + rng.uniform(-0.3, 0.3)
            lines.append(f"v {x!r} {y!r} {z!r}")
    for j in range(ny - 1):
        for i in range(nx - 1):
            a = j * nx + i + 1
            lines.append(f"f {a} {a + 1} {a + nx + 1} {a + nx}")
    return "\n".join(lines) + "\n"


def polygons() -> str:
    # n-gons (convex and concave), index forms, relative indices, other statements, CRLF
    L = ["# polygons", "mtllib none.mtl", "o poly", "g first", "s 1"]
    pent = [(np.cos(2 * np.pi * k / 5), np.sin(2 * np.pi * k / 5), 0.0) for k in range(5)]
    hexa = [(2 + np.cos(2 * np.pi * k / 6), 0.1 * k, np.sin(2 * np.pi * k / 6)) for k in range(6)]
    ell = [(0, 0, 3), (2, 0, 3), (2, 0, 3.5), (0.5, 0, 3.5), (0.5, 0, 5), (0, 0, 5)]   # concave L
    star = []
    for k in range(10):
        r = 1.0 if k % 2 == 0 else 0.4
        star.append((4 + r * np.cos(np.pi * k / 5), 1 + r * np.sin(np.pi * k / 5), 0.3 * r))
    V = pent + hexa + ell + star
    for v in V:
        L.append("v " + " ".join(repr(float(c)) for c in v))
    L += ["vt 0 0", "vt 1 0", "vn 0 0 1"]
    L.append("f " + " ".join(f"{k + 1}/1/1" for k in range(5)))
    L.append("usemtl red")
    L.append("f\t" + "\t".join(f"{k + 6}//1" for k in range(6)))
    L.append("g second")
    L.append("f " + " ".join(f"{k + 12}/2" for k in range(6)))
    L.append("f " + " ".join(str(k - 10) for k in range(10)))     # relative: the star
    L.append("f 1 2")                                             # degenerate: skipped
    L.append("f 1 3 4")
    return "\r\n".join(L) + "\r\n"


def blob() -> str:
    from raytracingproject_amd import meshgen
    V, F = meshgen.blob(2, radius=1.0, center=meshgen.MESH_CENTER)
    import io
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        p = Path(d) / "b.obj"
        meshgen.write_obj(p, V, F)
        return p.read_text()


CASES = {"quads": quads, "polygons": polygons, "blob2": blob}


def main() -> None:
    dump = ROOT / "oracle" / "_ref" / "obj_dump"
    if not dump.exists():
        subprocess.run(["make", "-C", str(ROOT / "oracle"), "_ref/obj_dump"], check=True)
    OUT.mkdir(exist_ok=True)
    for name, fn in CASES.items():
        obj = OUT / f"{name}.obj"
        obj.write_bytes(fn().encode())
        txt = subprocess.run([str(dump), str(obj)], check=True, capture_output=True, text=True).stdout
        (OUT / f"{name}.tinyobj.txt").write_text(txt)
        print(name, txt.splitlines()[0], [l for l in txt.splitlines() if l.startswith("T")][0])


if __name__ == "__main__":
    main()

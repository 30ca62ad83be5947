#!/usr/bin/env python3
"""Where the mesh kernel's registers go (VERDICT r03 "Next" 3: move the C4 kernel off 5
waves per SIMD).  Six waves need <= 80 VGPRs (512 per SIMD lane, 8-register granules);
the C4 kernel render_kernel<float, false, 256, 1, false, 8792, true> held 94 with the
packed all-children slab form of rounds 1-3, 88 with the per-child form built since r04 and
86 once closest_hit stopped carrying the hit distance (t = tmax); the 6-wave instantiations
(mesh_waves_per_eu = 6, the default since ABI 7) fit 80 without spilling.

Each probe applies one source edit to a scratch copy of csrc/ (the product tree is not
touched), compiles rt_render_f32.hip for gfx950 with build.py's flags and reports the
VGPRs of the if-if mesh kernels (-Rpass-analysis=kernel-resource-usage).  Most edits
break the kernel's results on purpose: they only measure what a part of the code costs in
registers.

  python tools/vgpr_probes.py [--out profiles/r04/vgpr_probes_c4_r04.txt]
"""
from __future__ import annotations

import argparse
import re
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
DEV = "raytracingproject_amd/csrc/rt_device.h"

LOADS = ("                const nu4 w0 = qa[0], w1 = qa[1], w2 = qa[2], w3 = qb[0], w4 = qb[1], w5 = qb[2], "
         "w6 = qc[0];")
SPHERE_TREE = "    if (sc.n_nodes > 0) {\n        const Node* nodes = sc.nodes;"
MESH = "    if (MESH && sc.n_mnodes > 0) {\n        // Mesh BVH (4-wide)"
NODE_STEP = "                if (!leaf) {\n                    if (DIAG) DiagCounters::count(dg->mnode_it, dg->mnode_act);"
TRI = "            if ((EXACT || (MESH_HIT_BASE | k) != self_id) && tri_root<R>(v0, e1, e2, o, d, TMIN, tmax, t)) {"
PER_CHILD_START = "                // the slab planes one child at a time (scalar FMAs: the same fused results as"
PER_CHILD_END = "            } else {\n                const float lo[4][3] = {{lx.x, ly.x, lz.x}"
PACKED = '''                // PROBE: rounds 1-3's packed all-children slab form
                typedef float f2 __attribute__((ext_vector_type(2)));
                const f2 ix = {inv.x, inv.x}, iy = {inv.y, inv.y}, iz = {inv.z, inv.z};
                const f2 nx = {-oi.x, -oi.x}, ny = {-oi.y, -oi.y}, nz = {-oi.z, -oi.z};
                f2 p[2][6];
#pragma unroll
                for (int g = 0; g < 2; ++g) {
                    p[g][0] = __builtin_elementwise_fma(g ? f2{lx.z, lx.w} : f2{lx.x, lx.y}, ix, nx);
                    p[g][1] = __builtin_elementwise_fma(g ? f2{hx.z, hx.w} : f2{hx.x, hx.y}, ix, nx);
                    p[g][2] = __builtin_elementwise_fma(g ? f2{ly.z, ly.w} : f2{ly.x, ly.y}, iy, ny);
                    p[g][3] = __builtin_elementwise_fma(g ? f2{hy.z, hy.w} : f2{hy.x, hy.y}, iy, ny);
                    p[g][4] = __builtin_elementwise_fma(g ? f2{lz.z, lz.w} : f2{lz.x, lz.y}, iz, nz);
                    p[g][5] = __builtin_elementwise_fma(g ? f2{hz.z, hz.w} : f2{hz.x, hz.y}, iz, nz);
                }
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const f2* q2 = p[c >> 1];
                    const int e = c & 1;
                    const float t0x = q2[0][e], t1x = q2[1][e], t0y = q2[2][e], t1y = q2[3][e];
                    const float t0z = q2[4][e], t1z = q2[5][e];
                    const float tn = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fmaxf(fminf(t0z, t1z), (float)TMIN));
                    const float tf = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fminf(fmaxf(t0z, t1z), (float)tmax));
                    t[c] = tn <= tf && r[c] != MREF_EMPTY ? (R)tn : INF;
                }
                if (false) {
'''

PROBES = {
    "as built": [],
    "in-flight loads 7 -> 4 (node and leaf lanes load 64 B)": [(LOADS, "                const nu4 w0 = qa[0], w1 = "
                                                                "qa[1], w2 = qa[2], w3 = qb[0];\n                const nu4 "
                                                                "w4 = w0, w5 = w1, w6 = w2;")],
    "slab distances of all four children first (packed FMAs, rounds 1-3)": [
        (PER_CHILD_START, PACKED + PER_CHILD_START), (PER_CHILD_END, "}\n" + PER_CHILD_END)],
    "sphere-tree traversal compiled out": [(SPHERE_TREE, SPHERE_TREE.replace("if (sc.n_nodes", "if (!MESH && sc.n_nodes"))],
    "triangle tests compiled out": [(TRI, TRI.replace("if ((EXACT", "if (false && (EXACT"))],
    "sphere tree out + node step trivial (no slab math)": [
        (SPHERE_TREE, SPHERE_TREE.replace("if (sc.n_nodes", "if (!MESH && sc.n_nodes")),
        (NODE_STEP, "                if (!leaf) {\n                    ref = (w0.x ^ w1.y ^ w2.z ^ w3.w ^ w4.x ^ w5.y ^ w6.z) & 1 ? "
                    "w6.x : mpop();\n                    continue;\n                }\n" + NODE_STEP)],
    "mesh traversal compiled out": [(MESH, MESH.replace("if (MESH &&", "if (false && MESH &&"))],
    "both traversals compiled out": [(MESH, MESH.replace("if (MESH &&", "if (false && MESH &&")),
                                     (SPHERE_TREE, SPHERE_TREE.replace("if (sc.n_nodes", "if (!MESH && sc.n_nodes"))],
}


def vgprs(src_root: Path) -> dict:
    cmd = ["/opt/rocm/bin/hipcc", "-x", "hip", "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{src_root / 'include'}",
           "-fno-hip-fp32-correctly-rounded-divide-sqrt", "-fgpu-flush-denormals-to-zero", "-ffp-contract=on",
           "--cuda-device-only", "-c", str(src_root / "raytracingproject_amd/csrc/rt_render_f32.hip"), "-o", "/dev/null",
           "-Rpass-analysis=kernel-resource-usage"]
    err = subprocess.run(cmd, capture_output=True, text=True).stderr
    out, cur = {}, None
    for line in err.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            continue
        m = re.search(r"remark:\s+VGPRs: (\d+)", line)
        if m and cur:
            k = re.search(r"render_kernelIfLb0ELi(\d+)ELi(\d+)ELb0ELi(8792|8920)ELb1", cur)
            if k:
                wpe = "" if k.group(2) == "1" else f"/wpe{k.group(2)}"
                out[f"{k.group(1)}/{k.group(3)}{wpe}"] = int(m.group(1))
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    lines = []
    for name, edits in PROBES.items():
        with tempfile.TemporaryDirectory(prefix="rt_vgpr_") as d:
            d = Path(d)
            shutil.copytree(ROOT / "raytracingproject_amd" / "csrc", d / "raytracingproject_amd" / "csrc")
            shutil.copytree(ROOT / "include", d / "include")
            p = d / DEV
            s = p.read_text()
            for old, new in edits:
                assert s.count(old) == 1, (name, old[:60])
                s = s.replace(old, new)
            p.write_text(s)
            v = vgprs(d)
        line = f"{name:70s} " + "  ".join(f"{k}: {v[k]}" for k in sorted(v))
        print(line, flush=True)
        lines.append(line)
    if a.out:
        Path(a.out).write_text("VGPRs of the if-if mesh kernels (block/traversal[/wpe6]), 6 waves per SIMD need <= 80, "
                               "7 need <= 72\n" +
                               "\n".join(lines) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""Per-iteration instruction counts of the traversal loops of one kernel, from its ISA
(VERDICT r03 "Next" 6: settle the C3 kernel at the instruction level).

Compiles csrc/rt_render_f32.hip for gfx950 with --save-temps (device only; same flags
as build.py), extracts one kernel (default: the C3 kernel render_kernel<float, false,
1024, 8, false, 600, false>), splits it into basic blocks, and finds the natural loops
whose header block loads a BVH node (four ds_read_b128 of one 64-B Node) or a sphere
record (two ds_read_b128).  For each such loop it prints the instruction mix of the whole
loop body (a wave whose lanes take different branches executes every block of it under
exec masks) and of the straight "all lanes hit both children" path, against a minimal
sequence for the same work (this formulation, all lanes active):

  node step (two child slabs, while-while loop with a register top and an LDS stack):
    1 node address + 12 slab FMAs + per child 9 for the entry/exit distances (3 min,
    3 max, max3, max with t_min, min3) and 2 compares (entry <= exit, entry <= t_max)
    = 1 + 12 + 22 = 35; order the children: 1 compare + 3 selects = 4; the one-child
    select 1; push: top valid?, counter, address = 3; pop: top valid?, culled?, stack
    empty?, counter, address = 5; leaf test 2  =>  50 VALU;
  sphere test (stable roots, closest-approach form, rt_device.h sphere_root): miss path:
    not-the-origin-sphere 1, centre at the ray time 3, f = o - c 3, f.d 3, t_ca 1,
    q = f - t_ca d 3, |q|^2 3, r^2 1, disc 1, compare 1 = 20; hit path: |f|^2 3, sqrt 2,
    q' = -(b + sign(b) sqrt) 2, rcp 1, the two roots 2, root choice and range 5 = 15;
    loop: counter and exit 2, closest-hit update 3, record address 1 = 6  =>  41 VALU.

python tools/isa_loops.py [--kernel MANGLED] [--out profiles/r04/isa_loops_r04.txt]
"""
from __future__ import annotations

import argparse
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
DEFAULT = "_ZN3rtx13render_kernelIfLb0ELi1024ELi8ELb0ELi600ELb0EEEvNS_12RenderParamsE"
MIN_NODE, MIN_SPHERE = 50, 41


def kernel_asm(kernel: str) -> list[str]:
    with tempfile.TemporaryDirectory(prefix="rt_isa_") as d:
        cmd = ["/opt/rocm/bin/hipcc", "-x", "hip", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
               "-Wno-unused-function", f"-I{ROOT / 'include'}", "-fno-hip-fp32-correctly-rounded-divide-sqrt",
               "-fgpu-flush-denormals-to-zero", "-ffp-contract=on", "--save-temps", "--cuda-device-only", "-c",
               str(ROOT / "raytracingproject_amd/csrc/rt_render_f32.hip"), "-o", str(Path(d) / "k.o")]
        subprocess.run(cmd, check=True, cwd=d, capture_output=True)
        s = next(Path(d).glob("*gfx950.s")).read_text().splitlines()
    start = next(i for i, l in enumerate(s) if l.startswith(kernel + ":"))
    end = next(i for i in range(start, len(s)) if s[i].strip().startswith(".Lfunc_end"))
    return s[start:end]


def blocks_of(lines: list[str]):
    blocks, cur = [], {"name": "entry", "ins": []}
    blocks.append(cur)
    for l in lines[1:]:
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            cur = {"name": m.group(1), "ins": []}
            blocks.append(cur)
            continue
        t = l.split(";")[0].strip()
        if t and not t.startswith("."):
            cur["ins"].append(t)
    return blocks


def succs(blocks):
    idx = {b["name"]: i for i, b in enumerate(blocks)}
    out = []
    for i, b in enumerate(blocks):
        s = set()
        last = b["ins"][-1] if b["ins"] else ""
        for x in b["ins"]:
            m = re.match(r"s_(cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", x)
            if m:
                s.add(idx[m.group(2)])
        if not last.startswith("s_branch") and not last.startswith("s_endpgm") and i + 1 < len(blocks):
            s.add(i + 1)
        out.append(s)
    return out


def dominators(sc, preds):
    n = len(sc)
    full = set(range(n))
    dom = [full.copy() for _ in range(n)]
    dom[0] = {0}
    changed = True
    while changed:
        changed = False
        for i in range(1, n):
            ps = [dom[p] for p in preds[i]]
            d = set.intersection(*ps) | {i} if ps else {i}
            if d != dom[i]:
                dom[i], changed = d, True
    return dom


def natural_loop(header, latch, preds):
    body, work = {header, latch}, [latch]
    while work:
        n = work.pop()
        for p in preds[n]:
            if p not in body:
                body.add(p)
                work.append(p)
    return body


def innermost_loop(h, sc, preds, dom):
    """The smallest natural loop containing block h (back edge p -> x with x dominating p)."""
    best = None
    for x in range(len(sc)):
        for p in preds[x]:
            if x in dom[p]:   # back edge p -> x
                body = natural_loop(x, p, preds)
                if h in body and (best is None or len(body) < len(best[1])):
                    best = (x, body)
    return best


def cat(ins: str) -> str:
    op = ins.split()[0]
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_waitcnt") or op.startswith("s_nop"):
        return "wait"
    if op.startswith("s_cbranch") or op.startswith("s_branch"):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    return "vmem"


def mix(ins):
    c = {}
    for x in ins:
        k = cat(x)
        c[k] = c.get(k, 0) + 1
    return c


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default=DEFAULT)
    ap.add_argument("--out", default=None)
    ap.add_argument("--listing", action="store_true", help="print the instructions of every loop found")
    a = ap.parse_args()
    blocks = blocks_of(kernel_asm(a.kernel))
    sc = succs(blocks)
    preds = [set() for _ in blocks]
    for i, s in enumerate(sc):
        for j in s:
            preds[j].add(i)
    dom = dominators(sc, preds)
    out = [f"kernel {a.kernel}: {sum(len(b['ins']) for b in blocks)} instructions in {len(blocks)} blocks"]
    seen = set()
    for h, b in enumerate(blocks):
        b128 = [x for x in b["ins"] if x.startswith("ds_read_b128")]
        kind = "node" if len(b128) >= 4 else "sphere" if len(b128) == 2 else None
        if not kind:
            continue
        lp = innermost_loop(h, sc, preds, dom)
        if lp is None:
            continue
        loop_hdr, body = lp
        key = (kind, frozenset(body))
        if key in seen:
            continue
        seen.add(key)
        ins = [x for i in sorted(body) for x in blocks[i]["ins"]]
        m = mix(ins)
        hb = mix(b["ins"])
        minimal = MIN_NODE if kind == "node" else MIN_SPHERE
        out.append(f"{kind} loop at {b['name']} ({len(body)} blocks): whole body {m}; load block {hb}; "
                   f"VALU whole body {m.get('valu', 0)} vs minimal {minimal} "
                   f"(removable at most {max(0, m.get('valu', 0) - minimal) / max(1, m.get('valu', 0)):.0%})")
        out.append("   blocks: " + " ".join(f"{blocks[i]['name']}:{mix(blocks[i]['ins']).get('valu', 0)}v"
                                              for i in sorted(body)))
        if a.listing and len(body) < 12:
            for i in sorted(body):
                out.append(f"   {blocks[i]['name']}:")
                out.extend(f"      {x}" for x in blocks[i]["ins"])
    text = "\n".join(out) + "\n"
    print(text, end="")
    if a.out:
        Path(a.out).write_text(text)
    return 0


if __name__ == "__main__":
    sys.exit(main())

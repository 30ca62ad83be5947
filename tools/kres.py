#!/usr/bin/env python3
"""Register / spill summary of the fp32 render kernels (hipcc -Rpass-analysis=kernel-resource-usage).

python tools/kres.py [filter-substring]
"""
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
cmd = ["/opt/rocm/bin/hipcc", "-x", "hip", "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{ROOT / 'include'}",
       "-fno-hip-fp32-correctly-rounded-divide-sqrt", "-fgpu-flush-denormals-to-zero", "-ffp-contract=on",
       "--cuda-device-only", "-c", str(ROOT / "raytracingproject_amd/csrc/rt_render_f32.hip"), "-o", "/dev/null",
       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
flt = sys.argv[1] if len(sys.argv) > 1 else ""
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+?): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for name, r in rows.items():
    if flt in name:
        m = re.search(r"render_kernelIfLb0ELi(\d+)ELi(\d+)ELb(\d)ELi(\d+)ELb(\d)", name)
        tag = f"block={m.group(1)} wpe={m.group(2)} diag={m.group(3)} trav={m.group(4)} mesh={m.group(5)}" if m else name
        print(f"{tag:48s} vgpr={r.get('VGPRs')} vspill={r.get('VGPRs Spill')} sspill={r.get('SGPRs Spill')} "
              f"scratch={r.get('ScratchSize [bytes/lane]')} occ={r.get('Occupancy [waves/SIMD]')}")

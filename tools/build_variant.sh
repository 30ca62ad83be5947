#!/bin/bash
# Build an experimental library raytracingproject_amd/lib/librt_hip_NAME.so: every unit
# recompiled with extra defines (e.g. -DRT_EXP_FLATY=1), with build.py's per-unit flags.
# For same-box A/Bs (tools/gpu_session.sh libab: every lib/librt_hip*.so on C3 and the C5
# geometry).
#   bash tools/build_variant.sh NAME "-DRT_EXP_X=1 ..."
set -euo pipefail
NAME=$1; DEFS=${2:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/rt_var_XXXXXX); trap 'rm -rf "$T"' EXIT
cd "$ROOT"
python - "$T" "$DEFS" <<'PY'
import subprocess, sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path
from raytracingproject_amd import build as b
out, defs = Path(sys.argv[1]), sys.argv[2].split()
def comp(kv):
    src, extra = kv
    o = out / (src.rsplit(".", 1)[0] + ".o")
    subprocess.run([b.HIPCC, *b.COMMON, *defs, *extra, "-c", str(b.CSRC / src), "-o", str(o)], check=True)
    return o
with ThreadPoolExecutor(max_workers=4) as ex:
    objs = list(ex.map(comp, b.UNITS.items()))
PY
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/raytracingproject_amd/lib/librt_hip_$NAME.so" \
    "$T"/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "raytracingproject_amd/lib/librt_hip_$NAME.so ($DEFS)"

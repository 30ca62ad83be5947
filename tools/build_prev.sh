#!/bin/bash
# Build the library of another commit as raytracingproject_amd/lib/librt_hip_prev.so, the
# "previous" side of the same-box A/B steps in tools/gpu_session.sh (ab, abmesh, mw6: run
# with RT_ALLOW_ABI_MISMATCH=1 RT_LIB_PATH=...librt_hip_prev.so).  The commit is checked out
# into a temporary git worktree and built there (build.build_native), so the working tree
# and its own build are not touched.
#   bash tools/build_prev.sh [REF]        (default: HEAD, i.e. A/B of uncommitted changes)
set -euo pipefail
REF=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=$(mktemp -d /tmp/rt_prev_XXXXXX)
cleanup() { git -C "$ROOT" worktree remove --force "$WT" >/dev/null 2>&1 || rm -rf "$WT"; }
trap cleanup EXIT
git -C "$ROOT" worktree add --detach "$WT" "$REF" >/dev/null
(cd "$WT" && python -c "from raytracingproject_amd import build; build.build_native()")
mkdir -p "$ROOT/raytracingproject_amd/lib"
cp "$WT/raytracingproject_amd/lib/librt_hip.so" "$ROOT/raytracingproject_amd/lib/librt_hip_prev.so"
echo "raytracingproject_amd/lib/librt_hip_prev.so <- $(git -C "$ROOT" rev-parse --short "$REF")"

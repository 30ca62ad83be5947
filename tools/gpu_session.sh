#!/bin/bash
# One GPU session: smoke, GPU tests, bench, rocprof kernel-trace summary.
# Each GPU step has its own time limit; after a crash/abort/timeout nothing else runs.
# Usage: bash tools/gpu_session.sh TAG [steps...]   steps: smoke tests bench prof pmc
set -u
TAG=${1:-r01}; shift || true
STEPS=${*:-smoke tests bench prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
export PYTHONUNBUFFERED=1
echo "host $(hostname) $(date -u +%FT%TZ)" > "$OUT/status"
ok() {  # rc 0 = pass, 1 = test failures (not a GPU fault): keep going
  [ "$1" -eq 0 ] || [ "$1" -eq 1 ]
}
step() {
  local name=$1 limit=$2; shift 2
  echo "== $name: $*" >> "$OUT/status"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> "$OUT/status"
  tail -5 "$OUT/$name.log"
  ok $rc || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
for s in $STEPS; do
  case $s in
    smoke) step smoke 400 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) step tests 900 python -m pytest tests -m gpu -q -rA ;;
    bench) step bench 600 python bench.py ;;
    prof)  step prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ;;
    pmc)   step pmc_fetch 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o bench --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
           step pmc_write 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_write" -o bench --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    sweep) step sweep 600 python tools/sweep.py ;;
    *) echo "unknown step $s" ;;
  esac
done
echo done >> "$OUT/status"

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
    tests) step tests 900 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread ;;
    quick) step quick 600 python -u -m pytest tests/test_gpu_parity.py tests/test_mesh.py -m gpu -x -q -rA --timeout 300 --timeout-method thread -k "tuning or variants or coherent or golden or exact" ;;
    bench) step bench 600 python bench.py ;;
    prof)  step prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ;;
    prof2) step prof2 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof2" -o target --output-format csv -- python3 tools/profile_target.py --frames 3 ;;
    pmc)   T="python3 tools/profile_target.py --frames 2 --meta $OUT/meta_c3.json"
           step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o pmc --output-format csv -- $T
           step pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o pmc --output-format csv -- $T
           step pmc_sum 60 python3 tools/pmc_traffic.py "$OUT/pmc_c3.json" "$OUT/pmc_fetch" "$OUT/pmc_write" --meta $OUT/meta_c3.json ;;
    sq)    step sq1 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d "$OUT/sq1" -o pmc --output-format csv -- python3 tools/profile_target.py --frames 1
           step sq3 600 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_INT32 SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_CVT -d "$OUT/sq3" -o pmc --output-format csv -- python3 tools/profile_target.py --frames 1
           step sq2 600 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d "$OUT/sq2" -o pmc --output-format csv -- python3 tools/profile_target.py --frames 1
           step sq_sum 60 python3 tools/pmc_traffic.py "$OUT/sq.json" "$OUT/sq1" "$OUT/sq2" "$OUT/sq3" ;;
    mtests) step mtests 900 python -m pytest tests/test_mesh.py -m gpu -q -rA -s ;;
    mbench) step mbench 600 python bench.py --scene mesh --no-cpu-baseline
            step mbench_mixed 900 python bench.py --scene mixed --steps 3 --warmup 1
            step mbench_gpubuild 600 python bench.py --scene mesh --no-cpu-baseline --mesh-builder gpu ;;
    f64bench) step f64bench 600 python bench.py --precision f64 --width 1280 --spp 64 --steps 3 --warmup 1 --no-cpu-baseline
              step f64bench_c3 600 python bench.py --precision f64 --steps 3 --warmup 1 --no-cpu-baseline
              step f64prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/f64prof" -o f64 --output-format csv -- python3 tools/profile_target.py --precision f64 --frames 3 ;;
    # mesh configs at their bench sizes: kernel trace, then FETCH / WRITE passes filed under
    # the launch's PMC keys (profile_target --meta), for C4 (mesh 1080p x 128) and C5 (mixed 4K x 1024)
    mprof) for cfg in "mesh 1920 128 c4" "mixed 3840 1024 c5"; do
             set -- $cfg
             T="python3 tools/profile_target.py --scene $1 --width $2 --spp $3 --frames 2 --meta $OUT/meta_$4.json"
             step mprof_$4 600 rocprofv3 --kernel-trace --stats -d "$OUT/mprof_$4" -o target --output-format csv -- $T
             step mpmc_fetch_$4 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/mpmc_fetch_$4" -o pmc --output-format csv -- $T
             step mpmc_write_$4 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/mpmc_write_$4" -o pmc --output-format csv -- $T
             step mpmc_sum_$4 60 python3 tools/pmc_traffic.py "$OUT/pmc_$4.json" "$OUT/mpmc_fetch_$4" "$OUT/mpmc_write_$4" --meta $OUT/meta_$4.json
           done ;;
    msq)   for cfg in "mesh 1920 128 c4" "mixed 3840 1024 c5"; do
             set -- $cfg
             T="python3 tools/profile_target.py --scene $1 --width $2 --spp $3 --frames 1"
             step msq1_$4 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_LDS -d "$OUT/msq1_$4" -o pmc --output-format csv -- $T
             step msq2_$4 600 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_FLAT SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d "$OUT/msq2_$4" -o pmc --output-format csv -- $T
             step msq3_$4 600 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES TCC_HIT TCC_MISS TCC_REQ -d "$OUT/msq3_$4" -o pmc --output-format csv -- $T
             step msq_sum_$4 60 python3 tools/pmc_traffic.py "$OUT/msq_$4.json" "$OUT/msq1_$4" "$OUT/msq2_$4" "$OUT/msq3_$4"
           done ;;
    msq16)   T="python3 tools/profile_target.py --frames 1 --scene mesh --spp 16"
           step msq1 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_LDS -d "$OUT/msq1" -o pmc --output-format csv -- $T
           step msq2 600 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_FLAT SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d "$OUT/msq2" -o pmc --output-format csv -- $T
           step msq3 600 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES TCC_HIT TCC_MISS TCC_REQ -d "$OUT/msq3" -o pmc --output-format csv -- $T
           step msq4 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/msq4" -o pmc --output-format csv -- $T
           step msq_sum 60 python3 tools/pmc_traffic.py "$OUT/msq.json" "$OUT/msq1" "$OUT/msq2" "$OUT/msq3" "$OUT/msq4" --key mesh7:1920x1080x16 ;;
    scal)  step scal 600 python tools/shard_scaling.py --reps 3 ;;
    scal8) step scal8_base 300 python tools/shard_scaling.py --ns 1,8 --reps 3
           step scal8_ib8 300 python tools/shard_scaling.py --ns 1,8 --reps 3 --tune item_balance=8.0
           step scal8_ib16 300 python tools/shard_scaling.py --ns 1,8 --reps 3 --tune item_balance=16.0
           step scal8_is4 300 python tools/shard_scaling.py --ns 8 --reps 3 --tune item_samples=4
           step scal8_r32 300 python tools/shard_scaling.py --ns 1,8 --reps 3 --tune coh_refill=32
           step scal8_base2 300 python tools/shard_scaling.py --ns 1,8 --reps 3 ;;
    cohgap) step cohgap 600 python tools/variant_probe.py --frames 3 --variants "block=512,traversal=8;block=1024,traversal=88;block=512,traversal=8" ;;
    overlap) step overlap 600 python tools/overlap_probe.py --ns 1,2,4,8 ;;
    # fixed per-launch part: kernel time against spp for the whole frame and an 8-GPU shard
    scalspp) for spp in 64 128 256 512; do step scal_spp$spp 600 python tools/shard_scaling.py --ns 1,8 --reps 3 --spp $spp; done ;;
    # same-box A/B of the in-tree library against raytracingproject_amd/lib/librt_hip_prev.so
    # (built from another commit by tools/build_prev.sh REF)
    # (the previous commit, built beside it): default kernel, C3, alternating processes
    ab)    for i in 1 2 3; do
             step ab_prev_$i 300 env RT_ALLOW_ABI_MISMATCH=1 RT_LIB_PATH=raytracingproject_amd/lib/librt_hip_prev.so python tools/variant_probe.py --frames 3
             step ab_new_$i 300 python tools/variant_probe.py --frames 3
           done ;;
    abmesh) for i in 1 2; do
             step abm_prev_$i 300 env RT_ALLOW_ABI_MISMATCH=1 RT_LIB_PATH=raytracingproject_amd/lib/librt_hip_prev.so python tools/variant_probe.py --scene mesh --spp 128 --frames 3
             step abm_new_$i 300 python tools/variant_probe.py --scene mesh --spp 128 --frames 3
             step abx_prev_$i 300 env RT_ALLOW_ABI_MISMATCH=1 RT_LIB_PATH=raytracingproject_amd/lib/librt_hip_prev.so python tools/variant_probe.py --scene mixed --spp 256 --frames 2
             step abx_new_$i 300 python tools/variant_probe.py --scene mixed --spp 256 --frames 2
           done ;;
    trace) step trace_tests 300 python -u -m pytest tests/test_trace_rays.py -m gpu -x -q -rA --timeout 120 --timeout-method thread
           step sort_bound 600 python tools/sort_bound.py ;;
    # workgroup-local regrouping bound (1,024 rays), first and later bounces
    sortwg) step sortwg_b1 300 python tools/sort_bound.py --spp 1
            step sortwg_b2 300 python tools/sort_bound.py --spp 1 --bounce 2
            step sortwg_b3 300 python tools/sort_bound.py --spp 1 --bounce 3
            step sortwg_s2 300 python tools/sort_bound.py --spp 2 ;;
    front) step front_tests 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rA --timeout 120 --timeout-method thread -k "front or tuning_never"
           step front_probe 600 python tools/variant_probe.py --frames 3 --variants "front_spheres=0;front_spheres=-1;front_spheres=0;front_spheres=-1" ;;
    list)  step list 120 rocprofv3 -L ;;
    diagfb) step diagfb 300 python tools/diag.py --spp 256 ;;
    mdiag) step mdiag_tests 300 python -u -m pytest tests/test_gpu_diag.py -m gpu -x -q -rA --timeout 120 --timeout-method thread
           step mdiag_c4 300 python tools/diag.py --scene mesh --spp 32
           step mdiag_c5 300 python tools/diag.py --scene mixed --spp 16 ;;
    # knob re-check of the C3 default after the r03 kernel changes (all bit-identical frames)
    knobs) step knobs1 600 python tools/variant_probe.py --frames 3 --variants "coh_refill=40;coh_refill=56;coh_refill=32;item_balance=2.0;item_balance=6.0;coh_refill=48"
           step knobs2 600 python tools/variant_probe.py --frames 3 --variants "max_leaf=5;max_leaf=7;max_leaf=8;cost_intersect=0.2;cost_intersect=0.35;front_spheres=4;front_spheres=8;max_leaf=6" ;;
    # fp64 kernels: tests, then C2 timings of every f64_kernel (same frame bit for bit)
    f64k)  step f64_tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_trace_rays.py tests/test_mesh.py -m gpu -x -q -rA --timeout 300 --timeout-method thread -k "f64 or trace or exact or oracle"
           step f64_probe 600 python tools/variant_probe.py --precision f64 --width 1280 --spp 64 --frames 3 --variants "f64_kernel=3;f64_kernel=4;f64_kernel=3;f64_kernel=4"
           step f64_probe_c3 600 python tools/variant_probe.py --precision f64 --spp 256 --frames 2 --variants "f64_kernel=4;f64_kernel=3;f64_kernel=4" ;;
    diag)  step diag 300 python tools/diag.py ;;
    sweep) step sweep 600 python tools/sweep.py ;;

    # if-if mesh loop (TRAV_MIFIF = 8192): equality tests, then C4 and C5 (4K @ 32) timings
    mifif) step mifif_tests 600 python -u -m pytest tests/test_mesh.py -m gpu -x -q -rA --timeout 300 --timeout-method thread -k "variants or full_frame or watertight"
           step mifif_c4 600 python tools/variant_probe.py --scene mesh --spp 128 --frames 3 --variants "traversal=8792;traversal=600;traversal=8792"
           step mifif_c5 900 python tools/variant_probe.py --scene mixed --width 3840 --spp 32 --frames 2 --variants "traversal=8792;traversal=600;traversal=8792" ;;
    # mesh knobs re-checked under the if-if loop (C4; C5 geometry at 4K @ 32)
    mknobs) step mknobs_c4 900 python tools/variant_probe.py --scene mesh --spp 128 --frames 3 --variants "mesh_max_leaf=2;mesh_max_leaf=3;mesh_max_leaf=6;mesh_cost_traverse=1.0;mesh_cost_traverse=3.0;mesh_block=512;mesh_lds_stack=8;mesh_lds_stack=16;mesh_item_balance=10.0;mesh_item_balance=40.0;mesh_max_leaf=4"
            step mknobs_c5 900 python tools/variant_probe.py --scene mixed --width 3840 --spp 32 --frames 2 --variants "mesh_max_leaf=2;mesh_max_leaf=3;mesh_cost_traverse=1.0;mesh_cost_traverse=3.0;mesh_block=256;mesh_lds_stack=8;mesh_max_leaf=4" ;;
    # leaf size / SAH node cost under the if-if loop
    mleaf) step mleaf_c4 900 python tools/variant_probe.py --scene mesh --spp 128 --frames 3 --variants "mesh_max_leaf=2;mesh_max_leaf=1;mesh_max_leaf=2,mesh_cost_traverse=1.0;mesh_max_leaf=2,mesh_cost_traverse=1.5;mesh_max_leaf=3,mesh_cost_traverse=1.0;mesh_cost_traverse=0.5;mesh_builder=1;mesh_builder=1,mesh_max_leaf=2;mesh_max_leaf=2"
           step mleaf_c5 900 python tools/variant_probe.py --scene mixed --width 3840 --spp 32 --frames 2 --variants "mesh_max_leaf=2;mesh_max_leaf=1;mesh_max_leaf=2,mesh_cost_traverse=1.0;mesh_max_leaf=2,mesh_cost_traverse=1.5;mesh_max_leaf=2" ;;
    # C4 kernel time against spp (the fixed per-launch part of the mesh kernel)
    mspp) for spp in 32 64 128 256; do step mspp_$spp 300 python tools/variant_probe.py --scene mesh --spp $spp --frames 3; done
          step mspp_ib 600 python tools/variant_probe.py --scene mesh --spp 128 --frames 3 --variants "mesh_item_balance=5.0;mesh_item_balance=80.0;item_samples=16;item_samples=8" ;;
    # coherent-kernel refill threshold for mesh scenes
    mrefill) step mrefill_c4 600 python tools/variant_probe.py --scene mesh --spp 128 --frames 3 --variants "coh_refill=32;coh_refill=40;coh_refill=56;coh_refill=64;coh_refill=24"
             step mrefill_c5 900 python tools/variant_probe.py --scene mixed --width 3840 --spp 32 --frames 2 --variants "coh_refill=32;coh_refill=56;coh_refill=64" ;;
    msmall) step msmall 300 python -u -m pytest tests/test_mesh.py -m gpu -x -q -rA --timeout 120 --timeout-method thread -k "small or plan" ;;
    # predicted strong scaling per config (slowest shard of N on one GPU)
    scalall) step scal_c3 300 python tools/shard_scaling.py --reps 3
             step scal_c4 300 python tools/shard_scaling.py --scene mesh --spp 128 --reps 3
             step scal_c5 600 python tools/shard_scaling.py --scene mixed --width 3840 --spp 1024 --reps 2 ;;
    # C4 small shards: work-queue item knobs at N = 8
    scalc4) step sc4_base 300 python tools/shard_scaling.py --scene mesh --spp 128 --ns 1,8 --reps 3
            step sc4_ib5 300 python tools/shard_scaling.py --scene mesh --spp 128 --ns 1,8 --reps 3 --tune mesh_item_balance=5.0
            step sc4_ib80 300 python tools/shard_scaling.py --scene mesh --spp 128 --ns 1,8 --reps 3 --tune mesh_item_balance=80.0
            step sc4_is8 300 python tools/shard_scaling.py --scene mesh --spp 128 --ns 1,8 --reps 3 --tune item_samples=8
            step sc4_is4 300 python tools/shard_scaling.py --scene mesh --spp 128 --ns 1,8 --reps 3 --tune item_samples=4
            step sc4_b512 300 python tools/shard_scaling.py --scene mesh --spp 128 --ns 1,8 --reps 3 --tune mesh_block=512 ;;
    scalc4b) for ib in 20.0 40.0 80.0 160.0 320.0 20.0; do step sc4b_ib$ib 300 python tools/shard_scaling.py --scene mesh --spp 128 --ns 1,2,8 --reps 3 --tune mesh_item_balance=$ib; done ;;
    # C4: the 6-wave mesh kernel (mesh_waves_per_eu=6) against the 5-wave default, and the
    # previous library (packed slab form) for the per-child slab change, alternating
    mw6)  step mw6_tests 600 python -u -m pytest tests/test_mesh.py -m gpu -x -q -rA --timeout 300 --timeout-method thread -k "six_wave or variants or full_frame or watertight"
          for i in 1 2; do
            step mw6_prev_$i 300 env RT_ALLOW_ABI_MISMATCH=1 RT_LIB_PATH=raytracingproject_amd/lib/librt_hip_prev.so python tools/variant_probe.py --scene mesh --spp 128 --frames 3
            step mw6_new_$i 300 python tools/variant_probe.py --scene mesh --spp 128 --frames 3 --variants "mesh_waves_per_eu=6,mesh_block=256;mesh_waves_per_eu=0;mesh_waves_per_eu=6,mesh_block=256"
          done ;;
    # C5 (4K @ 32): 6 waves per SIMD need 3 512-thread workgroups per CU, i.e. the mesh
    # traversal stack out of LDS (mesh_lds_stack=0) and the <= 80-VGPR kernel
    mw6c5) for i in 1 2; do
             step mw6c5_$i 900 python tools/variant_probe.py --scene mixed --width 3840 --spp 32 --frames 2 --variants "mesh_waves_per_eu=6,mesh_block=512,mesh_lds_stack=0;mesh_lds_stack=0;mesh_waves_per_eu=6,mesh_block=512,mesh_lds_stack=0"
           done ;;
    # C4: 7 waves per SIMD (<= 72 VGPRs, 4 spill ops in the if-if loop) and the 512-thread
    # 6-wave kernel against the auto default (256 / 6 waves); the 5-wave kernel as the anchor
    mw7)  step mw7_tests 600 python -u -m pytest tests/test_mesh.py -m gpu -x -q -rA --timeout 300 --timeout-method thread -k "six_wave or variants or auto_plan"
          for i in 1 2; do
            step mw7_c4_$i 300 python tools/variant_probe.py --scene mesh --spp 128 --frames 3 --variants "mesh_waves_per_eu=7,mesh_block=256;mesh_block=512;mesh_waves_per_eu=0,mesh_block=256;mesh_waves_per_eu=7,mesh_block=256"
          done ;;
    # work-queue / refill knobs re-checked under the 6-wave defaults (C4; C5 geometry at 4K @ 32)
    mk6)  step mk6_c4 600 python tools/variant_probe.py --scene mesh --spp 128 --frames 3 --variants "coh_refill=40;coh_refill=56;mesh_item_balance=10.0;mesh_item_balance=40.0;mesh_max_leaf=3;coh_refill=48"
          step mk6_c5 900 python tools/variant_probe.py --scene mixed --width 3840 --spp 32 --frames 2 --variants "coh_refill=40;coh_refill=56;mesh_item_balance=10.0;mesh_item_balance=40.0;mesh_block=256" ;;
    # C4 / C5 knobs after t = tmax: LDS stack depth beyond the auto cap, item size, SAH node cost
    mk7)  step mk7_c4 600 python tools/variant_probe.py --scene mesh --spp 128 --frames 3 --variants "mesh_lds_stack=14;mesh_lds_stack=6;item_samples=16;mesh_cost_traverse=1.5;mesh_cost_traverse=3.0;mesh_lds_stack=14"
          step mk7_c5 900 python tools/variant_probe.py --scene mixed --width 3840 --spp 32 --frames 2 --variants "mesh_lds_stack=2;item_samples=16;mesh_cost_traverse=3.0" ;;
    # C4: the two knobs that came out ahead in mk7, alternated against the default
    mk8)  for i in 1 2 3; do
            step mk8_c4_$i 300 python tools/variant_probe.py --scene mesh --spp 128 --frames 3 --variants "mesh_lds_stack=14;mesh_cost_traverse=3.0;mesh_lds_stack=14,mesh_cost_traverse=3.0"
          done
          step mk8_c5 900 python tools/variant_probe.py --scene mixed --width 3840 --spp 32 --frames 2 --variants "mesh_cost_traverse=3.0;mesh_cost_traverse=2.5" ;;
    # C4 small shards under the final kernels: mesh_item_balance at N = 8 (and N = 1)
    scalc4c) for ib in 20.0 80.0 160.0 40.0 20.0; do step sc4c_ib$ib 300 python tools/shard_scaling.py --scene mesh --spp 128 --ns 1,8 --reps 3 --tune mesh_item_balance=$ib; done ;;
    # C3 small shards: item_balance at N = 8 (and N = 1), the driver's scaling config
    scalc3b) for ib in 4.0 8.0 16.0 2.0 4.0; do step sc3b_ib${ib}_$RANDOM 300 python tools/shard_scaling.py --ns 1,8 --reps 3 --tune item_balance=$ib; done ;;
    # r05: fp32 watertightness probe (rays from inside the C4 blob; leaks saved for tools/leak_probe.py --analyze)
    leak) step leak 600 python tools/leak_probe.py --rays 33554432 --out "$OUT/leaks.npz" ;;
    # r05: C5 traffic split at 4K @ 32: FETCH / WRITE / TCC hit + SQ memory
    # instruction counts per plan -- default (stack in scratch, no LDS sums, 3 workgroups per CU),
    # 4 / 8 / 32 LDS stack entries without sums, 8 with sums
    c5split) i=0
             for v in "" "mesh_lds_stack=4,traversal=728" "mesh_lds_stack=8,traversal=728" "mesh_lds_stack=8" "mesh_lds_stack=32,traversal=728"; do
               i=$((i+1))
               T="python3 tools/profile_target.py --scene mixed --width 3840 --spp 32 --frames 2 --tune $v --meta $OUT/meta_c5v$i.json"
               [ -z "$v" ] && T="python3 tools/profile_target.py --scene mixed --width 3840 --spp 32 --frames 2 --meta $OUT/meta_c5v$i.json"
               echo "c5v$i: $v" >> "$OUT/status"
               step c5v${i}_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/c5v${i}_fetch" -o pmc --output-format csv -- $T
               step c5v${i}_write 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/c5v${i}_write" -o pmc --output-format csv -- $T
               step c5v${i}_tcc 300 rocprofv3 --pmc TCC_HIT TCC_REQ SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_FLAT SQ_INSTS_VALU SQ_BUSY_CYCLES -d "$OUT/c5v${i}_tcc" -o pmc --output-format csv -- $T
               step c5v${i}_sum 60 python3 tools/pmc_traffic.py "$OUT/pmc_c5v$i.json" "$OUT/c5v${i}_fetch" "$OUT/c5v${i}_write" "$OUT/c5v${i}_tcc" --meta $OUT/meta_c5v$i.json
             done
             step c5split_time 600 python tools/variant_probe.py --scene mixed --width 3840 --spp 32 --frames 3 --variants "mesh_lds_stack=4,traversal=728;mesh_lds_stack=8,traversal=728;mesh_lds_stack=8;mesh_lds_stack=32,traversal=728;mesh_lds_stack=-1" ;;
    # r05: watertight fp32 triangles (36-B records) + 768-thread C5 plan: the mesh / progressive /
    # diag GPU tests, then a same-box A/B of C4 and C5 (4K @ 32) against the r04 library (prev)
    # and the one-triangle-per-iteration build (librt_hip_one.so)
    wt)   step wt_tests 900 python -u -m pytest tests/test_mesh.py tests/test_progressive.py tests/test_gpu_diag.py tests/test_gpu_parity.py -m gpu -x -q -rA --timeout 300 --timeout-method thread -k "watertight or mesh or variants or plan or progressive or diag or if_if or triangles_only or full_frame or six_wave"
          for i in 1 2; do
            for lib in prev one cur; do
              L=raytracingproject_amd/lib/librt_hip_$lib.so; [ $lib = cur ] && L=raytracingproject_amd/lib/librt_hip.so
              step wt_c4_${lib}_$i 300 env RT_ALLOW_ABI_MISMATCH=1 RT_LIB_PATH=$L python tools/variant_probe.py --scene mesh --spp 128 --frames 3
              step wt_c5_${lib}_$i 300 env RT_ALLOW_ABI_MISMATCH=1 RT_LIB_PATH=$L python tools/variant_probe.py --scene mixed --width 3840 --spp 32 --frames 2
            done
          done ;;
    # r05: C5 plans under the 48-B watertight build: 512 (no sums, stack in scratch) against 768
    # (sums + 2 LDS entries), 768 without LDS stack, 768 without sums (5 LDS entries)
    c5plan) step c5plan 900 python tools/variant_probe.py --scene mixed --width 3840 --spp 32 --frames 2 --variants "mesh_block=512;mesh_block=768,mesh_lds_stack=0;mesh_block=768,traversal=728;mesh_block=512;mesh_block=768" ;;
    # (r05's same-box A/Bs against Moller-Trumbore builds, ab2-ab5 and mq, are recorded in
    # profiles/r05/r05d-r05g; the experiment switch they built with was removed)
    # r05: C5 at full size (4K @ 1024): PMC FETCH / WRITE / TCC hit per plan -- 768 threads with
    # sums and 2 LDS stack entries (auto), 768 with sums and the stack in scratch, 512 without sums
    c5full) i=0
            for v in "" "mesh_lds_stack=0" "mesh_block=512"; do
              i=$((i+1))
              T="python3 tools/profile_target.py --scene mixed --width 3840 --spp 1024 --frames 1 --meta $OUT/meta_c5f$i.json"
              [ -n "$v" ] && T="$T --tune $v"
              echo "c5f$i: $v" >> "$OUT/status"
              step c5f${i}_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/c5f${i}_fetch" -o pmc --output-format csv -- $T
              step c5f${i}_write 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/c5f${i}_write" -o pmc --output-format csv -- $T
              step c5f${i}_tcc 300 rocprofv3 --pmc TCC_HIT TCC_REQ -d "$OUT/c5f${i}_tcc" -o pmc --output-format csv -- $T
              step c5f${i}_sum 60 python3 tools/pmc_traffic.py "$OUT/pmc_c5f$i.json" "$OUT/c5f${i}_fetch" "$OUT/c5f${i}_write" "$OUT/c5f${i}_tcc" --meta $OUT/meta_c5f$i.json
            done ;;
    # r05: the C4 kernel at the compiler's register budget (5 waves, no spills) against the
    # 6-wave kernel that spills around the bounce
    c4w)  step c4w 600 python tools/variant_probe.py --scene mesh --spp 128 --frames 3 --variants "mesh_waves_per_eu=0;mesh_waves_per_eu=6;mesh_waves_per_eu=0;mesh_waves_per_eu=6" ;;
    # r05: the uniform sphere grid (traversal 65536) against the sphere tree on C3, by density
    grid) step grid_tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_mesh.py -m gpu -x -q -rA --timeout 300 --timeout-method thread -k "tuning_never or sphere_grid or golden or mixed or plan"
          step grid_c3 900 python tools/variant_probe.py --frames 3 --variants "traversal=66136,sphere_grid_density=1.0;traversal=66136,sphere_grid_density=2.0;traversal=66136,sphere_grid_density=3.0;traversal=66136,sphere_grid_density=4.0;traversal=66136,sphere_grid_density=0.5;traversal=66136,sphere_grid_density=2.0,front_spheres=0" ;;
    # same-box A/B of the grid kernel: this tree's library against librt_hip_prev.so
    gridab) for i in 1 2; do
              for lib in prev cur; do
                L=raytracingproject_amd/lib/librt_hip_$lib.so; [ $lib = cur ] && L=raytracingproject_amd/lib/librt_hip.so
                step gridab_${lib}_$i 300 env RT_ALLOW_ABI_MISMATCH=1 RT_LIB_PATH=$L python tools/variant_probe.py --frames 3 --variants "traversal=66136,sphere_grid_density=2.0;traversal=66136,sphere_grid_density=1.5;traversal=66136,sphere_grid_density=2.5"
              done
            done ;;
    # same-box A/B of every library variant in lib/ (librt_hip.so and librt_hip_*.so, built
    # by tools/build_prev.sh or by hand), C3 and the C5 geometry, interleaved twice
    # r06: knob re-check on the final mixed kernel (C5 geometry, 4K @ 32), same process, twice
    c5knobs) for i in 1 2; do
               step c5knobs_$i 900 python tools/variant_probe.py --scene mixed --width 3840 --spp 32 --frames 2 --variants "coh_refill=40;coh_refill=56;mesh_item_balance=10.0;mesh_item_balance=40.0;item_samples=16;sphere_grid_density=2.5;coh_refill=48"
             done ;;
    libab) for i in 1 2; do
             for L in raytracingproject_amd/lib/librt_hip.so raytracingproject_amd/lib/librt_hip_*.so; do
               n=$(basename "$L" .so)
               step libab_c3_${n}_$i 300 env RT_ALLOW_ABI_MISMATCH=1 RT_LIB_PATH=$L python tools/variant_probe.py --frames 3
               step libab_c5_${n}_$i 300 env RT_ALLOW_ABI_MISMATCH=1 RT_LIB_PATH=$L python tools/variant_probe.py --scene mixed --width 3840 --spp 32 --frames 2
               [ -n "${LIBAB_C4:-}" ] && step libab_c4_${n}_$i 300 env RT_ALLOW_ABI_MISMATCH=1 RT_LIB_PATH=$L python tools/variant_probe.py --scene mesh --spp 128 --frames 3
               [ -n "${LIBAB_F64:-}" ] && step libab_f64_${n}_$i 300 env RT_ALLOW_ABI_MISMATCH=1 RT_LIB_PATH=$L python tools/variant_probe.py --precision f64 --spp 64 --frames 2
             done
           done ;;
    # the sphere grid in the mixed scene (C5 geometry at 4K @ 32, and C3): auto plan against the tree
    gridc5) step gridc5 900 python tools/variant_probe.py --scene mixed --width 3840 --spp 32 --frames 2 --variants "traversal=600;mesh_block=512;traversal=600;mesh_block=768,traversal=66136" ;;
    # r05: the grid's time slabs (sphere_grid_time_slabs), same process, C3 and the C5 geometry
    slabs) for i in 1 2; do
             step slabs_c3_$i 600 python tools/variant_probe.py --frames 3 --variants "sphere_grid_time_slabs=1;sphere_grid_time_slabs=4;sphere_grid_time_slabs=8;sphere_grid_time_slabs=16;sphere_grid_time_slabs=32;sphere_grid_time_slabs=64;sphere_grid_time_slabs=1"
           done
           step slabs_c5 900 python tools/variant_probe.py --scene mixed --width 3840 --spp 32 --frames 2 --variants "sphere_grid_time_slabs=1;sphere_grid_time_slabs=16;sphere_grid_time_slabs=64;sphere_grid_time_slabs=1" ;;
    # r05: knob re-check on the final grid kernel (density, refill threshold, item sizes)
    gridknobs) for i in 1 2; do
                 step gridknobs_$i 600 python tools/variant_probe.py --frames 3 --variants "sphere_grid_density=1.5;sphere_grid_density=2.5;sphere_grid_density=3.0;coh_refill=32;coh_refill=40;coh_refill=56;coh_refill=64;item_samples=16;item_balance=2.0;item_balance=8.0"
               done ;;
    gridknobs2) for i in 1 2; do
                  step gridknobs2_$i 600 python tools/variant_probe.py --frames 3 --variants "item_balance=4.0;item_balance=8.0;coh_refill=40;item_balance=8.0,coh_refill=40;item_balance=4.0;item_balance=16.0;item_balance=8.0;coh_refill=48"
                done ;;
    griddiag) step griddiag 300 python tools/diag.py --spp 64 --trav 66136 && step bvhdiag 300 python tools/diag.py --spp 64 --trav 600 ;;
    # same-box A/B of this tree's library against librt_hip_prev.so on C3 and the C5 geometry
    abc3) for i in 1 2; do
            for lib in prev cur; do
              L=raytracingproject_amd/lib/librt_hip_$lib.so; [ $lib = cur ] && L=raytracingproject_amd/lib/librt_hip.so
              step abc3_${lib}_$i 300 env RT_ALLOW_ABI_MISMATCH=1 RT_LIB_PATH=$L python tools/variant_probe.py --frames 3
              step abc5_${lib}_$i 300 env RT_ALLOW_ABI_MISMATCH=1 RT_LIB_PATH=$L python tools/variant_probe.py --scene mixed --width 3840 --spp 32 --frames 2
            done
          done ;;
    mdiag2) step mdiag_c4 300 python tools/diag.py --scene mesh --spp 32 && step mdiag_c5 300 python tools/diag.py --scene mixed --width 3840 --spp 8 ;;
    # r05: the mesh tree's shape under the watertight triangle test (C4, and the C5 geometry)
    mshape) step mshape_c4 900 python tools/variant_probe.py --scene mesh --spp 128 --frames 3 --variants "mesh_max_leaf=1;mesh_max_leaf=3;mesh_max_leaf=4;mesh_cost_traverse=1.0;mesh_cost_traverse=3.0;mesh_cost_traverse=4.0"
            step mshape_c5 900 python tools/variant_probe.py --scene mixed --width 3840 --spp 32 --frames 2 --variants "mesh_max_leaf=1;mesh_max_leaf=3;mesh_cost_traverse=1.0;mesh_cost_traverse=3.0" ;;
    # same-box A/B on the mesh configs (C4, the C5 geometry): this tree against librt_hip_prev.so
    abmesh2) for i in 1 2; do
              for lib in prev cur; do
                L=raytracingproject_amd/lib/librt_hip_$lib.so; [ $lib = cur ] && L=raytracingproject_amd/lib/librt_hip.so
                step abm_c4_${lib}_$i 300 env RT_ALLOW_ABI_MISMATCH=1 RT_LIB_PATH=$L python tools/variant_probe.py --scene mesh --spp 128 --frames 3
                step abm_c5_${lib}_$i 300 env RT_ALLOW_ABI_MISMATCH=1 RT_LIB_PATH=$L python tools/variant_probe.py --scene mixed --width 3840 --spp 32 --frames 2
              done
            done
            step abm_tests 900 python -u -m pytest tests/test_mesh.py tests/test_gpu_diag.py -m gpu -x -q -rA --timeout 300 --timeout-method thread ;;
    abmesh3) for i in 1 2; do
              step abm3_c4_prev_$i 300 env RT_ALLOW_ABI_MISMATCH=1 RT_LIB_PATH=raytracingproject_amd/lib/librt_hip_prev.so python tools/variant_probe.py --scene mesh --spp 128 --frames 3
              step abm3_c4_cur_$i 300 python tools/variant_probe.py --scene mesh --spp 128 --frames 3 --variants "mesh_block=256;mesh_block=512;mesh_block=256,mesh_lds_stack=8"
            done ;;
    # r06: the bounded grid walk (far cameras, scan list) and the grid / golden tests around it
    far)  step far_tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_progressive.py -m gpu -x -q -rA --timeout 300 --timeout-method thread -k "far_cameras or grid_reach or sphere_grid or tuning_never or golden or exact or progressive" ;;
    # r06: rank 0's per-step work at N = 8 beside the kernel, C3 and C5
    step8) step step8_c3 600 python tools/shard_scaling.py --ns 1,8 --reps 3 --step
           step step8_c5 900 python tools/shard_scaling.py --scene mixed --width 3840 --spp 1024 --ns 1,8 --reps 2 --step ;;
    # r06: the GPU-built (LBVH) mesh tree on C4: kernel trace + FETCH / WRITE
    # r06: the fp32 mesh kernels' path state parked in LDS (throughput, scatter count) against
    # HEAD (librt_hip_prev.so): mesh tests, then C3 / C4 / C5 interleaved, then C4 traffic
    park) step park_tests 900 python -u -m pytest tests/test_mesh.py tests/test_progressive.py tests/test_gpu_diag.py -m gpu -x -q -rA --timeout 300 --timeout-method thread -k "variants or full_frame or watertight or six_wave or plan or golden or mixed or progressive or diag"
          for i in 1 2; do
            for L in raytracingproject_amd/lib/librt_hip_prev.so raytracingproject_amd/lib/librt_hip.so; do
              n=$(basename "$L" .so)
              step park_c3_${n}_$i 300 env RT_ALLOW_ABI_MISMATCH=1 RT_LIB_PATH=$L python tools/variant_probe.py --frames 3
              step park_c4_${n}_$i 300 env RT_ALLOW_ABI_MISMATCH=1 RT_LIB_PATH=$L python tools/variant_probe.py --scene mesh --spp 128 --frames 3
              step park_c5_${n}_$i 600 env RT_ALLOW_ABI_MISMATCH=1 RT_LIB_PATH=$L python tools/variant_probe.py --scene mixed --width 3840 --spp 1024 --frames 2
            done
          done
          T="python3 tools/profile_target.py --scene mesh --width 1920 --spp 128 --frames 2 --meta $OUT/meta_c4.json"
          step park_prof_c4 600 rocprofv3 --kernel-trace --stats -d "$OUT/park_prof_c4" -o target --output-format csv -- $T
          step park_fetch_c4 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/park_fetch_c4" -o pmc --output-format csv -- $T
          step park_write_c4 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/park_write_c4" -o pmc --output-format csv -- $T
          step park_sum_c4 60 python3 tools/pmc_traffic.py "$OUT/pmc_c4_park.json" "$OUT/park_fetch_c4" "$OUT/park_write_c4" --meta $OUT/meta_c4.json ;;
    # ... C4's block and LDS stack entries with the parked state (1 KB more LDS per wave)
    park2) for i in 1 2; do
             step park2_prev_$i 300 env RT_ALLOW_ABI_MISMATCH=1 RT_LIB_PATH=raytracingproject_amd/lib/librt_hip_prev.so python tools/variant_probe.py --scene mesh --spp 128 --frames 3 --variants "mesh_block=256;mesh_block=512"
             step park2_new_$i 600 python tools/variant_probe.py --scene mesh --spp 128 --frames 3 --variants "mesh_block=256;mesh_block=256,mesh_lds_stack=8;mesh_block=256,mesh_lds_stack=12;mesh_block=512;mesh_block=512,mesh_lds_stack=0;mesh_block=256,mesh_lds_stack=0"
           done ;;
    # ... parked only in the mixed-scene (grid) kernels: tests, then C5 / C4 / C3 against HEAD
    park3) step park3_tests 900 python -u -m pytest tests/test_mesh.py tests/test_progressive.py tests/test_gpu_diag.py tests/test_gpu_parity.py -m gpu -x -q -rA --timeout 300 --timeout-method thread -k "variants or full_frame or watertight or six_wave or plan or golden or mixed or progressive or diag or grid or far"
           for i in 1 2; do
             for L in raytracingproject_amd/lib/librt_hip_prev.so raytracingproject_amd/lib/librt_hip.so; do
               n=$(basename "$L" .so)
               step park3_c5_${n}_$i 600 env RT_ALLOW_ABI_MISMATCH=1 RT_LIB_PATH=$L python tools/variant_probe.py --scene mixed --width 3840 --spp 1024 --frames 2
               step park3_c4_${n}_$i 300 env RT_ALLOW_ABI_MISMATCH=1 RT_LIB_PATH=$L python tools/variant_probe.py --scene mesh --spp 128 --frames 3
               step park3_c3_${n}_$i 300 env RT_ALLOW_ABI_MISMATCH=1 RT_LIB_PATH=$L python tools/variant_probe.py --frames 3
             done
           done
           T="python3 tools/profile_target.py --scene mixed --width 3840 --spp 1024 --frames 2 --meta $OUT/meta_c5.json"
           step park3_prof_c5 600 rocprofv3 --kernel-trace --stats -d "$OUT/park3_prof_c5" -o target --output-format csv -- $T
           step park3_fetch_c5 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/park3_fetch_c5" -o pmc --output-format csv -- $T
           step park3_write_c5 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/park3_write_c5" -o pmc --output-format csv -- $T
           step park3_sum_c5 60 python3 tools/pmc_traffic.py "$OUT/pmc_c5_park.json" "$OUT/park3_fetch_c5" "$OUT/park3_write_c5" --meta $OUT/meta_c5.json ;;
    # r06: C5 knobs on the parked mixed-scene kernel (full size), then its bench line
    c5park) for i in 1 2; do
              step c5park_$i 900 python tools/variant_probe.py --scene mixed --width 3840 --spp 1024 --frames 2 --variants "mesh_lds_stack=1;coh_refill=40;coh_refill=56;mesh_item_balance=10.0;mesh_item_balance=40.0;item_samples=16;mesh_block=512"
            done
            step mbench_mixed 900 python bench.py --scene mixed --steps 3 --warmup 1 ;;
    # r06: frames in flight on the GPU (two render streams) against one stream, per N's shard
    pipe) step pipe_c3 600 python tools/pipeline_probe.py --ns 1,2,4,8 --frames 8 --reps 3
          step pipe_c4 600 python tools/pipeline_probe.py --scene mesh --spp 128 --ns 1,8 --frames 8 --reps 3
          step pipe_c5 900 python tools/pipeline_probe.py --scene mixed --width 3840 --spp 1024 --ns 1,8 --frames 4 --reps 2 ;;
    mprofgpu) T="python3 tools/profile_target.py --scene mesh --width 1920 --spp 128 --frames 2 --tune mesh_builder=1 --meta $OUT/meta_c4gpu.json"
           step mprof_c4gpu 600 rocprofv3 --kernel-trace --stats -d "$OUT/mprof_c4gpu" -o target --output-format csv -- $T
           step mpmc_fetch_c4gpu 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/mpmc_fetch_c4gpu" -o pmc --output-format csv -- $T
           step mpmc_write_c4gpu 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/mpmc_write_c4gpu" -o pmc --output-format csv -- $T
           step mpmc_sum_c4gpu 60 python3 tools/pmc_traffic.py "$OUT/pmc_c4gpu.json" "$OUT/mpmc_fetch_c4gpu" "$OUT/mpmc_write_c4gpu" --meta $OUT/meta_c4gpu.json ;;
    # r06: does C4 wait on its per-bounce spill?  6-wave (16 VGPRs spilled per bounce) against
    # the compiler's budget (5 waves, no spill): time, then WRITE_SIZE / FETCH_SIZE and SQ waits of each
    c4spill) for i in 1 2; do
               step c4spill_t_$i 600 python tools/variant_probe.py --scene mesh --spp 128 --frames 3 --variants "mesh_waves_per_eu=6;mesh_waves_per_eu=0"
             done
             for w in 6 0; do
               T="python3 tools/profile_target.py --scene mesh --width 1920 --spp 128 --frames 2 --tune mesh_waves_per_eu=$w --meta $OUT/meta_c4w$w.json"
               step c4w${w}_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/c4w${w}_fetch" -o pmc --output-format csv -- $T
               step c4w${w}_write 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/c4w${w}_write" -o pmc --output-format csv -- $T
               step c4w${w}_sq 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d "$OUT/c4w${w}_sq" -o pmc --output-format csv -- $T
               step c4w${w}_sum 60 python3 tools/pmc_traffic.py "$OUT/pmc_c4w$w.json" "$OUT/c4w${w}_fetch" "$OUT/c4w${w}_write" "$OUT/c4w${w}_sq" --meta $OUT/meta_c4w$w.json
             done ;;
    # r06: C5's traffic by source, the C5 geometry at 4K @ 32 (traffic per
    # launch scales with spp): the default plan, no per-bounce spill (the compiler's budget),
    # and 0 / 2 / 8 LDS mesh-stack entries (the rest in scratch); time, FETCH, WRITE each
    c5src) step c5src_t 900 python tools/variant_probe.py --scene mixed --width 3840 --spp 32 --frames 2 --variants "mesh_waves_per_eu=0;mesh_lds_stack=0;mesh_lds_stack=2;mesh_lds_stack=8;mesh_waves_per_eu=0,mesh_block=512"
           for v in default mesh_waves_per_eu=0 mesh_lds_stack=0 mesh_lds_stack=8; do
             n=$(echo $v | tr '=,' '__')
             tn=""; [ $v != default ] && tn="--tune $v"
             T="python3 tools/profile_target.py --scene mixed --width 3840 --spp 32 --frames 2 $tn --meta $OUT/meta_c5_$n.json"
             step c5src_fetch_$n 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/c5src_fetch_$n" -o pmc --output-format csv -- $T
             step c5src_write_$n 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/c5src_write_$n" -o pmc --output-format csv -- $T
             step c5src_sq_$n 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d "$OUT/c5src_sq_$n" -o pmc --output-format csv -- $T
             step c5src_tcc_$n 600 rocprofv3 --pmc TCC_HIT TCC_MISS TCC_REQ -d "$OUT/c5src_tcc_$n" -o pmc --output-format csv -- $T
             step c5src_sum_$n 60 python3 tools/pmc_traffic.py "$OUT/pmc_c5_$n.json" "$OUT/c5src_fetch_$n" "$OUT/c5src_write_$n" "$OUT/c5src_sq_$n" "$OUT/c5src_tcc_$n" --meta $OUT/meta_c5_$n.json
           done ;;
    # r06: LDS mesh-stack entries re-checked (the C5 geometry ran 1.7 % faster with none, r06h)
    mstack) for i in 1 2; do
              step mstack_c4_$i 600 python tools/variant_probe.py --scene mesh --spp 128 --frames 3 --variants "mesh_lds_stack=0;mesh_lds_stack=4;mesh_lds_stack=8;mesh_lds_stack=12"
              step mstack_c5_$i 900 python tools/variant_probe.py --scene mixed --width 3840 --spp 1024 --frames 2 --variants "mesh_lds_stack=0;mesh_lds_stack=2"
            done ;;
    mstack2) for i in 1 2; do
              step mstack2_c5_$i 900 python tools/variant_probe.py --scene mixed --width 3840 --spp 1024 --frames 2 --variants "mesh_lds_stack=0,mesh_block=768;mesh_lds_stack=0,mesh_block=512;mesh_lds_stack=0,mesh_block=256"
            done ;;
    # r06: the regrouping precondition -- C3 at one 1024-thread workgroup per CU (what a
    # 32-B-per-ray exchange buffer would leave: 69 + 32 KB of LDS per workgroup) against two
    regroupocc) for i in 1 2; do
                  step regroupocc_$i 600 python tools/variant_probe.py --frames 3 --variants "grid_workgroups=256;grid_workgroups=384"
                done ;;
    # r06: the GPU mesh build with treelet restructuring
    gpubvh) step gpubvh_tests 900 python -u -m pytest tests/test_mesh.py tests/test_trace_rays.py -m gpu -x -q -rA --timeout 300 --timeout-method thread -k "gpu_bvh or watertight or small_meshes or trace_rays or auto_plan"
            for i in 1 2; do
              step gpubvh_c4_$i 600 python tools/variant_probe.py --scene mesh --spp 128 --frames 3 --variants "mesh_builder=1;mesh_builder=2;mesh_builder=0"
            done ;;
    *) echo "unknown step $s" ;;
  esac
done
echo done >> "$OUT/status"

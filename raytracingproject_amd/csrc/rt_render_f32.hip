// rt_render_f32.hip -- fp32 fast path.  Built (raytracingproject_amd/build.py) with FMA
// contraction, hardware reciprocal / square root (-fno-hip-fp32-correctly-rounded-divide-sqrt:
// v_rcp_f32 / v_sqrt_f32 instead of the ~10-instruction IEEE sequences) and fp32
// denormals flushed; the parity tests bound the effect (<= 2 LSB vs the reference).
#include <algorithm>

#include "rt_render_impl.h"

namespace rtx {

template <int BLOCK, int MINW, int TRAV, bool MESH = false, bool DIAG = false>
static hipError_t launch(const RenderParams& P, size_t lds_bytes, hipStream_t stream) {
    const int waves = BLOCK / 64;
    long items = 0;   // the work queue's items (persistent lanes: resident workgroups only)
    for (int p = 0; p < P.nph; ++p) items += (long)P.shard_tiles * P.ph_k[p];
    int grid = (int)((items + waves - 1) / waves);
    if (grid > P.max_wgs) grid = P.max_wgs;
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL((render_kernel<float, false, BLOCK, MINW, DIAG, TRAV, MESH>), dim3(grid), dim3(BLOCK),
                       lds_bytes, stream, P);
    return hipGetLastError();
}

// Instrumented builds (rt_render_diag): the same persistent kernels with loop-utilisation
// counters and phase / timeline stamps into P.diag, for exactly the instantiations that
// render frames (RT_DIAG_VARIANTS); any other combination is refused, so the counters
// always describe the kernel that renders the frames.
#define RT_DIAG_VARIANTS(X) \
    X(1024, 8, 600) X(1024, 8, 728) X(512, 8, 8) X(1024, 8, 66136) X(1024, 8, 66264) X(1024, 8, 197208) X(1024, 8, 197336)
// mesh scenes: the default mesh kernels (if-if loop, with / without LDS item sums) at the
// register budget they render with (6 waves per SIMD, <= 80 VGPRs), so that the occupancy,
// LDS stack depth and max_wgs the plan sized for them hold for the instrumented copy too
#define RT_DIAG_MESH_VARIANTS(X) \
    X(256, 6, 8792) X(512, 6, 8792) X(768, 6, 8792) X(256, 6, 8920) X(512, 6, 8920) X(768, 6, 8920) \
    X(768, 6, 74328) X(512, 6, 74456) X(768, 6, 205400) X(512, 6, 205528)

bool render_f32_diag_supported(int block, int waves_per_eu, int trav, bool mesh) {
#define RT_DSUP(B, W, T) \
    if (block == B && waves_per_eu == W && trav == T) return true;
    if (mesh) {
        RT_DIAG_MESH_VARIANTS(RT_DSUP)
    } else {
        RT_DIAG_VARIANTS(RT_DSUP)
    }
#undef RT_DSUP
    return false;
}

hipError_t launch_render_f32_diag(const RenderParams& P, size_t lds_bytes, hipStream_t stream, int trav, int block,
                                  int waves_per_eu) {
#define RT_DCASE(B, W, T) \
    if (block == B && waves_per_eu == W && trav == T) return launch<B, W, T, false, true>(P, lds_bytes, stream);
#define RT_DMCASE(B, W, T) \
    if (block == B && waves_per_eu == W && trav == T) return launch<B, W, T, true, true>(P, lds_bytes, stream);
    if (P.n_mnodes > 0) {
        RT_DIAG_MESH_VARIANTS(RT_DMCASE)
    } else {
        RT_DIAG_VARIANTS(RT_DCASE)
    }
#undef RT_DCASE
#undef RT_DMCASE
    return hipErrorInvalidValue;
}

// The instantiated (block, waves_per_eu, traversal) combinations (r04: the default kernel,
// its automatic no-LDS-sums form (128), the kernel without pop culling (88 / 216) for the
// culling equality tests, and the one-path-per-lane kernel that every coherent kernel is
// tested against; the time-binned trees 856 / 984 were removed).
#define RT_VARIANTS(X) \
    X(1024, 8, 600) X(1024, 8, 728) X(1024, 8, 88) X(1024, 8, 216) X(512, 8, 8) X(1024, 8, 66136) X(1024, 8, 66264) \
    X(1024, 8, 197208) X(1024, 8, 197336)
// scenes with a triangle mesh (MESH instantiation: HBM-resident mesh BVH): the if-if mesh
// loop (TRAV_MIFIF: 8792 / 8920 = 600 / 728 + 8192, with / without the LDS item sums) at
// both workgroup sizes the plan chooses from, within 80 VGPRs (6 waves per SIMD: C4 -5 %,
// C5 geometry -12 %, profiles/r04/mw6_ab_r04f.txt); as equality references the same loop
// at the compiler's budget (5 waves, the default of rounds 1-3), the while-while loop of
// rounds 1-3 (728, TRAV_MWHILE) and the one-path-per-lane kernel (8).  (7 waves, <= 72 VGPRs,
// spilled inside the traversal loop: C4 45.0 against 37.8 ms, r04i; not kept.)  (r04 removed the LDS
// tree-top kernels 4696 / 4824, measured -2.8 %, and the other 5-wave copies.)
// Whole-record sphere-BVH reads (TRAV_B128) are kept for meshes since r03ag: the mixed
// scene's sphere traversal gains 0.7-0.8 % (profiles/r03/mixed_b128_probe_r03ag.jsonl).
// r05: 768-thread workgroups (12 waves, two per CU = 6 waves per SIMD) for the mixed scene:
// one LDS copy of the sphere scene serves 12 waves instead of 8, which leaves room for the
// LDS item sums and two LDS mesh-stack entries per lane at the 6-wave occupancy (512-thread
// workgroups fit three per CU only without both).
// (r05 also built the quantised 64-B node kernels, 41560 / 41688: C4 +12 %, C5 +7 %, removed.)
// r06: the grid kernels again with the flat walk (TRAV_GFLAT, + 131072: 197208 / 197336 for
// spheres, 205400 / 205528 mixed), which the C ABI picks where the grid is one cell tall in y;
// the 3-D ones serve every other grid and the flat walk's equality tests (traversal | 262144).
#define RT_MESH_VARIANTS(X)                                                                                \
    X(256, 6, 8792) X(512, 6, 8792) X(768, 6, 8792) X(256, 6, 8920) X(512, 6, 8920) X(768, 6, 8920)      \
    X(768, 6, 74328) X(512, 6, 74456) X(768, 6, 205400) X(512, 6, 205528) X(256, 0, 8792) X(512, 0, 728)   \
    X(512, 0, 8)

// Batched world.hit (rt_trace_rays), fp32: the default kernel's traversal flags
// (select root, whole-record LDS reads for spheres, pop culling; meshes: the if-if mesh
// loop); DIAG counts loop utilisation (tools/sort_bound.py).
hipError_t launch_trace_f32(const RenderParams& P, size_t lds_bytes, hipStream_t stream, const void* rays, int n,
                            void* hits, const int* remap, bool diag) {
    if (n <= 0) return hipSuccess;
    constexpr int B = TRACE_BLOCK;
    const int grid = std::min((n + B - 1) / B, 8192);
    constexpr int TS = TRAV_SELROOT | TRAV_B128 | TRAV_CULL, TM = TRAV_SELROOT | TRAV_CULL | TRAV_MIFIF;
    const float* r = (const float*)rays;
    TraceHit* h = (TraceHit*)hits;
    if (P.n_mnodes > 0)
        hipLaunchKernelGGL((trace_kernel<float, false, B, TM, true>), dim3(grid), dim3(B), lds_bytes, stream, P, r, n, h,
                           remap);
    else if (diag)
        hipLaunchKernelGGL((trace_kernel<float, false, B, TS, false, true>), dim3(grid), dim3(B), lds_bytes, stream, P,
                           r, n, h, remap);
    else
        hipLaunchKernelGGL((trace_kernel<float, false, B, TS, false>), dim3(grid), dim3(B), lds_bytes, stream, P, r, n,
                           h, remap);
    return hipGetLastError();
}

bool render_f32_supported(int block, int waves_per_eu, int trav, bool mesh) {
#define RT_SUP(B, W, T) \
    if (block == B && waves_per_eu == W && trav == T) return true;
    if (mesh) {
        RT_MESH_VARIANTS(RT_SUP)
    } else {
        RT_VARIANTS(RT_SUP)
    }
#undef RT_SUP
    return false;
}

int render_f32_vgprs(int block, int waves_per_eu, int trav, bool mesh) {
    hipFuncAttributes a;
#define RT_ATTR(B, W, T, M)                                                                                     \
    if (block == B && waves_per_eu == W && trav == T)                                                           \
        return hipFuncGetAttributes(&a, (const void*)render_kernel<float, false, B, (W ? W : 1), false, T, M>) == \
                       hipSuccess                                                                               \
                   ? a.numRegs                                                                                  \
                   : -1;
#define RT_ATTR_S(B, W, T) RT_ATTR(B, W, T, false)
#define RT_ATTR_M(B, W, T) RT_ATTR(B, W, T, true)
    if (mesh) {
        RT_MESH_VARIANTS(RT_ATTR_M)
    } else {
        RT_VARIANTS(RT_ATTR_S)
    }
#undef RT_ATTR
#undef RT_ATTR_S
#undef RT_ATTR_M
    return -1;
}

int render_f32_static_lds(int block, int waves_per_eu, int trav, bool mesh) {
    hipFuncAttributes a;
#define RT_SLDS(B, W, T, M)                                                                                     \
    if (block == B && waves_per_eu == W && trav == T)                                                           \
        return hipFuncGetAttributes(&a, (const void*)render_kernel<float, false, B, (W ? W : 1), false, T, M>) == \
                       hipSuccess                                                                               \
                   ? (int)a.sharedSizeBytes                                                                     \
                   : -1;
#define RT_SLDS_S(B, W, T) RT_SLDS(B, W, T, false)
#define RT_SLDS_M(B, W, T) RT_SLDS(B, W, T, true)
    if (mesh) {
        RT_MESH_VARIANTS(RT_SLDS_M)
    } else {
        RT_VARIANTS(RT_SLDS_S)
    }
#undef RT_SLDS
#undef RT_SLDS_S
#undef RT_SLDS_M
    return -1;
}

hipError_t launch_render_f32(const RenderParams& P, size_t lds_bytes, hipStream_t stream, int block,
                             int waves_per_eu, int trav) {
#define RT_CASE(B, W, T) \
    if (block == B && waves_per_eu == W && trav == T) return launch<B, (W ? W : 1), T>(P, lds_bytes, stream);
#define RT_MCASE(B, W, T) \
    if (block == B && waves_per_eu == W && trav == T) return launch<B, (W ? W : 1), T, true>(P, lds_bytes, stream);
    if (P.n_mnodes > 0) {
        RT_MESH_VARIANTS(RT_MCASE)
    } else {
        RT_VARIANTS(RT_CASE)
    }
#undef RT_CASE
#undef RT_MCASE
    return hipErrorInvalidValue;
}

}  // namespace rtx

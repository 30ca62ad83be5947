// rt_render_f32.hip -- fp32 fast path.  Built (raytracingproject_amd/build.py) with FMA
// contraction, hardware reciprocal / square root (-fno-hip-fp32-correctly-rounded-divide-sqrt:
// v_rcp_f32 / v_sqrt_f32 instead of the ~10-instruction IEEE sequences) and fp32
// denormals flushed; the parity tests bound the effect (<= 2 LSB vs the reference).
#include "rt_render_impl.h"

namespace rtx {

template <int BLOCK, int MINW, int TRAV, bool MESH = false, bool DIAG = false>
static hipError_t launch(const RenderParams& P, size_t lds_bytes, hipStream_t stream) {
    const int waves = BLOCK / 64;
    long items = (long)P.shard_tiles * (P.chunk > 0 ? P.nchunks : 1);
    if (P.queue) {
        items = 0;
        for (int p = 0; p < P.nph; ++p) items += (long)P.shard_tiles * P.ph_k[p];
    }
    int grid = (int)((items + waves - 1) / waves);
    if (P.queue && grid > P.max_wgs) grid = P.max_wgs;   // persistent lanes: resident workgroups only
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL((render_kernel<float, false, BLOCK, MINW, DIAG, TRAV, MESH>), dim3(grid), dim3(BLOCK),
                       lds_bytes, stream, P);
    return hipGetLastError();
}

// Instrumented build (rt_render_diag): the same persistent kernel, <= 64 VGPRs, with
// loop-utilisation counters and phase cycle stamps into P.diag (block 512; the coherent
// kernel at 512 or 1024, with whole-record reads for the default traversal flags).
hipError_t launch_render_f32_diag(const RenderParams& P, size_t lds_bytes, hipStream_t stream, int trav, int block) {
    if (trav & TRAV_COH) {
        constexpr int T = TRAV_COH | TRAV_SELROOT, TN = T | TRAV_NOSUM, TB = T | TRAV_B128;
        if ((trav & TRAV_B128) && !(trav & TRAV_NOSUM) && block == 1024)   // the default kernel
            return launch<1024, 8, TB, false, true>(P, lds_bytes, stream);
        if (trav & TRAV_NOSUM)
            return block == 1024 ? launch<1024, 8, TN, false, true>(P, lds_bytes, stream)
                                 : launch<512, 8, TN, false, true>(P, lds_bytes, stream);
        return block == 1024 ? launch<1024, 8, T, false, true>(P, lds_bytes, stream)
                             : launch<512, 8, T, false, true>(P, lds_bytes, stream);
    }
    if (block != 512) return hipErrorInvalidValue;
    if (trav == 1) return launch<512, 8, 1, false, true>(P, lds_bytes, stream);
    if (trav == 0) return launch<512, 8, 0, false, true>(P, lds_bytes, stream);
    if (trav & TRAV_POOL) return launch<512, 4, TRAV_POOL | TRAV_SELROOT, false, true>(P, lds_bytes, stream);
    return launch<512, 8, 8, false, true>(P, lds_bytes, stream);
}

// The instantiated (block, waves_per_eu, traversal) combinations; tools/sweep.py times them.
#define RT_VARIANTS(X)                                                                                    \
    X(512, 8, 8) X(512, 8, 0) X(512, 8, 1) X(512, 8, 2) X(512, 8, 4) X(512, 8, 12) X(512, 0, 8) X(512, 6, 8)  \
        X(448, 8, 8) X(256, 8, 8) X(1024, 0, 8) X(512, 8, 24) X(512, 4, 40) X(512, 0, 40) X(1024, 8, 8)     \
        X(1024, 8, 72) X(512, 8, 72) X(1024, 0, 72) X(1024, 8, 74) X(768, 6, 72) X(1024, 8, 73) X(1024, 8, 88)\
        X(1024, 8, 200) X(512, 8, 200) X(1024, 0, 200) X(1024, 8, 202) X(768, 6, 200) X(1024, 8, 201) X(1024, 8, 216) \
        X(1024, 8, 344) X(1024, 8, 472) X(1024, 8, 600) X(1024, 8, 602) X(1024, 8, 728) \
        X(1024, 8, 856) X(1024, 8, 984)
// scenes with a triangle mesh (MESH instantiation: HBM-resident mesh BVH)
#define RT_MESH_VARIANTS(X)                                                                             \
    X(512, 0, 8) X(512, 8, 8) X(512, 6, 8) X(512, 5, 8) X(256, 0, 8) X(256, 6, 8) X(256, 5, 8) X(512, 0, 0) \
        X(512, 0, 200) X(256, 0, 200) X(512, 0, 712) X(256, 0, 712)

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

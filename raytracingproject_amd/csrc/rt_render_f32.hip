// rt_render_f32.hip -- fp32 fast path.  Built (raytracingproject_amd/build.py) with FMA
// contraction, hardware reciprocal / square root (-fno-hip-fp32-correctly-rounded-divide-sqrt:
// v_rcp_f32 / v_sqrt_f32 instead of the ~10-instruction IEEE sequences) and fp32
// denormals flushed; the parity tests bound the effect (<= 2 LSB vs the reference).
#include "rt_render_impl.h"

namespace rtx {

template <int BLOCK, int MINW>
static hipError_t launch(const RenderParams& P, size_t lds_bytes, hipStream_t stream) {
    const int waves = BLOCK / 64;
    const int grid = (P.shard_tiles + waves - 1) / waves;
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL((render_kernel<float, false, BLOCK, MINW>), dim3(grid), dim3(BLOCK), lds_bytes, stream, P);
    return hipGetLastError();
}

hipError_t launch_render_f32_diag(const RenderParams& P, size_t lds_bytes, hipStream_t stream) {
    const int grid = (P.shard_tiles + 7) / 8;
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL((render_kernel<float, false, 512, 1, true>), dim3(grid), dim3(512), lds_bytes, stream, P);
    return hipGetLastError();
}

hipError_t launch_render_f32(const RenderParams& P, size_t lds_bytes, hipStream_t stream, int block,
                             int waves_per_eu) {
    if (waves_per_eu == 6) {
        if (block == 512) return launch<512, 6>(P, lds_bytes, stream);
        if (block == 256) return launch<256, 6>(P, lds_bytes, stream);
        return hipErrorInvalidValue;
    }
    switch (block) {
        case 256: return launch<256, 1>(P, lds_bytes, stream);
        case 512: return launch<512, 1>(P, lds_bytes, stream);
        case 1024: return launch<1024, 1>(P, lds_bytes, stream);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace rtx

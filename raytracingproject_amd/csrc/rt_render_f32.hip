// rt_render_f32.hip -- fp32 fast path (FMA contraction allowed).  Built with
// hipcc --offload-arch=gfx950 -O3 (see raytracingproject_amd/build.py).
#include "rt_render_impl.h"

namespace rtx {

template <int BLOCK>
static hipError_t launch(const RenderParams& P, size_t lds_bytes, hipStream_t stream) {
    const int waves = BLOCK / 64;
    const int grid = (P.shard_tiles + waves - 1) / waves;
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL((render_kernel<float, false, BLOCK>), dim3(grid), dim3(BLOCK), lds_bytes, stream, P);
    return hipGetLastError();
}

hipError_t launch_render_f32(const RenderParams& P, size_t lds_bytes, hipStream_t stream, int block) {
    switch (block) {
        case 256: return launch<256>(P, lds_bytes, stream);
        case 512: return launch<512>(P, lds_bytes, stream);
        case 1024: return launch<1024>(P, lds_bytes, stream);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace rtx

// rt_render_f32.hip -- fp32 fast path (FMA contraction allowed).  Built with
// hipcc --offload-arch=gfx950 -O3 (see raytracingproject_amd/build.py).
#include "rt_render_impl.h"

namespace rtx {

hipError_t launch_render_f32(const RenderParams& P, size_t lds_bytes, hipStream_t stream) {
    const int waves = RENDER_BLOCK / 64;
    const int grid = (P.shard_tiles + waves - 1) / waves;
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL((render_kernel<float, false, RENDER_BLOCK>), dim3(grid), dim3(RENDER_BLOCK), lds_bytes, stream,
                       P);
    return hipGetLastError();
}

}  // namespace rtx

// rt_render_f64.hip -- fp64 reference-exact path, built with -ffp-contract=off so every
// operation rounds as in the g++ build of the reference.  Also hosts the small
// precision-agnostic kernels (unshard, quantize).
#include "rt_render_impl.h"

namespace rtx {

int render_f64_vgprs(bool mesh) {
    hipFuncAttributes a;
    const hipError_t e =
        mesh ? hipFuncGetAttributes(&a, (const void*)render_kernel<double, true, RENDER_BLOCK_F64, 1, false, 0, true>)
             : hipFuncGetAttributes(&a, (const void*)render_kernel<double, true, RENDER_BLOCK_F64>);
    return e == hipSuccess ? a.numRegs : -1;
}

hipError_t launch_render_f64(const RenderParams& P, size_t lds_bytes, hipStream_t stream) {
    const int waves = RENDER_BLOCK_F64 / 64;
    const long items = (long)P.shard_tiles * (P.chunk > 0 ? P.nchunks : 1);
    const int grid = (int)((items + waves - 1) / waves);
    if (grid == 0) return hipSuccess;
    if (P.n_mnodes > 0)
        hipLaunchKernelGGL((render_kernel<double, true, RENDER_BLOCK_F64, 1, false, 0, true>), dim3(grid),
                           dim3(RENDER_BLOCK_F64), lds_bytes, stream, P);
    else
        hipLaunchKernelGGL((render_kernel<double, true, RENDER_BLOCK_F64>), dim3(grid), dim3(RENDER_BLOCK_F64),
                           lds_bytes, stream, P);
    return hipGetLastError();
}

hipError_t launch_tape_f64(const RenderParams& P, int max_depth, const double* ray7, const double* tape, int tape_len,
                           double* out, int* used, hipStream_t stream) {
    hipLaunchKernelGGL(tape_kernel<double>, dim3(1), dim3(64), 0, stream, P, max_depth, ray7, tape, tape_len, out,
                       used);
    return hipGetLastError();
}

hipError_t launch_unshard(const void* gathered, void* frame, int elem_bytes, int channels, int W, int H, int tiles_x,
                          int nshards, int max_shard_tiles, hipStream_t stream) {
    const dim3 block(256), grid((W + 255) / 256, H);
    if (W <= 0 || H <= 0) return hipSuccess;
    if (elem_bytes == 8 && channels == 3)
        hipLaunchKernelGGL((unshard_kernel<double, 3>), grid, block, 0, stream, (const double*)gathered,
                           (double*)frame, W, H, tiles_x, nshards, max_shard_tiles);
    else if (elem_bytes == 4 && channels == 3)
        hipLaunchKernelGGL((unshard_kernel<float, 3>), grid, block, 0, stream, (const float*)gathered, (float*)frame,
                           W, H, tiles_x, nshards, max_shard_tiles);
    else if (elem_bytes == 4 && channels == 1)
        hipLaunchKernelGGL((unshard_kernel<uint32_t, 1>), grid, block, 0, stream, (const uint32_t*)gathered,
                           (uint32_t*)frame, W, H, tiles_x, nshards, max_shard_tiles);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t launch_reduce(const void* samples, void* out, int elem_bytes, size_t n, int nsamples, int accumulate,
                         hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const dim3 block(256), grid((unsigned)((n + 255) / 256));
    if (elem_bytes == 8)
        hipLaunchKernelGGL(reduce_kernel<double>, grid, block, 0, stream, (const double*)samples, (double*)out, n,
                           nsamples, accumulate);
    else if (elem_bytes == 4)
        hipLaunchKernelGGL(reduce_kernel<float>, grid, block, 0, stream, (const float*)samples, (float*)out, n,
                           nsamples, accumulate);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t launch_quantize(const void* frame, int elem_bytes, int32_t* rgb, size_t n, int spp, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const dim3 block(256), grid((unsigned)((n + 255) / 256));
    if (elem_bytes == 8)
        hipLaunchKernelGGL(quantize_kernel<double>, grid, block, 0, stream, (const double*)frame, rgb, n, spp);
    else if (elem_bytes == 4)
        hipLaunchKernelGGL(quantize_kernel<float>, grid, block, 0, stream, (const float*)frame, rgb, n, spp);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace rtx

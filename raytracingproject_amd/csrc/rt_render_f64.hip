// rt_render_f64.hip -- fp64 reference-exact path, built with -ffp-contract=off so every
// operation rounds as in the g++ build of the reference.  Also hosts the small
// precision-agnostic kernels (unshard, quantize).
#include "rt_render_impl.h"

namespace rtx {

// The fp64 kernels (rt_tuning.f64_kernel), (id, waves_per_eu, traversal flags, block):
//  3 conservative fp32 slab tests (TRAV_F32BOX: each slab widened by a bound of its
//    rounding, so no box the exact ray enters is rejected) on persistent lanes over the
//    work queue (TRAV_PERSIST, render_lanes<EXACT>: each sample's radiance stored, ordered
//    reduction afterwards), 512-thread workgroups within 128 VGPRs: 4 waves per SIMD;
//  4 (default) kernel 3 with coherent primaries (TRAV_COH: render_coherent<double, EXACT>,
//    camera rays traced in per-tile batches, their fp64 hits queued in LDS): C2 11.9 ms,
//    C3 97.9 ms against kernel 3's 14.3 / 119.2 on the same box (f64_probe*_r03ak.jsonl).
// Both render the same frame bit for bit (the boxes only prune; spheres and triangles are
// tested in fp64; the sums are the reference's in-order fp64 additions).  Kernels 1 (fp64
// slabs, one wave per 8x8 tile: C2 26.2 ms) and 2 (kernel 3's box tests, one wave per
// tile: 23.6 ms) of rounds 1-3 were removed in r04
// (profiles/r03/f64_kernel_probe_r03{m,n,o}*.jsonl).
//  5 (default where rt_upload_scene built a sphere grid and the tuning's traversal asks for
//    it, RT_TRAV_GRID) kernel 4 walking the uniform sphere grid instead of the sphere tree:
//    the cells chosen in fp32 from the rounded ray (the listed boxes' padding covers the
//    rounding), every listed sphere tested in fp64 -- the same frame bit for bit.
//  6 (r06; never asked for: the C ABI runs it for 5 where the grid is one cell tall in y,
//    unless the traversal carries 262144) kernel 5 with the flat walk (TRAV_GFLAT).
#define RT_F64_VARIANTS(X)                                                                     \
    X(3, 4, TRAV_F32BOX | TRAV_PERSIST, 512) X(4, 4, TRAV_F32BOX | TRAV_PERSIST | TRAV_COH, 512) \
    X(5, 4, TRAV_F32BOX | TRAV_PERSIST | TRAV_COH | TRAV_GRID, 512)                               \
    X(6, 4, TRAV_F32BOX | TRAV_PERSIST | TRAV_COH | TRAV_GRID | TRAV_GFLAT, 512)

int render_f64_block(int kernel) {
#define RT_F64_BLK(K, W, T, B) \
    if (kernel == K) return B;
    RT_F64_VARIANTS(RT_F64_BLK)
#undef RT_F64_BLK
    return -1;
}

int render_f64_vgprs(bool mesh, int kernel) {
    hipFuncAttributes a;
    hipError_t e = hipErrorInvalidValue;
#define RT_F64_ATTR(K, W, T, B)                                                                            \
    if (kernel == K)                                                                                       \
        e = mesh ? hipFuncGetAttributes(&a, (const void*)render_kernel<double, true, B, W, false, T, true>) \
                 : hipFuncGetAttributes(&a, (const void*)render_kernel<double, true, B, W, false, T, false>);
    RT_F64_VARIANTS(RT_F64_ATTR)
#undef RT_F64_ATTR
    return e == hipSuccess ? a.numRegs : -1;
}

int render_f64_static_lds(bool mesh, int kernel) {
    hipFuncAttributes a;
    hipError_t e = hipErrorInvalidValue;
#define RT_F64_SLDS(K, W, T, B)                                                                            \
    if (kernel == K)                                                                                       \
        e = mesh ? hipFuncGetAttributes(&a, (const void*)render_kernel<double, true, B, W, false, T, true>) \
                 : hipFuncGetAttributes(&a, (const void*)render_kernel<double, true, B, W, false, T, false>);
    RT_F64_VARIANTS(RT_F64_SLDS)
#undef RT_F64_SLDS
    return e == hipSuccess ? (int)a.sharedSizeBytes : -1;
}

hipError_t launch_render_f64(const RenderParams& P, size_t lds_bytes, hipStream_t stream, int kernel) {
#define RT_F64_LAUNCH(K, W, T, B)                                                                          \
    if (kernel == K) {                                                                                     \
        constexpr int waves = B / 64;                                                                      \
        long items = 0; /* persistent lanes: the queue's items, resident workgroups only */                \
        for (int p = 0; p < P.nph; ++p) items += (long)P.shard_tiles * P.ph_k[p];                          \
        int grid = (int)((items + waves - 1) / waves);                                                     \
        if (grid > P.max_wgs) grid = P.max_wgs;                                                            \
        if (grid == 0) return hipSuccess;                                                                  \
        if (P.n_mnodes > 0)                                                                                \
            hipLaunchKernelGGL((render_kernel<double, true, B, W, false, T, true>), dim3(grid), dim3(B),   \
                               lds_bytes, stream, P);                                                      \
        else                                                                                               \
            hipLaunchKernelGGL((render_kernel<double, true, B, W, false, T, false>), dim3(grid), dim3(B),  \
                               lds_bytes, stream, P);                                                      \
        return hipGetLastError();                                                                          \
    }
    RT_F64_VARIANTS(RT_F64_LAUNCH)
#undef RT_F64_LAUNCH
    return hipErrorInvalidValue;
}

int render_f64_trav(int kernel) {
#define RT_F64_TRV(K, W, T, B) \
    if (kernel == K) return (T);
    RT_F64_VARIANTS(RT_F64_TRV)
#undef RT_F64_TRV
    return 0;
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

hipError_t launch_finish_u8(const void* gathered, int elem_bytes, uint8_t* rgb, int W, int H, int tiles_x,
                            int nshards, int max_shard_tiles, int spp, hipStream_t stream) {
    const dim3 block(256), grid((W + 255) / 256, H);
    if (W <= 0 || H <= 0) return hipSuccess;
    const double scale = 1.0 / spp;
    if (elem_bytes == 8)
        hipLaunchKernelGGL(finish_u8_kernel<double>, grid, block, 0, stream, (const double*)gathered, rgb, W, H,
                           tiles_x, nshards, max_shard_tiles, scale);
    else if (elem_bytes == 4)
        hipLaunchKernelGGL(finish_u8_kernel<float>, grid, block, 0, stream, (const float*)gathered, rgb, W, H,
                           tiles_x, nshards, max_shard_tiles, scale);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

// One pixel channel's fixed-point sum (and its flags) as the float out_sums value.
__device__ __forceinline__ float finalized(long long acc, uint32_t f) {
    if (f & FIX_NAN || (f & FIX_POS && f & FIX_NEG)) return __builtin_nanf("");
    if (f) return f & FIX_POS ? __builtin_huge_valf() : -__builtin_huge_valf();
    return (float)((double)acc * (1.0 / (double)(1ll << FIX_SHIFT)));
}

// fp32 fixed-point sums -> out_sums: one thread per pixel channel.
__global__ void finalize_kernel(long long* __restrict__ accum, const unsigned long long* __restrict__ packed,
                                const uint32_t* __restrict__ flags, float* __restrict__ out, size_t n) {
    const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    if (packed) {   // this launch's packed sums (units of 2^-FIX_SAMPLE_SHIFT) join the running sums
        const size_t p = e / 3;
        const int c = (int)(e % 3);
        const unsigned long long w = packed[2 * p + (c == 2 ? 1 : 0)];
        const unsigned long long u = c == 1 ? w >> 32 : c == 0 ? (w & 0xffffffffull) : w;
        accum[e] += (long long)(u << (FIX_SHIFT - FIX_SAMPLE_SHIFT));
    }
    out[e] = finalized(accum[e], (flags[e / 3] >> (3 * (e % 3))) & 7u);
}

// Continue sums the context holds no fixed-point state for: out_sums -> accum (rounded
// onto the grid), non-finite values -> flags.
__global__ void seed_accum_kernel(const float* __restrict__ out, long long* __restrict__ accum,
                                  uint32_t* __restrict__ flags, size_t npx) {
    const size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npx) return;
    uint32_t fl = 0;
    for (int c = 0; c < 3; ++c) {
        const double v = rint((double)out[p * 3 + c] * (double)(1ll << FIX_SHIFT));
        if (fabs(v) < 0x1p62) {
            accum[p * 3 + c] = (long long)v;
        } else {
            accum[p * 3 + c] = 0;
            fl |= (v != v ? FIX_NAN : v > 0 ? FIX_POS : FIX_NEG) << (3 * c);
        }
    }
    flags[p] = fl;
}

// Continue sums the context DOES hold fixed-point state for, per pixel channel: the
// state is kept only where out_sums still holds, bit for bit, what finalize_kernel last
// wrote from it; anywhere else (the caller changed the buffer, or freed it and got the
// same address back for another frame) the channel restarts from out_sums' float value,
// as for a buffer the context has never seen.
__global__ void reconcile_accum_kernel(const float* __restrict__ out, long long* __restrict__ accum,
                                       uint32_t* __restrict__ flags, size_t npx) {
    const size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npx) return;
    uint32_t fl = flags[p];
    for (int c = 0; c < 3; ++c) {
        const uint32_t fc = (fl >> (3 * c)) & 7u;
        const float have = out[p * 3 + c];
        if (__float_as_uint(finalized(accum[p * 3 + c], fc)) == __float_as_uint(have)) continue;
        const double v = rint((double)have * (double)(1ll << FIX_SHIFT));
        fl &= ~(7u << (3 * c));
        if (fabs(v) < 0x1p62) {
            accum[p * 3 + c] = (long long)v;
        } else {
            accum[p * 3 + c] = 0;
            fl |= (v != v ? FIX_NAN : v > 0 ? FIX_POS : FIX_NEG) << (3 * c);
        }
    }
    flags[p] = fl;
}

// Batched world.hit (rt_trace_rays), fp64: the reference's arithmetic (sphere.h:30-57).
hipError_t launch_trace_f64(const RenderParams& P, size_t lds_bytes, hipStream_t stream, const void* rays, int n,
                            void* hits, const int* remap) {
    if (n <= 0) return hipSuccess;
    constexpr int B = TRACE_BLOCK;
    const int grid = (n + B - 1) / B < 8192 ? (n + B - 1) / B : 8192;
    const double* r = (const double*)rays;
    TraceHit* h = (TraceHit*)hits;
    // the default fp64 kernel's box tests (conservative fp32 slabs)
    if (P.n_mnodes > 0)
        hipLaunchKernelGGL((trace_kernel<double, true, B, TRAV_F32BOX, true>), dim3(grid), dim3(B), lds_bytes, stream,
                           P, r, n, h, remap);
    else
        hipLaunchKernelGGL((trace_kernel<double, true, B, TRAV_F32BOX, false>), dim3(grid), dim3(B), lds_bytes, stream,
                           P, r, n, h, remap);
    return hipGetLastError();
}

hipError_t launch_reconcile_accum(const float* out, long long* accum, uint32_t* flags, size_t npx,
                                  hipStream_t stream) {
    if (npx == 0) return hipSuccess;
    hipLaunchKernelGGL(reconcile_accum_kernel, dim3((unsigned)((npx + 255) / 256)), dim3(256), 0, stream, out, accum,
                       flags, npx);
    return hipGetLastError();
}

hipError_t launch_finalize(long long* accum, const unsigned long long* packed, const uint32_t* flags, float* out,
                           size_t npx, hipStream_t stream) {
    const size_t n = npx * 3;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(finalize_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, accum, packed, flags,
                       out, n);
    return hipGetLastError();
}

hipError_t launch_seed_accum(const float* out, long long* accum, uint32_t* flags, size_t npx, hipStream_t stream) {
    if (npx == 0) return hipSuccess;
    hipLaunchKernelGGL(seed_accum_kernel, dim3((unsigned)((npx + 255) / 256)), dim3(256), 0, stream, out, accum,
                       flags, npx);
    return hipGetLastError();
}

}  // namespace rtx

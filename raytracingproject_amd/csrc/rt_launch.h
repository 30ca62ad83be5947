// rt_launch.h -- host-side launchers exported by the per-precision kernel translation
// units and called by the C ABI (rt_abi.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace rtx {

struct RenderParams;


// block: 256, 448, 512 or 1024 threads (4..16 tiles per workgroup, one scene copy in LDS);
// mesh: the scene has a triangle mesh (fewer instantiated variants)
bool render_f32_supported(int block, int waves_per_eu, int trav, bool mesh);
// VGPRs per lane of an instantiated kernel (-1 if unknown): sets how many workgroups share a CU
int render_f32_vgprs(int block, int waves_per_eu, int trav, bool mesh);
int render_f64_vgprs(bool mesh, int kernel);   // kernel: rt_tuning.f64_kernel (3, 4)
// static LDS bytes of an instantiated render kernel (-1: not instantiated / query failed); the
// sphere grid's walk addresses its dynamic LDS from 0, so a grid kernel must have none
int render_f32_static_lds(int block, int waves_per_eu, int trav, bool mesh);
int render_f64_static_lds(bool mesh, int kernel);
int render_f64_block(int kernel);              // its threads per workgroup (-1: no such kernel)
int render_f64_trav(int kernel);               // its traversal flags (TRAV_*)
hipError_t launch_render_f32(const RenderParams& P, size_t lds_bytes, hipStream_t stream, int block, int waves_per_eu,
                             int spec);
// instrumented builds (rt_render_diag): loop utilisation counters and timeline stamps into
// P.diag, for the (block, waves_per_eu, traversal) combinations that render frames
bool render_f32_diag_supported(int block, int waves_per_eu, int trav, bool mesh);
hipError_t launch_render_f32_diag(const RenderParams& P, size_t lds_bytes, hipStream_t stream, int trav, int block,
                                  int waves_per_eu);
hipError_t launch_render_f64(const RenderParams& P, size_t lds_bytes, hipStream_t stream, int kernel);
// batched world.hit (rt_trace_rays): n rays of 7 values (context precision) -> n rt_hit
constexpr int TRACE_BLOCK = 256;
hipError_t launch_trace_f32(const RenderParams& P, size_t lds_bytes, hipStream_t stream, const void* rays, int n,
                            void* hits, const int* remap, bool diag);
hipError_t launch_trace_f64(const RenderParams& P, size_t lds_bytes, hipStream_t stream, const void* rays, int n,
                            void* hits, const int* remap);
hipError_t launch_tape_f64(const RenderParams& P, int max_depth, const double* ray7, const double* tape, int tape_len,
                           double* out, int* used, hipStream_t stream);
// element: 4 (float/uint32) or 8 (double); channels: 1 or 3
hipError_t launch_unshard(const void* gathered, void* frame, int elem_bytes, int channels, int W, int H, int tiles_x,
                          int nshards, int max_shard_tiles, hipStream_t stream);
hipError_t launch_quantize(const void* frame, int elem_bytes, int32_t* rgb, size_t n, int spp, hipStream_t stream);
// gathered shard buffers -> row-major W*H*3 uint8 frame (unshard + write_color in one pass)
hipError_t launch_finish_u8(const void* gathered, int elem_bytes, uint8_t* rgb, int W, int H, int tiles_x,
                            int nshards, int max_shard_tiles, int spp, hipStream_t stream);
// sums of a sample-chunked launch: out[e] (+)= samples[0][e] + ... + samples[nsamples-1][e], in order
hipError_t launch_reduce(const void* samples, void* out, int elem_bytes, size_t n, int nsamples, int accumulate,
                         hipStream_t stream);
// fp32 fixed-point pixel sums (RenderParams::accum, 3 per pixel) -> float out_sums
hipError_t launch_finalize(long long* accum, const unsigned long long* packed, const uint32_t* flags, float* out,
                           size_t npx, hipStream_t stream);
// float out_sums -> fixed-point sums (continuing sums the context has no state for)
hipError_t launch_seed_accum(const float* out, long long* accum, uint32_t* flags, size_t npx, hipStream_t stream);
// continue the fixed-point sums where out still holds their finalized value, else re-seed
// that channel from out (a buffer reallocated at the same address, or changed by the caller)
hipError_t launch_reconcile_accum(const float* out, long long* accum, uint32_t* flags, size_t npx,
                                  hipStream_t stream);

}  // namespace rtx

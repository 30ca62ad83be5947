// Throughput of 32-bit integer multiplies vs 24-bit / fp32 FMA on gfx950 (one-off probe
// for the RNG hash cost).  hipcc --offload-arch=gfx950 -O3 mul_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP>
__global__ void k(uint32_t* out, uint32_t seed, int iters) {
    uint32_t a = seed ^ threadIdx.x, b = a * 3u + 1u, c = a * 5u + 7u, d = a * 11u + 13u;
    float fa = (float)a, fb = (float)b, fc = (float)c, fd = (float)d;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if (OP == 0) { a = a * b; b = b * c; c = c * d; d = d * a; }
            if (OP == 1) { a = __umul24(a, b); b = __umul24(b, c); c = __umul24(c, d); d = __umul24(d, a); }
            if (OP == 2) { fa = fmaf(fa, 1.0001f, fb); fb = fmaf(fb, 1.0001f, fc); fc = fmaf(fc, 1.0001f, fd); fd = fmaf(fd, 1.0001f, fa); }
            if (OP == 3) { a ^= b >> 15; b ^= c >> 15; c ^= d >> 15; d ^= a >> 15; }
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d + (uint32_t)(fa + fb + fc + fd);
}

int main() {
    uint32_t* out;
    (void)hipMalloc(&out, 256 * 2048 * 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const char* names[] = {"v_mul_lo_u32", "v_mul_u32_u24+add", "v_fma_f32", "xor+shift"};
    for (int op = 0; op < 4; ++op) {
        for (int rep = 0; rep < 2; ++rep) {
            const int iters = 4096;
            (void)hipEventRecord(e0);
            if (op == 0) hipLaunchKernelGGL(k<0>, dim3(2048), dim3(256), 0, 0, out, 1u, iters);
            if (op == 1) hipLaunchKernelGGL(k<1>, dim3(2048), dim3(256), 0, 0, out, 1u, iters);
            if (op == 2) hipLaunchKernelGGL(k<2>, dim3(2048), dim3(256), 0, 0, out, 1u, iters);
            if (op == 3) hipLaunchKernelGGL(k<3>, dim3(2048), dim3(256), 0, 0, out, 1u, iters);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double ops = 2048.0 * 256 * iters * 16 * 4;   // lane-ops
            if (rep) printf("%-20s %8.3f ms  %.1f Gop/s (lane ops; VALU instrs per op: see ISA)\n", names[op], ms, ops / ms / 1e6);
        }
    }
    return 0;
}

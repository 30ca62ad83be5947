// rt_render_impl.h -- the kernels, templated on precision.  Included by exactly one
// translation unit per precision (rt_render_f32.hip: FMA contraction allowed;
// rt_render_f64.hip: -ffp-contract=off, reference operation order), each of which
// instantiates them and exports plain host launchers (rt_launch.h).
#pragma once
#include "rt_device.h"
#include "rt_launch.h"

namespace rtx {

constexpr int NO_SELF = 0x7fffffff;

// Path radiance and pixel sums with explicit rounding: FP contraction may not fuse
// `acc + thr * L` differently in different inlined copies of the loop, so a frame split
// into sample ranges (rt_render_range) sums bit-identically to one launch.
// (`#pragma clang fp contract(off)`: the IR operations carry no `contract` flag, so no
// FMA forms across the inlined call; HIP's __fadd_rn is a plain `+` on this toolchain.)
__device__ __forceinline__ V3<float> mul_rn(V3<float> a, V3<float> b) {
#pragma clang fp contract(off)
    return {a.x * b.x, a.y * b.y, a.z * b.z};
}
__device__ __forceinline__ V3<float> add_rn(V3<float> a, V3<float> b) {
#pragma clang fp contract(off)
    return {a.x + b.x, a.y + b.y, a.z + b.z};
}
__device__ __forceinline__ V3<double> mul_rn(V3<double> a, V3<double> b) { return a * b; }   // TU has no contraction
__device__ __forceinline__ V3<double> add_rn(V3<double> a, V3<double> b) { return a + b; }

__device__ __forceinline__ void copy16(void* dst, const void* src, size_t bytes, int tid, int nthreads) {
    uint4* d = (uint4*)dst;
    const uint4* s = (const uint4*)src;
    const size_t n = bytes / 16;
    for (size_t k = (size_t)tid; k < n; k += (size_t)nthreads) d[k] = s[k];
}

// ---------------------------------------------------------------------------------
// fp32 render loop with persistent lanes.  The work is a queue of items (tile, sample
// range); an item is 64 pixel-chunks (one per pixel of the 8x8 tile), and a wave hands
// its items' pixel-chunks to its lanes one at a time: a lane that finishes a pixel-chunk
// takes the wave's next one (the rest of the current item, then the next item the wave
// takes from the queue, one returning atomic per item), so no lane waits for another
// until the queue runs dry.  Sums are order-free (fixed point, RenderParams::accum):
// which lane renders which pixel-chunk, and when, never changes a bit of the result.
//
// Items come in phases of decreasing size (RenderParams::ph_*): big chunks first, single
// samples last, so the work still in flight when the queue empties is small everywhere
// and the waves finish together (expensive pixels -- paths of tens of bounces in the
// crevices between spheres -- cost several times the average).
// ---------------------------------------------------------------------------------
constexpr uint32_t ITEM_NONE = 0xffffffffu;

// DIAG only: maximum of v over the wave's active lanes (scalar loop over exec)
__device__ __forceinline__ uint32_t wave_max_active(uint32_t v) {
    unsigned long long e = __builtin_amdgcn_read_exec();
    uint32_t m = 0;
    while (e) {
        const int l = __builtin_ctzll(e);
        const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)v, l);
        m = x > m ? x : m;
        e &= e - 1;
    }
    return m;
}

// The work queue is sharded per XCD (MI355X_MICROARCH.md "dequeue": one head word
// saturates at ~88 dequeues/us, so 8,192 waves starting together would queue ~0.1 ms on
// it): head q (its own 128-B line) hands out items q, q + 8, q + 16, ... to the waves of
// XCD q (HW_REG_XCC_ID; speed only -- any wave may take any item), and a wave whose head
// is exhausted takes from the other heads in turn.  One returning atomic per item per
// wave (more only at the very end), by its first active lane, broadcast to the wave.
// (Handing each XCD a band of neighbouring tiles instead, for L2 locality on meshes,
// measured 2.4 % slower on C4 and equal elsewhere: profiles/r03/ab_queue_bands_r03h/.)
constexpr int QUEUE_HEADS = 8, QUEUE_STRIDE = 32;   // words between heads (128 B)
// the v-th item of head q (ITEM_NONE past its end); PH: RenderParams or CohConst
template <class PH>
__device__ __forceinline__ uint32_t queue_item(const RenderParams& P, const PH& ph, uint32_t q, uint32_t v) {
    uint32_t nitems = 0;
    for (int p = 0; p < ph.nph; ++p) nitems += (uint32_t)P.shard_tiles * (uint32_t)ph.ph_k[p];
    const uint32_t i = v * (uint32_t)QUEUE_HEADS + q;
    return i < nitems ? i : ITEM_NONE;
}
template <class PH>
__device__ __forceinline__ uint32_t fetch_item(const RenderParams& P, const PH& ph) {
    uint32_t v = ITEM_NONE;
    if ((int)(threadIdx.x & 63) == __builtin_ctzll(__builtin_amdgcn_read_exec())) {
        const uint32_t x = (uint32_t)__builtin_amdgcn_s_getreg(6164) & 7u;   // hwreg(HW_REG_XCC_ID, 0, 4)
        for (uint32_t k = 0; k < (uint32_t)QUEUE_HEADS; ++k) {
            const uint32_t q = (x + k) & (uint32_t)(QUEUE_HEADS - 1);
            const uint32_t i = queue_item(P, ph, q, atomicAdd(P.queue + q * QUEUE_STRIDE, 1u));
            if (i != ITEM_NONE) {
                v = i;
                break;
            }
        }
    }
    return __builtin_amdgcn_readfirstlane(v);
}

// A work item decoded once per wave (all fields wave-uniform, so they live in SGPRs):
// local tile lt (-1: the queue is empty), its first sample s0 and sample count c, and the
// tile's top-left pixel (tx0, ty0).
struct ItemDec {
    int lt, s0, c, tx0, ty0;
};
// PH: where the phase tables are read from (RenderParams, or CohConst in LDS)
template <class PH>
__device__ __forceinline__ ItemDec decode_item(const RenderParams& P, const PH& ph, uint32_t item) {
    ItemDec d;
    if (item == ITEM_NONE) {
        d.lt = -1;
        d.s0 = d.c = d.tx0 = d.ty0 = 0;
        return d;
    }
    int p = 0, k = (int)item;
    while (p + 1 < ph.nph && k >= P.shard_tiles * ph.ph_k[p]) k -= P.shard_tiles * ph.ph_k[p++];
    d.lt = k / ph.ph_k[p];
    const int ci = k - d.lt * ph.ph_k[p];
    d.c = ph.ph_c[p];
    d.s0 = P.sample_begin + ph.ph_s0[p] + ci * d.c;
    const int t = d.lt * P.nshards + P.shard;
    d.ty0 = t / P.tiles_x;
    d.tx0 = (t - d.ty0 * P.tiles_x) * 8;
    d.ty0 *= 8;
    return d;
}

// EXACT (fp64, TRAV_PERSIST): the same hand-out, but each finished sample's radiance is
// stored at P.samples[s - sample_begin][pixel] (every slot written exactly once, so the
// order of completion does not matter) and reduce_kernel adds them per pixel in sample
// order afterwards -- the reference's sequential fp64 sums (camera.h:41-44); attenuations
// are multiplied innermost-first at the end of the path as in render_tiles_exact.
template <class R, int BLOCK, int TRAV, bool MESH, bool DIAG = false, bool EXACT = false>
__device__ __forceinline__ void render_lanes(const RenderParams& P, const SceneView<R>& sc, uint16_t* stack,
                                             float* facc) {
    static_assert(!EXACT || !DIAG, "no instrumented fp64 build");
    const int lane = threadIdx.x & 63;
    [[maybe_unused]] R* const samp = (R*)P.samples;
    [[maybe_unused]] const size_t npx_all = (size_t)P.shard_tiles * 64;   // EXACT: pixels per stored sample

    // this lane's pixel-chunk: pixel pix of the shard at (px, py), samples [s, s_end)
    uint32_t pix = 0;
    int pxy = 0, s = 0, s_end = 0;
    uint32_t segs = 0;
    int cnt = 0;   // samples of the current pixel-chunk
    float fx = 0.f, fy = 0.f, fz = 0.f;   // its samples, each on the 2^-FIX_SAMPLE_SHIFT grid
    if (MESH && !EXACT) facc[0] = facc[BLOCK] = facc[2 * BLOCK] = 0.f;
    bool fin = false;   // the queue ran dry for this lane
    // DIAG builds (rt_render_diag): loop utilisation and phase cycles, summed per wave
    DiagCounters dg;
    unsigned long long bounce_it = 0, bounce_act = 0, cyc_trav = 0, cyc_shade = 0, cyc_hand = 0, nflush = 0, nseg = 0;
    unsigned long long k_it1 = 0, k_it2 = 0, k_it4 = 0;   // DIAG: K-rays-per-lane model (see below)
    uint32_t ring[4] = {0, 0, 0, 0};
    uint32_t kn = 0;
    const unsigned long long t_start = DIAG ? __builtin_amdgcn_s_memtime() : 0;

    auto flush = [&]() {
        if constexpr (EXACT) {   // the samples are already stored; segment counts only
            if (P.out_segs && segs) atomicAdd(P.out_segs + pix, segs);
            segs = 0;
            return;
        }
        if (MESH) {
            fx = facc[0];
            fy = facc[BLOCK];
            fz = facc[2 * BLOCK];
            facc[0] = facc[BLOCK] = facc[2 * BLOCK] = 0.f;
        }
        uint32_t fl = 0;
        unsigned long long prg = 0, pb = 0;   // packed sums (RenderParams::accp)
        auto add = [&](float v, int c) {
#ifdef RT_DIAG_NO_FLUSH
            // measurement-only build (never shipped): the sums stay live, no atomics
            asm volatile("" ::"v"(v));
            return;
#endif
            if (v == 0.f) return;
            if (v > 0.f && v <= (float)cnt) {   // every sample <= 1: packed, exact (v is on the grid)
                const unsigned long long u = (unsigned long long)(v * (float)(1 << FIX_SAMPLE_SHIFT));
                if (c == 0) prg |= u;
                else if (c == 1) prg |= u << 32;
                else pb = u;
                return;
            }
            const double q = (double)v * (double)(1ll << FIX_SHIFT);   // an integer: v is on the grid
            if (fabs(q) < 0x1p62)
                atomicAdd((unsigned long long*)P.accum + (size_t)pix * 3 + c, (unsigned long long)(long long)q);
            else   // NaN, inf or overflow
                fl |= (q != q ? FIX_NAN : q > 0 ? FIX_POS : FIX_NEG) << (3 * c);
        };
        add(fx, 0);
        add(fy, 1);
        add(fz, 2);
        if (prg) atomicAdd(P.accp + (size_t)pix * 2, prg);
        if (pb) atomicAdd(P.accp + (size_t)pix * 2 + 1, pb);
        if (fl) atomicOr(P.accum_flags + pix, fl);
        if (P.out_segs && segs) atomicAdd(P.out_segs + pix, segs);
        fx = fy = fz = 0.f;
        segs = 0;
    };
    // pixel q (0..63) of the decoded item d (per lane; d is wave-uniform)
    auto start = [&](const ItemDec& d, int q) {
        if (d.lt < 0) {
            fin = true;
            return;
        }
        pix = (uint32_t)d.lt * 64u + (uint32_t)q;
        const int px = d.tx0 + (q & 7), py = d.ty0 + (q >> 3);
        pxy = px | (py << 16);
        s = d.s0;
        s_end = px < P.W && py < P.H && P.max_depth > 0 ? s + d.c : s;
        cnt = s_end - s;
        if constexpr (EXACT) {
            if (s_end == s)   // no path traced (outside the image, or depth 0): the samples are 0
                for (int q2 = 0; q2 < d.c; ++q2) {
                    R* o = samp + ((size_t)(d.s0 + q2 - P.sample_begin) * npx_all + pix) * 3;
                    o[0] = o[1] = o[2] = (R)0;
                }
        }
    };

    // the wave's hand-out position (wave-uniform): pixel `npx` of the current item
    ItemDec cur = decode_item(P, P, ITEM_NONE);
    int npx = 64;

    CounterRng rng;
    Ray<R> ray;
    V3<R> thr = mk((R)1, (R)1, (R)1);
    [[maybe_unused]] V3<R> att_stack[EXACT ? 64 : 1];   // EXACT: this path's attenuations (scratch)
    int nsc = 0;
    int self_id = NO_SELF;
    for (;;) {
        // lanes done with their pixel-chunk flush it and take the wave's next ones
        const unsigned long long th = DIAG ? __builtin_amdgcn_s_memtime() : 0;
        for (;;) {
            const bool need = !fin && s >= s_end;
            const unsigned long long m = __ballot(need);
            if (m == 0) break;
            const int k = __popcll(m);
            // this lane's rank among the lanes that need one (v_mbcnt, no lane-mask register)
            const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                           __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            int q = npx + rank;
            if (npx + k > 64) {   // the current item runs out: the wave takes the next one
                const ItemDec nxt = decode_item(P, P, fetch_item(P, P));
                if (need) {
                    flush();
                    if (q >= 64)
                        start(nxt, q - 64);
                    else
                        start(cur, q);
                }
                cur = nxt;
                npx = npx + k - 64;
            } else {
                if (need) {
                    flush();
                    start(cur, q);
                }
                npx += k;
            }
            if (need) nsc = -1;   // a new sample starts below
            if (DIAG && need) ++nflush;
        }
        if (DIAG) cyc_hand += __builtin_amdgcn_s_memtime() - th;
        if (!__any(!fin)) break;
        if (fin) continue;
        if (nsc < 0) {
            // the ONE inlined copy of get_ray (see render_kernel)
            rng.start(hash32(P.seed32 ^ (uint32_t)((pxy >> 16) * P.W + (pxy & 0xffff))), (uint32_t)s);
            ray = camera_ray<R>(P, pxy & 0xffff, pxy >> 16, rng);
            thr = mk((R)1, (R)1, (R)1);
            nsc = 0;
            self_id = NO_SELF;
        }
        ++segs;
        if (DIAG) ++nseg;
        bool lead = false;
        unsigned long long t0 = 0, t1 = 0;
        if (DIAG) {
            const unsigned long long e = __builtin_amdgcn_read_exec();
            lead = lane == __builtin_ctzll(e);
            if (lead) {
                ++bounce_it;
                bounce_act += (unsigned long long)__builtin_popcountll(e);
            }
            t0 = __builtin_amdgcn_s_memtime();
        }
        const Hit<R> h = closest_hit<R, EXACT, DIAG, TRAV, MESH>(sc, ray, stack, BLOCK, EXACT ? NO_SELF : self_id, &dg);
        if (DIAG) {
            t1 = __builtin_amdgcn_s_memtime();
            // what K traversals per lane per bounce iteration would cost: the wave's
            // slowest lane over K consecutive closest_hit calls, vs K slowest lanes
            const uint32_t st = dg.steps;
            dg.steps = 0;
            ring[kn & 3] = st;
            const uint32_t m1 = wave_max_active(st);
            const uint32_t m2 = (kn & 1) ? wave_max_active(st + ring[(kn - 1) & 3]) : 0u;
            const uint32_t m4 = (kn & 3) == 3 ? wave_max_active(st + ring[0] + ring[1] + ring[2]) : 0u;
            if (lead) {
                k_it1 += m1;
                k_it2 += m2;
                k_it4 += m4;
            }
            ++kn;
        }
        bool done = true;
        V3<R> L = mk((R)0, (R)0, (R)0);
        if (h.id == -1) {
            if constexpr (EXACT) {   // camera_cpu.h:19, innermost attenuation first
                L = sky(ray.d);
                for (int k = nsc - 1; k >= 0; --k) L = att_stack[k] * L;
            } else {
                L = mul_rn(thr, sky(ray.d));
            }
        } else {
            const Shade<R> sh = shade<R, MESH>(sc, ray, h);
            V3<R> att, dir;
            if (scatter<R, EXACT>(sc.mat[sh.meta & META_MAT_MASK], (sh.meta >> 24) & 3u, ray.d, sh, rng, att, dir)) {
                if constexpr (EXACT)
                    att_stack[nsc] = att;
                else
                    thr = thr * att;
                ++nsc;
                ray.o = sh.p;
                ray.d = dir;
                self_id = h.id;
                done = nsc >= P.max_depth;
            }
        }
        if (DIAG && lead) {
            cyc_trav += t1 - t0;
            cyc_shade += __builtin_amdgcn_s_memtime() - t1;
        }
        if (EXACT && done) {
            R* o = samp + ((size_t)(s - P.sample_begin) * npx_all + pix) * 3;
            o[0] = L.x;
            o[1] = L.y;
            o[2] = L.z;
            ++s;
            nsc = -1;
        } else if (done) {
            // rounded onto the grid (exact scalings), then summed exactly: at most
            // FIX_ITEM_SAMPLES values in [0, 1] on a 2^-19 grid need <= 24 bits
            constexpr float SC = (float)(1 << FIX_SAMPLE_SHIFT), ISC = 1.f / SC;
            const float qx = __builtin_rintf(L.x * SC) * ISC, qy = __builtin_rintf(L.y * SC) * ISC,
                        qz = __builtin_rintf(L.z * SC) * ISC;
            if (MESH) {
                facc[0] += qx;
                facc[BLOCK] += qy;
                facc[2 * BLOCK] += qz;
            } else {
                fx += qx;
                fy += qy;
                fz += qz;
            }
            ++s;
            nsc = -1;
        }
    }
    if (DIAG) {
        // per-wave sums: lane 0 adds the wave's phase cycles, every lane its own counts
        const bool l0 = lane == 0;
        const unsigned long long v[DIAG_SLOTS] = {bounce_it, bounce_act, dg.inner_it, dg.inner_act, dg.leaf_it,
                                                  dg.leaf_act, cyc_trav, cyc_shade, l0 ? cyc_hand : 0ull,
                                                  l0 ? __builtin_amdgcn_s_memtime() - t_start : 0ull, nseg, nflush,
                                                  k_it1, k_it2, k_it4, 0};
        for (int k = 0; k < DIAG_SLOTS; ++k)
            if (v[k]) atomicAdd(P.diag + k, v[k]);
    }
}

// The sums of cnt samples (each channel on the 2^-FIX_SAMPLE_SHIFT grid) into pixel
// pix's sums: packed per-launch words when a channel is in (0, cnt] (every sample <= 1),
// the 64-bit running sums otherwise, flags for NaN / overflow (RenderParams::accp /
// accum / accum_flags).
__device__ __forceinline__ void flush_sample(const RenderParams& P, uint32_t pix, float fx, float fy, float fz,
                                             uint32_t segs, float cnt = 1.f) {
    uint32_t fl = 0;
    unsigned long long prg = 0, pb = 0;
    auto add = [&](float v, int c) {
        if (v == 0.f) return;
        if (v > 0.f && v <= cnt) {
            const unsigned long long u = (unsigned long long)(v * (float)(1 << FIX_SAMPLE_SHIFT));
            if (c == 0) prg |= u;
            else if (c == 1) prg |= u << 32;
            else pb = u;
            return;
        }
        const double q = (double)v * (double)(1ll << FIX_SHIFT);
        if (fabs(q) < 0x1p62)
            atomicAdd((unsigned long long*)P.accum + (size_t)pix * 3 + c, (unsigned long long)(long long)q);
        else
            fl |= (q != q ? FIX_NAN : q > 0 ? FIX_POS : FIX_NEG) << (3 * c);
    };
    add(fx, 0);
    add(fy, 1);
    add(fz, 2);
    if (prg) atomicAdd(P.accp + (size_t)pix * 2, prg);
    if (pb) atomicAdd(P.accp + (size_t)pix * 2 + 1, pb);
    if (fl) atomicOr(P.accum_flags + pix, fl);
    if (P.out_segs && segs) atomicAdd(P.out_segs + pix, segs);
}

// ---------------------------------------------------------------------------------
// fp32 sphere scenes with coherent primaries (TRAV_COH).  The rays of one wave's
// traversal diverge: a wave steps until its slowest lane is done, and in render_lanes
// only 39 % (nodes) / 32 % (spheres) of the lane-slots do work -- yet camera rays of one
// tile at one sample, traced together, keep 87 % / 85 % (diag at depth 1): they visit
// the same nodes in the same order.  So camera rays are traced apart from the rest:
//   * batch: the wave traces sample s of all 64 pixels of its current work item (tile,
//     samples [s0, s0 + c)) -- one coherent wave of camera rays.  Misses (the sky) are
//     finished on the spot; hits go to the wave's FIFO of primary hits in LDS;
//   * bounce loop: a lane whose path ended pops the next primary hit and regenerates its
//     camera ray (same RNG stream); then ONE shade pass serves popped primaries and
//     scattered rays alike, so the wave shades once per bounce instead of twice.  Batches
//     run when the FIFO holds fewer hits than lanes waiting; lanes are refilled until
//     fewer than coh_refill of them idle.  Only scattered rays are traced in the bounce
//     loop.
// A finished sample of the current item is added to the item's pixel sums in LDS (exact:
// <= 32 values in [0, 1] on the 2^-19 grid), which go to HBM once per pixel when the
// wave moves on to its next item; samples of earlier items (paths still in flight at
// the switch) and samples outside [0, 1] go straight to the fixed-point sums.  Either
// way the sums are order-free, so which lane shades which path never changes a bit of
// the frame; every camera ray is traced by the batch's code, every scattered ray by the
// bounce loop's.
// ---------------------------------------------------------------------------------
// EXACT (fp64, f64_kernel 4): the same structure in the reference's arithmetic -- camera
// rays from the fp64 camera (camera_ray<double>), fp64 hit distances in the FIFO,
// attenuations multiplied innermost-first at the end of the path, and each finished
// sample stored at P.samples[s - sample_begin][pixel] for the ordered reduction (no LDS
// sums: fp64 sums must follow sample order).
template <class R, bool EXACT, int BLOCK, int TRAV, bool MESH, bool DIAG = false>
__device__ __forceinline__ void render_coherent(const RenderParams& P0, const SceneView<R>& sc, uint16_t* stack,
                                                CohEntryX<R, MESH>* fifo, float* isum, const CohConst& kc) {
    static_assert(!EXACT || (sizeof(R) == 8 && !DIAG), "EXACT: fp64, no instrumented build");
    // P0 is the kernel's argument (render_kernel's RenderParams, at offset 0 of the kernel-
    // argument segment).  Its fields are read through a pointer into that segment which the
    // compiler cannot see through, renewed every bounce round, so that each round scalar-loads
    // what it uses instead of the whole kernel holding ~40 words of it in SGPRs -- which the
    // allocator spilled to VGPR lanes and read back with a VALU v_readlane per use (C3 kernel:
    // SGPR spills 72 -> 32, v_readlane 392 -> 85 in the code; C3 -0.2 %, C5 -0.4 %, C4's VGPR
    // spills 16 -> 10 -- but the mesh-only C4 kernel ran 12 % slower that way, 44.7 against
    // 39.9-40.1 ms, so it keeps P0; profiles/r06/r06ac, r06ad)
    constexpr bool LAUNDER = !MESH || (TRAV & TRAV_GRID) != 0;
    typedef __attribute__((address_space(4))) const RenderParams KArg;
    auto kernarg = []() {
        KArg* p = (KArg*)__builtin_amdgcn_kernarg_segment_ptr();
        if constexpr (LAUNDER) asm volatile("" : "+s"(p));
        return p;
    };
    [[maybe_unused]] KArg* Pp = kernarg();
#define P (LAUNDER ? *(const RenderParams*)Pp : P0)
    const float* cam = kc.cam;
    constexpr float SC = (float)(1 << FIX_SAMPLE_SHIFT), ISC = 1.f / SC;
    constexpr int TR = TRAV & ~(TRAV_COH | TRAV_NOSUM | TRAV_PERSIST);   // closest_hit's flags
    constexpr bool SUMS = !EXACT && (TRAV & TRAV_NOSUM) == 0;   // the item's pixel sums in LDS
    [[maybe_unused]] R* const samp = (R*)P.samples;                   // EXACT: stored samples
    [[maybe_unused]] const size_t npx_all = (size_t)P.shard_tiles * 64;
    // fp32: the defocus disk's rejected candidates ride in the FIFO entry (bits 28-31 of sid;
    // 15: fifteen or more, drawn again), so that the pop regenerates the batch's ray without
    // the rejection loop -- its draws are skipped in one add (r06ar: C3 -1.6 %, same frames;
    // r06as: the mixed kernels -1.5 %).  Not in the kernels that trace meshes without the
    // sphere grid: C4's kernel (no defocus) spilled 3 more registers with it, +1.7 GB of
    // scratch traffic per launch at equal time (r06av against r06aq).
#ifndef RT_KDEF_MESH
#define RT_KDEF_MESH 1
#endif
    constexpr bool KDEF = !EXACT && (!MESH || (RT_KDEF_MESH && (TRAV & TRAV_GRID) != 0));
    static_assert(MAX_LEAF_FIRST + MAX_BIG + 16 <= 0xfff, "sphere hit id + 16 must fit sid bits 16-27");
    auto cam_ray = [&](int px, int py, CounterRng& rr, int kdef = -1, int* kout = nullptr) -> Ray<R> {
        if constexpr (EXACT)
            return camera_ray<R>(P, px, py, rr);
        else
            return camera_ray_lds(cam, P.defocus, px, py, rr, kdef, kout);
    };
    constexpr int FIFO = coh_fifo_entries(TRAV);       // primary hits the wave's FIFO holds
    const int lane = threadIdx.x & 63;
    DiagCounters dg, dgb;
    unsigned long long n_bounce = 0, n_live = 0, cyc_trav = 0, cyc_shade = 0, cyc_batch = 0, n_paths = 0, n_seg = 0,
                       n_batch = 0, n_pop = 0;
    const unsigned long long t_start = DIAG ? __builtin_amdgcn_s_memtime() : 0;
    // DIAG: the wave's timeline in s_memrealtime ticks (start, queue found dry) and the
    // bounce iterations after the queue ran dry
    const unsigned long long rt_start = DIAG ? __builtin_amdgcn_s_memrealtime() : 0;
    unsigned long long rt_dry = 0, n_drain = 0;
    unsigned long long n_in_item = 0, n_direct = 0, n_item_flush = 0;   // framebuffer traffic

    // wave-uniform: the FIFO (head, count) and the batch cursor (item cur, next sample bi)
    uint32_t head = 0, count = 0;
    ItemDec cur = decode_item(P, P, ITEM_NONE);
    int bi = 0;
    bool dry = false;       // the queue ran dry: no more batches
    if (SUMS) isum[lane] = isum[64 + lane] = isum[128 + lane] = 0.f;

    // a finished sample: into the current item's LDS sums, or straight to HBM
    // this lane's path: eligible for the LDS sums while its item is the wave's current one
    bool elig = false;
    auto finish = [&](uint32_t pp, bool in_item, V3<R> L, uint32_t sg, uint32_t srel) {
        if constexpr (EXACT) {
            R* o = samp + ((size_t)srel * npx_all + pp) * 3;
            o[0] = L.x;
            o[1] = L.y;
            o[2] = L.z;
            if (P.out_segs && sg) atomicAdd(P.out_segs + pp, sg);
            return;
        }
        const float qx = __builtin_rintf(L.x * SC) * ISC, qy = __builtin_rintf(L.y * SC) * ISC,
                    qz = __builtin_rintf(L.z * SC) * ISC;
        const bool in01 = qx >= 0.f && qx <= 1.f && qy >= 0.f && qy <= 1.f && qz >= 0.f && qz <= 1.f;
        if (SUMS && in_item && in01) {
            const uint32_t q = pp & 63u;
            if (qx != 0.f) atomicAdd(isum + q, qx);
            if (qy != 0.f) atomicAdd(isum + 64 + q, qy);
            if (qz != 0.f) atomicAdd(isum + 128 + q, qz);
            if (P.out_segs && sg) atomicAdd(P.out_segs + pp, sg);
            if (DIAG) ++n_in_item;
        } else {
            flush_sample(P, pp, qx, qy, qz, sg);
            if (DIAG) ++n_direct;
        }
        if (DIAG) ++n_paths;
    };

    auto batch = [&]() {
        const unsigned long long tb = DIAG ? __builtin_amdgcn_s_memtime() : 0;
        if (bi >= cur.c) {
            if (SUMS && cur.lt >= 0) {   // the item's pixel sums to HBM: lane q has pixel q
                const float fx = isum[lane], fy = isum[64 + lane], fz = isum[128 + lane];
                if (fx != 0.f || fy != 0.f || fz != 0.f) {
                    flush_sample(P, (uint32_t)cur.lt * 64u + (uint32_t)lane, fx, fy, fz, 0u, (float)cur.c);
                    if (DIAG) ++n_item_flush;
                }
                isum[lane] = isum[64 + lane] = isum[128 + lane] = 0.f;
            }
            cur = decode_item(P, kc, fetch_item(P, kc));
            bi = 0;
            elig = false;   // paths of the old item still in flight flush to HBM (the whole wave runs this)
            if (cur.lt < 0) {
                dry = true;
                if (DIAG) rt_dry = __builtin_amdgcn_s_memrealtime();
                return;
            }
        }
        const int s = cur.s0 + bi++;
        const int px = cur.tx0 + (lane & 7), py = cur.ty0 + (lane >> 3);
        const uint32_t pp = (uint32_t)cur.lt * 64u + (uint32_t)lane;
        bool hit = false;
        Hit<R> hb;
        hb.t = (R)0;
        hb.id = -1;
        [[maybe_unused]] int kd = 15;
        if (px < P.W && py < P.H && P.max_depth > 0) {
            CounterRng r2;
            r2.start(hash32(P.seed32 ^ (uint32_t)(py * P.W + px)), (uint32_t)s);
            const Ray<R> pr = KDEF ? cam_ray(px, py, r2, -1, &kd) : cam_ray(px, py, r2);
            hb = closest_hit<R, EXACT, DIAG, TR, MESH>(sc, pr, stack, BLOCK, NO_SELF, &dgb);
            if (hb.id == -1) {   // sky: the path ends here (camera_cpu.h:23-25 with attenuation 1)
                finish(pp, true, sky(pr.d), 1u, (uint32_t)(s - P.sample_begin));
            } else {
                hit = true;
            }
        } else if constexpr (EXACT) {   // no path (outside the image, depth 0): the sample is 0
            finish(pp, true, mk((R)0, (R)0, (R)0), 0u, (uint32_t)(s - P.sample_begin));
        }
        const unsigned long long hm = __ballot(hit);
        if (hit) {
            const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(hm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)hm, 0u));
            CohEntryX<R, MESH> e;
            e.t = hb.t;
            e.pix = pp;
            if constexpr (MESH) {
                e.sid = (uint32_t)(s - P.sample_begin);
                if constexpr (KDEF) e.sid |= (uint32_t)min(kd, 15) << 28;
                e.id = hb.id;
            } else {
                e.sid = (uint32_t)(s - P.sample_begin) | ((uint32_t)(hb.id + 16) << 16);
                if constexpr (KDEF) e.sid |= (uint32_t)min(kd, 15) << 28;
            }
            fifo[(head + count + r) & (FIFO - 1)] = e;
        }
        count += (uint32_t)__popcll(hm);
        if (DIAG && lane == 0) {
            ++n_batch;
            cyc_batch += __builtin_amdgcn_s_memtime() - tb;
        }
    };

    // this lane's path
    bool live = false, ready = false, fin = false;   // holds a path; holds a hit to shade; no work left
    uint32_t pix = 0;
    uint32_t psid = 0;   // EXACT: the path's sample - sample_begin
    V3<R> thr = mk((R)1, (R)1, (R)1);
    [[maybe_unused]] V3<R> att_stack[EXACT ? 64 : 1];   // EXACT: the path's attenuations (scratch)
    CounterRng rng;
    rng.st = 0;
    int nsc = 0, self = NO_SELF;
    // coh_parks: the throughput and scatter count live in LDS (COH_PARK_BYTES, lane-strided),
    // touched only where a hit is shaded or a path ends instead of held across the trace
    constexpr bool PARK = coh_parks(MESH, TRAV, EXACT);
    [[maybe_unused]] float* const park =
        (float*)((unsigned char*)fifo + (size_t)FIFO * sizeof(CohEntryX<R, MESH>) + (SUMS ? COH_SUM_BYTES : 0)) + lane;
    auto park_thr = [&]() -> V3<R> { return mk((R)park[0], (R)park[64], (R)park[128]); };
    auto park_nsc = [&]() -> int { return __float_as_int(park[192]); };
    auto park_set = [&](V3<R> t, int n) {
        park[0] = (float)t.x;
        park[64] = (float)t.y;
        park[128] = (float)t.z;
        park[192] = __int_as_float(n);
    };
    Ray<R> ray;
    ray.o = ray.d = thr;
    ray.time = (R)0;
    Hit<R> h;
    h.t = (R)0;
    h.td = 0.0;
    h.id = -1;
    // radiance of a path that left the scene (camera_cpu.h:19-25): EXACT multiplies the
    // attenuations innermost-first, as the reference recursion associates them
    auto sky_L = [&]() -> V3<R> {
        if constexpr (EXACT) {
            V3<R> L = sky(ray.d);
            for (int k = nsc - 1; k >= 0; --k) L = att_stack[k] * L;
            return L;
        } else if constexpr (PARK) {
            return mul_rn(park_thr(), sky(ray.d));
        } else {
            return mul_rn(thr, sky(ray.d));
        }
    };

    for (;;) {
        if constexpr (LAUNDER) Pp = kernarg();   // (a new opaque copy: nothing read through it is hoisted out of the round)
        const unsigned long long tsh = DIAG ? __builtin_amdgcn_s_memtime() : 0;
        // ---- shade: misses end their paths, free lanes pop primary hits, all hits shade
        for (;;) {
            // a ray that left the scene ends its path here (camera_cpu.h:23-25), before the
            // pops, so that the lanes it frees shade their next camera hit in this round
            // together with the lanes shading their own hits (one pass of the scatter code)
            if (ready && h.id == -1) {
                ready = false;
                if constexpr (PARK)
                    finish(pix, elig, sky_L(), (uint32_t)park_nsc() + 1u, psid);
                else
                    finish(pix, elig, sky_L(), (uint32_t)nsc + 1u, psid);
                live = false;
            }
            // lanes without a path pop a primary hit (batches refill the FIFO)
            for (;;) {
                const bool need = !fin && !live;
                const unsigned long long m = __ballot(need);
                if (m == 0) break;
                const uint32_t k = (uint32_t)__popcll(m);
                // a batch appends up to 64 hits: it runs when the FIFO has room for them
                // (always, at 128 entries: count < k <= 64); otherwise the hits already
                // there are popped first and the lanes still waiting batch next time round
                if (count < k && !dry && count + 64u <= (uint32_t)FIFO) {
                    batch();
                    continue;
                }
                if (need) {
                    const uint32_t r =
                        __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                    if (r < count) {
                        const CohEntryX<R, MESH> e = fifo[(head + r) & (FIFO - 1)];
                        pix = e.pix;
                        if constexpr (EXACT) psid = e.sid & 0xffffu;
                        const int lt = (int)(pix >> 6), q = (int)(pix & 63u), s = P.sample_begin + (int)(e.sid & 0xffffu);
                        const int t = lt * P.nshards + P.shard;
                        // t / tiles_x (RenderParams::tiles_x_inv; r06az: C3 -1.2 %, frames identical;
                        // the mesh-only kernels, which keep P0 in registers, spilled 3 more with it)
                        const int ty = LAUNDER ? (int)fma((double)t, P.tiles_x_inv, P.tiles_x_inv_half) : t / P.tiles_x;
                        const int px = (t - ty * P.tiles_x) * 8 + (q & 7), py = ty * 8 + (q >> 3);
                        elig = lt == cur.lt && s >= cur.s0 && s < cur.s0 + cur.c;
                        rng.start(hash32(P.seed32 ^ (uint32_t)(py * P.W + px)), (uint32_t)s);
                        if constexpr (KDEF) {
                            const int kd = (int)(e.sid >> 28);
                            ray = cam_ray(px, py, rng, kd == 15 ? -1 : kd);
                        } else {
                            ray = cam_ray(px, py, rng);   // the batch's ray, regenerated
                        }
                        h.t = e.t;
                        h.td = (double)e.t;
                        if constexpr (MESH)
                            h.id = e.id;
                        else
                            h.id = (int)((e.sid >> 16) & (KDEF ? 0xfffu : 0xffffu)) - 16;
                        if constexpr (PARK) {
                            park_set(mk((R)1, (R)1, (R)1), 0);
                        } else {
                            thr = mk((R)1, (R)1, (R)1);
                            nsc = 0;
                        }
                        self = NO_SELF;
                        live = ready = true;
                        if (DIAG) ++n_pop;
                    } else if (dry) {
                        fin = true;   // the FIFO is empty and the queue dry
                    }
                }
                const uint32_t took = k < count ? k : count;
                head += took;
                count -= took;
            }
            if (ready) {   // a hit: hit record, scatter (material.h)
                ready = false;
                bool done = true;
                const Shade<R> sh = shade<R, MESH>(sc, ray, h);
                V3<R> att, dir;
                if (scatter<R, EXACT>(sc.mat[sh.meta & META_MAT_MASK], (sh.meta >> 24) & 3u, ray.d, sh, rng, att,
                                      dir)) {
                    if constexpr (PARK) {
                        nsc = park_nsc();
                        park_set(park_thr() * att, nsc + 1);
                    } else if constexpr (EXACT) {
                        att_stack[nsc] = att;
                    } else {
                        thr = thr * att;
                    }
                    ++nsc;
                    ray.o = sh.p;
                    ray.d = dir;
                    self = h.id;
                    done = nsc >= P.max_depth;
                }
                if (done) {
                    // absorbed, or the depth limit: no radiance.  Traced segments: one per
                    // scatter, plus the last ray unless the depth limit ended the path (its
                    // scattered ray is never traced)
                    if constexpr (PARK) nsc = park_nsc();
                    finish(pix, elig, mk((R)0, (R)0, (R)0), (uint32_t)nsc + (nsc >= P.max_depth ? 0u : 1u), psid);
                    live = false;
                }
            }
            // another round only while enough lanes hold no ray (a round costs the whole wave;
            // the few left sit out one traversal and pop next time)
            const int idle = __popcll(__ballot(!fin && !live));
            if (idle == 0 || (idle < P.coh_refill && __any(live))) break;
        }
        const unsigned long long ttr = DIAG ? __builtin_amdgcn_s_memtime() : 0;
        if (DIAG && lane == 0) cyc_shade += ttr - tsh;
        if (!__any(live)) break;   // (idle lanes with work left keep the shade loop going)
        // ---- trace the scattered rays
        if (live) {
            if (DIAG) {
                const unsigned long long e = __builtin_amdgcn_read_exec();
                if (lane == __builtin_ctzll(e)) {
                    ++n_bounce;
                    n_live += (unsigned long long)__builtin_popcountll(e);
                    if (dry) ++n_drain;
                }
            }
            if (DIAG) ++n_seg;
            h = closest_hit<R, EXACT, DIAG, TR, MESH>(sc, ray, stack, BLOCK, EXACT ? NO_SELF : self, &dg);
            ready = true;
        }
        if (DIAG && lane == 0) cyc_trav += __builtin_amdgcn_s_memtime() - ttr;
    }
    if (DIAG) {
        const bool l0 = lane == 0;
        const unsigned long long v[DIAG_SLOTS] = {n_bounce, n_live, dg.inner_it, dg.inner_act, dg.leaf_it,
                                                  dg.leaf_act, l0 ? cyc_trav : 0ull, l0 ? cyc_shade : 0ull,
                                                  l0 ? cyc_batch : 0ull,
                                                  l0 ? __builtin_amdgcn_s_memtime() - t_start : 0ull, n_seg, n_paths,
                                                  n_batch, dgb.inner_it + dgb.leaf_it, dgb.inner_act + dgb.leaf_act,
                                                  n_pop};
        for (int k = 0; k < 16; ++k)
            if (v[k]) atomicAdd(P.diag + k, v[k]);
        if (n_drain) atomicAdd(P.diag + 23, n_drain);   // counted by varying lanes
        if (n_in_item) atomicAdd(P.diag + 24, n_in_item);
        if (n_direct) atomicAdd(P.diag + 25, n_direct);
        if (n_item_flush) atomicAdd(P.diag + 26, n_item_flush);
        if constexpr (MESH) {   // mesh BVH loops (batches and bounces together)
            const unsigned long long mv[4] = {dg.mnode_it + dgb.mnode_it, dg.mnode_act + dgb.mnode_act,
                                              dg.mtri_it + dgb.mtri_it, dg.mtri_act + dgb.mtri_act};
            for (int k = 0; k < 4; ++k)
                if (mv[k]) atomicAdd(P.diag + 27 + k, mv[k]);
        }
        if (l0) {
            const unsigned long long rt_end = __builtin_amdgcn_s_memrealtime();
            if (!dry) rt_dry = rt_end;
            atomicMax(P.diag + 16, rt_end);
            atomicMax(P.diag + 17, ~rt_start);
            atomicAdd(P.diag + 18, rt_end - rt_dry);
            atomicAdd(P.diag + 19, rt_dry - rt_start);
            atomicMax(P.diag + 20, ~rt_dry);
            atomicMax(P.diag + 21, rt_dry);
            atomicAdd(P.diag + 22, 1ull);
        }
    }
#undef P
}

// The scene copy render_kernel and trace_kernel keep in LDS: BVH nodes, spheres,
// materials and big spheres, each copied once per workgroup by 16-B loads; then one
// traversal-stack column per lane (s_stack[k * BLOCK + tid]) and, with a mesh, P.mstack
// mesh-stack entries per lane (s_mstack).  The caller synchronises the workgroup before use.
template <class R, int BLOCK, int TRAV, bool MESH>
__device__ __forceinline__ SceneView<R> load_scene_lds(const RenderParams& P, unsigned char* smem, uint16_t*& s_stack,
                                                       uint32_t*& s_mstack) {
    using Sph = typename Prec<R>::Sph;
    using Mat = typename Prec<R>::Mat;
    const size_t nb_nodes = (size_t)P.n_nodes * sizeof(Node);
    const size_t nb_sph = (size_t)P.n_spheres * sizeof(Sph);
    const size_t nb_mat = (size_t)P.n_mats * sizeof(Mat);
    const size_t nb_big = (size_t)P.n_big * sizeof(SphereD);
    const size_t nb_bigf = (size_t)P.n_big * sizeof(BigF);
    unsigned char* base = smem;
    Node* s_nodes = (Node*)base;
    base += nb_nodes;
    Sph* s_sph = (Sph*)base;
    base += nb_sph;
    Mat* s_mat = (Mat*)base;
    base += nb_mat;
    SphereD* s_big = (SphereD*)base;
    base += nb_big;
    BigF* s_bigf = (BigF*)base;
    base += nb_bigf;
    s_stack = (uint16_t*)base;
    base += ((size_t)BLOCK * (size_t)P.stack_size * 2 + 15) & ~(size_t)15;
    s_mstack = (uint32_t*)base;
    const int tid = threadIdx.x;
    copy16(s_nodes, P.nodes, nb_nodes, tid, BLOCK);
    copy16(s_sph, P.spheres, nb_sph, tid, BLOCK);
    copy16(s_mat, P.mats, nb_mat, tid, BLOCK);
    copy16(s_big, P.big, nb_big, tid, BLOCK);
    copy16(s_bigf, P.bigf, nb_bigf, tid, BLOCK);
    SceneView<R> sc;
    sc.nodes = s_nodes;
    sc.sph = s_sph;
    sc.mat = s_mat;
    sc.big = s_big;
    sc.bigf = s_bigf;
    sc.n_nodes = P.n_nodes;
    sc.n_big = P.n_big;
    sc.n_front = P.n_front;
    sc.mnodes = P.mnodes;
    sc.tris = (const typename Prec<R>::Tri*)P.tris;
    sc.tmeta = P.tmeta;
    sc.n_mnodes = MESH ? P.n_mnodes : 0;
    sc.mstack = s_mstack + tid;
    sc.n_mstack = MESH ? P.mstack : 0;
    sc.box_extent = P.box_extent;
    for (int a = 0; a < 6; ++a) sc.mbox[a] = P.mbox[a];
    sc.grid = P.grid;
    // (the kernel arguments are RenderParams: the header's copy there, by address, without
    // taking P's address -- which would copy all of P to scratch)
    sc.gridp = (const __attribute__((address_space(4))) GridHdr*)((const __attribute__((address_space(4))) char*)
                                                                       __builtin_amdgcn_kernarg_segment_ptr() +
                                                                   offsetof(RenderParams, grid));
    return sc;
}


// ---------------------------------------------------------------------------------
// The megakernel: camera::render's pixel x sample loop (camera.h:37-47) with the
// ray_color recursion (camera_cpu.h:8-26) unrolled into a per-lane bounce loop.
//
//   * one wave = one 8x8 tile of the shard, one lane = one pixel;
//   * the scene (BVH nodes, spheres, materials, big spheres) is copied to LDS once per
//     workgroup; each lane's traversal stack is an LDS column (stack[k*BLOCK + tid]);
//   * path regeneration: when a lane's path ends (sky, absorbed, depth limit) it adds
//     the path's colour to its pixel sum and immediately starts its next sample, so the
//     wave keeps all lanes tracing until every lane has done its spp samples; each
//     lane still sums its samples in order 0..spp-1 (camera.h:41-44), keeping the
//     result deterministic and identical for any tiling or GPU count;
//   * EXACT (fp64): attenuations are kept per bounce and multiplied innermost-first at
//     the end of the path, the association of the reference recursion
//     (camera_cpu.h:19: attenuation * ray_color(scattered, depth-1)).
// ---------------------------------------------------------------------------------
template <class R, bool EXACT, int BLOCK, int MINW = 1, bool DIAG = false, int TRAV = 0, bool MESH = false>
__global__ __attribute__((amdgpu_flat_work_group_size(1, BLOCK), amdgpu_waves_per_eu(MINW))) void render_kernel(
    RenderParams P) {
    static_assert(!EXACT || sizeof(R) == 8, "EXACT needs fp64");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

    using Sph = typename Prec<R>::Sph;
    using Mat = typename Prec<R>::Mat;
    const size_t nb_nodes = (size_t)P.n_nodes * sizeof(Node);
    const size_t nb_sph = (size_t)P.n_spheres * sizeof(Sph);
    const size_t nb_mat = (size_t)P.n_mats * sizeof(Mat);
    const size_t nb_big = (size_t)P.n_big * sizeof(SphereD);
    const size_t nb_bigf = (size_t)P.n_big * sizeof(BigF);
    unsigned char* base = smem;
    Node* s_nodes = (Node*)base;
    base += nb_nodes;
    Sph* s_sph = (Sph*)base;
    base += nb_sph;
    Mat* s_mat = (Mat*)base;
    base += nb_mat;
    SphereD* s_big = (SphereD*)base;
    base += nb_big;
    BigF* s_bigf = (BigF*)base;
    base += nb_bigf;
    uint16_t* s_stack = (uint16_t*)base;
    base += ((size_t)BLOCK * (size_t)P.stack_size * 2 + 15) & ~(size_t)15;
    uint32_t* s_mstack = (uint32_t*)base;   // MESH: P.mstack entries per lane

    const int tid = threadIdx.x;
    copy16(s_nodes, P.nodes, nb_nodes, tid, BLOCK);
    copy16(s_sph, P.spheres, nb_sph, tid, BLOCK);
    copy16(s_mat, P.mats, nb_mat, tid, BLOCK);
    copy16(s_big, P.big, nb_big, tid, BLOCK);
    copy16(s_bigf, P.bigf, nb_bigf, tid, BLOCK);
    if constexpr ((TRAV & TRAV_COH) != 0) {
        // the camera vectors and phase tables (CohConst), after the per-wave regions
        constexpr size_t WB =
            coh_wave_bytes(MESH, (TRAV & TRAV_NOSUM) == 0, coh_fifo_entries(TRAV), EXACT, coh_parks(MESH, TRAV, EXACT));
        CohConst* kc = (CohConst*)((unsigned char*)(s_mstack + (size_t)BLOCK * P.mstack) + (size_t)(BLOCK / 64) * WB);
        if (tid == 0) {
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                kc->cam[k] = P.f_center[k];
                kc->cam[3 + k] = P.f_p00[k];
                kc->cam[6 + k] = P.f_du[k];
                kc->cam[9 + k] = P.f_dv[k];
                kc->cam[12 + k] = P.f_ddu[k];
                kc->cam[15 + k] = P.f_ddv[k];
            }
            kc->nph = P.nph;
#pragma unroll
            for (int k = 0; k < MAX_PHASES; ++k) {
                kc->ph_s0[k] = P.ph_s0[k];
                kc->ph_c[k] = P.ph_c[k];
                kc->ph_k[k] = P.ph_k[k];
            }
        }
    }
    __syncthreads();

    SceneView<R> sc;
    sc.nodes = s_nodes;
    sc.sph = s_sph;
    sc.mat = s_mat;
    sc.big = s_big;
    sc.bigf = s_bigf;
    sc.n_nodes = P.n_nodes;
    sc.n_big = P.n_big;
    sc.n_front = P.n_front;
    sc.mnodes = P.mnodes;
    sc.tris = (const typename Prec<R>::Tri*)P.tris;
    sc.tmeta = P.tmeta;
    sc.n_mnodes = MESH ? P.n_mnodes : 0;
    sc.mstack = s_mstack + tid;
    sc.n_mstack = MESH ? P.mstack : 0;
    sc.box_extent = P.box_extent;
    for (int a = 0; a < 6; ++a) sc.mbox[a] = P.mbox[a];
    sc.grid = P.grid;
    // (the kernel arguments are RenderParams: the header's copy there, by address, without
    // taking P's address -- which would copy all of P to scratch)
    sc.gridp = (const __attribute__((address_space(4))) GridHdr*)((const __attribute__((address_space(4))) char*)
                                                                       __builtin_amdgcn_kernarg_segment_ptr() +
                                                                   offsetof(RenderParams, grid));
    uint16_t* stack = s_stack + tid;
    if constexpr ((TRAV & TRAV_COH) != 0) {
        // coherent primaries: per wave a FIFO of primary hits and (fp32) the item sums,
        // after the mesh stacks (none for sphere scenes), then the CohConst block
        constexpr size_t WB =
            coh_wave_bytes(MESH, (TRAV & TRAV_NOSUM) == 0, coh_fifo_entries(TRAV), EXACT, coh_parks(MESH, TRAV, EXACT));
        unsigned char* r0 = (unsigned char*)(s_mstack + (size_t)BLOCK * P.mstack);
        unsigned char* w = r0 + (size_t)(tid >> 6) * WB;
        const CohConst* kc = (const CohConst*)(r0 + (size_t)(BLOCK / 64) * WB);
        // (P must be this kernel's argument, its first: render_coherent re-reads it from the
        // kernel-argument segment)
        render_coherent<R, EXACT, BLOCK, TRAV, MESH, DIAG>(
            P, sc, stack, (CohEntryX<R, MESH>*)w, (float*)(w + coh_fifo_entries(TRAV) * sizeof(CohEntryX<R, MESH>)),
            *kc);
    } else if constexpr (!EXACT) {
        // fp32: persistent lanes over the item queue (fixed-point sums, render_lanes)
        render_lanes<R, BLOCK, TRAV, MESH, DIAG>(P, sc, stack, (float*)(s_mstack + (size_t)BLOCK * P.mstack) + tid);
    } else {
        // fp64: the same persistent lanes, samples stored for the ordered reduction
        static_assert(!EXACT || (TRAV & TRAV_PERSIST) != 0, "fp64 kernels run on persistent lanes");
        render_lanes<R, BLOCK, TRAV, MESH, false, true>(P, sc, stack, nullptr);
    }
}

// ---------------------------------------------------------------------------------
// Batched world.hit (rt_trace_rays): hittable_list::hit / bvh_node::hit
// (hittable_list.h:25-39, bvh.h:16-24) over (0.001, inf) for many rays, one ray per lane
// (grid-stride), the scene in LDS as in render_kernel; the hit record of the closest hit
// (hit_record, hittable.h:7-22: p, normal, front_face, material) -- shade() -- written per
// ray.  ids are mapped back to the caller's input order (remap: BVH sphere position ->
// input index; big sphere k -> remap[n_spheres + k]; triangle k (BVH leaf order) ->
// remap[n_spheres + n_big + k]).  DIAG counts the node / sphere loop lane utilisation.
// ---------------------------------------------------------------------------------
struct TraceHit {   // = rt_hit (include/rt_hip.h)
    double t, p[3], normal[3];
    int32_t id, front_face, mat, pad;
};
static_assert(sizeof(TraceHit) == 72, "rt_hit");

template <class R, bool EXACT, int BLOCK, int TRAV, bool MESH, bool DIAG = false>
__global__ __launch_bounds__(BLOCK) void trace_kernel(RenderParams P, const R* __restrict__ rays, int n,
                                                      TraceHit* __restrict__ hits, const int* __restrict__ remap) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint16_t* s_stack;
    uint32_t* s_mstack;
    const SceneView<R> sc = load_scene_lds<R, BLOCK, TRAV, MESH>(P, smem, s_stack, s_mstack);
    __syncthreads();
    uint16_t* stack = s_stack + threadIdx.x;
    DiagCounters dg;
    for (int base = blockIdx.x * BLOCK; base < n; base += gridDim.x * BLOCK) {
        const int i = base + (int)threadIdx.x;
        if (i >= n) break;
        const R* q = rays + (size_t)i * 7;
        Ray<R> ray;
        ray.o = mk(q[0], q[1], q[2]);
        ray.d = mk(q[3], q[4], q[5]);
        ray.time = q[6];
        const Hit<R> h = closest_hit<R, EXACT, DIAG, TRAV, MESH>(sc, ray, stack, BLOCK, NO_SELF, &dg);
        TraceHit o{};
        o.id = -1;
        if (h.id != -1) {
            const Shade<R> sh = shade<R, MESH>(sc, ray, h);
            o.t = EXACT && h.id <= -2 ? h.td : (double)h.t;   // (fp32 keeps no td: its t is exact in h.t)
            o.p[0] = (double)sh.p.x;
            o.p[1] = (double)sh.p.y;
            o.p[2] = (double)sh.p.z;
            o.normal[0] = (double)sh.normal.x;
            o.normal[1] = (double)sh.normal.y;
            o.normal[2] = (double)sh.normal.z;
            o.front_face = sh.front_face ? 1 : 0;
            o.mat = (int32_t)(sh.meta & META_MAT_MASK);
            const int slot = h.id >= MESH_HIT_BASE ? P.n_spheres + P.n_big + (h.id & (MESH_HIT_BASE - 1))
                             : h.id <= -2          ? P.n_spheres + (-2 - h.id)
                                                   : h.id;
            o.id = remap[slot];
        }
        hits[i] = o;
    }
    if (DIAG) {
        if (dg.inner_it) atomicAdd(P.diag + 2, dg.inner_it);
        if (dg.inner_act) atomicAdd(P.diag + 3, dg.inner_act);
        if (dg.leaf_it) atomicAdd(P.diag + 4, dg.leaf_it);
        if (dg.leaf_act) atomicAdd(P.diag + 5, dg.leaf_act);
    }
}

// Sum the per-sample radiance of a chunked launch into the pixel sums, in sample order
// (camera.h:41-44), continuing `out` when accumulating.  One thread per pixel channel.
template <class R>
__global__ void reduce_kernel(const R* __restrict__ samples, R* __restrict__ out, size_t n, int nsamples,
                              int accumulate) {
#pragma clang fp contract(off)
    const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    R acc = accumulate ? out[e] : (R)0;
    for (int q = 0; q < nsamples; ++q) acc = acc + samples[(size_t)q * n + e];
    out[e] = acc;
}

// Gathered shard buffers -> row-major frame (see rt_hip.h rt_shard_info).
template <class T, int C>
__global__ void unshard_kernel(const T* __restrict__ gathered, T* __restrict__ frame, int W, int H, int tiles_x,
                               int nshards, int max_shard_tiles) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    if (x >= W || y >= H) return;
    const int t = (y >> 3) * tiles_x + (x >> 3);
    const int sh = t % nshards, lt = t / nshards;
    const size_t src = ((size_t)sh * max_shard_tiles * 64 + (size_t)lt * 64 + (y & 7) * 8 + (x & 7)) * C;
    const size_t dst = ((size_t)y * W + x) * C;
#pragma unroll
    for (int c = 0; c < C; ++c) frame[dst + c] = gathered[src + c];
}

// write_color for one channel sum (color.h:14-35): /spp, sqrt, clamp [0, 0.999], 256 x
// (the caller truncates to int; NaN -- a NaN sum, or sqrt of a negative one -- passes
// the clamp unchanged, as interval::clamp's comparisons are false for it).
__device__ __forceinline__ double write_color_channel(double sum, double scale) {
    double x = sqrt(sum * scale);
    if (x < 0.000)
        x = 0.000;
    else if (x > 0.999)
        x = 0.999;
    return 256 * x;
}

// write_color (color.h:14-35), in fp64 as the reference: one int32 per channel (a NaN sum
// prints static_cast<int>(NaN) = INT_MIN on x86, and stays INT_MIN here).
template <class T>
__global__ void quantize_kernel(const T* __restrict__ frame, int32_t* __restrict__ rgb, size_t n, int spp) {
    const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const double y = write_color_channel((double)frame[k], 1.0 / spp);
    rgb[k] = (y != y) ? (int32_t)0x80000000u : (int32_t)y;
}

// Gathered shard buffers -> row-major 8-bit frame in one pass (unshard + write_color):
// the host-bound frame is W*H*3 bytes instead of W*H*3 int32 (or the fp32 sums), and the
// row-major fp32 frame is never written.  A NaN sum (the reference prints
// static_cast<int>(NaN), INT_MIN on x86) becomes 0 here; rt_quantize keeps INT_MIN.
// `scale` = 1 / spp, as color.h:22.
template <class T>
__global__ void finish_u8_kernel(const T* __restrict__ gathered, uint8_t* __restrict__ rgb, int W, int H,
                                 int tiles_x, int nshards, int max_shard_tiles, double scale) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    if (x >= W || y >= H) return;
    const int t = (y >> 3) * tiles_x + (x >> 3);
    const int sh = t % nshards, lt = t / nshards;
    const size_t src = ((size_t)sh * max_shard_tiles * 64 + (size_t)lt * 64 + (y & 7) * 8 + (x & 7)) * 3;
    const size_t dst = ((size_t)y * W + x) * 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const double y = write_color_channel((double)gathered[src + c], scale);
        rgb[dst + c] = (y != y) ? (uint8_t)0 : (uint8_t)(int)y;
    }
}

// One path on an explicit tape of uniforms, reference recursion order (fp64 only).
template <class R>
__global__ void tape_kernel(RenderParams P, int max_depth, const double* ray7, const double* tape, int tape_len,
                            double* out, int* used) {
    __shared__ uint16_t stack[STACK_MAX];
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    SceneView<R> sc;
    sc.nodes = P.nodes;
    sc.sph = (const typename Prec<R>::Sph*)P.spheres;
    sc.mat = (const typename Prec<R>::Mat*)P.mats;
    sc.big = P.big;
    sc.bigf = P.bigf;
    sc.n_nodes = P.n_nodes;
    sc.n_big = P.n_big;
    sc.n_front = P.n_front;
    sc.mnodes = P.mnodes;
    sc.tris = (const typename Prec<R>::Tri*)P.tris;
    sc.tmeta = P.tmeta;
    sc.n_mnodes = P.n_mnodes;
    sc.mstack = nullptr;
    sc.n_mstack = 0;
    sc.box_extent = P.box_extent;
    for (int a = 0; a < 6; ++a) sc.mbox[a] = P.mbox[a];
    sc.grid = P.grid;
    // (the kernel arguments are RenderParams: the header's copy there, by address, without
    // taking P's address -- which would copy all of P to scratch)
    sc.gridp = (const __attribute__((address_space(4))) GridHdr*)((const __attribute__((address_space(4))) char*)
                                                                       __builtin_amdgcn_kernarg_segment_ptr() +
                                                                   offsetof(RenderParams, grid));
    TapeRng rng{tape, tape_len, 0};
    Ray<R> ray;
    ray.o = mk((R)ray7[0], (R)ray7[1], (R)ray7[2]);
    ray.d = mk((R)ray7[3], (R)ray7[4], (R)ray7[5]);
    ray.time = (R)ray7[6];
    V3<R> att_stack[64];
    int nsc = 0;
    V3<R> L = mk((R)0, (R)0, (R)0);
    if (max_depth > 0) {
        for (;;) {
            const Hit<R> h = closest_hit<R, true, false, 0, true>(sc, ray, stack, 1, NO_SELF);
            if (h.id == -1) {
                L = sky(ray.d);
                for (int k = nsc - 1; k >= 0; --k) L = att_stack[k] * L;
                break;
            }
            const Shade<R> sh = shade<R, true>(sc, ray, h);
            V3<R> att, dir;
            if (!scatter<R, true>(sc.mat[sh.meta & META_MAT_MASK], (sh.meta >> 24) & 3u, ray.d, sh, rng, att, dir))
                break;
            att_stack[nsc++] = att;
            ray.o = sh.p;
            ray.d = dir;
            if (nsc >= max_depth) break;
        }
    }
    out[0] = (double)L.x;
    out[1] = (double)L.y;
    out[2] = (double)L.z;
    *used = rng.pos;
}

}  // namespace rtx

// rt_device.h -- device-side building blocks of the path tracer, templated on the
// arithmetic type R (float = fast path, double = reference-exact path).
//
// Each function restates one piece of the reference CPU path (file:line cited) for one
// GPU lane.  In the double instantiation (compiled with -ffp-contract=off) the operation
// order is the reference's, so results are bit-identical to the g++ build; the float
// instantiation keeps the same control flow and random-number consumption, with fp32
// arithmetic (FMA allowed) and the large-sphere test kept in fp64.
#pragma once
#include <type_traits>
#include <hip/hip_runtime.h>

#include <cstdint>

#include "rt_scene.h"


namespace rtx {

// ---------------------------------------------------------------------------------
// RNG: RT-CRNG-1 (spec: oracle/rt_rng_spec.h, restated independently here).
// Replaces the global mt19937 stream of rtweekend.h:25-29 with one stream per
// (pixel, sample); uniforms are k * 2^-24, exact in fp32 and fp64.
// ---------------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x21f0aaadu;
    x ^= x >> 15;
    x *= 0xd35a2d97u;
    x ^= x >> 15;
    return x;
}
__host__ __device__ __forceinline__ uint32_t seed32_of(uint64_t seed) {
    return hash32((uint32_t)seed ^ hash32((uint32_t)(seed >> 32)));
}
constexpr uint32_t RNG_GOLDEN = 0x9e3779b9u;
constexpr uint32_t RNG_SAMPLE_SALT = 0x85ebca6bu;

struct CounterRng {
    uint32_t st;  // key + n * golden after n draws
    __device__ __forceinline__ void start(uint32_t pixel_key, uint32_t sample) {
        st = hash32(pixel_key ^ hash32(sample ^ RNG_SAMPLE_SALT));
    }
    template <class R>
    __device__ __forceinline__ R next() {
        st += RNG_GOLDEN;
        return (R)(hash32(st) >> 8) * (R)(1.0 / 16777216.0);
    }
    // c + s * next() as one FMA: u = k 2^-24 (k < 2^24), so s * u (s = 1, 2) and c + s * u
    // (c = -0.5, -1) are exact in fp32 and fp64, and the FMA's one rounding of the exact
    // value is that value -- the two-operation form's result bit for bit, one VALU fewer
    template <class R>
    __device__ __forceinline__ R next_affine(R s, R c) {
        st += RNG_GOLDEN;
        return fma((R)(hash32(st) >> 8), s * (R)(1.0 / 16777216.0), c);
    }
    __device__ __forceinline__ void skip(uint32_t n) { st += n * RNG_GOLDEN; }   // n draws, unused
};

// An explicit tape of uniforms (the caller's sequential stream): rt_trace_tape.
struct TapeRng {
    const double* tape;
    int len, pos;
    template <class R>
    __device__ __forceinline__ R next() {
        R u = pos < len ? (R)tape[pos] : (R)0.5;
        ++pos;
        return u;
    }
    __device__ __forceinline__ void skip(uint32_t n) { pos += (int)n; }
    template <class R>
    __device__ __forceinline__ R next_affine(R s, R c) {   // (tape values: the two-operation form)
        return c + s * next<R>();
    }
};

// ---------------------------------------------------------------------------------
// vec3 (vec3.h:8-158) -- same association order as the reference.
// ---------------------------------------------------------------------------------
// 1/x: v_rcp_f32 (1 ulp) on the fp32 path, IEEE division on the fp64 path.
__device__ __forceinline__ float rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ double rcp(double x) { return 1.0 / x; }
// 1/d for the slab tests.  fp32 computes a slab as one FMA, lo * (1/d) - o * (1/d); for a
// direction component of exactly 0 that is inf - inf = NaN, and a NaN slab made the box
// test fail (r03: 355 of 1,279 axis-aligned rays missed their sphere, rt_trace_rays).  A
// component of exactly +-0 becomes +-2^-100 (d + copysign(2^-100, d): every other
// component is unchanged, 2^-100 being at most half an ulp of any |d| >= 2^-76 that a
// scatter direction could have), so 1/d = +-2^100 is exact and the slab is
// (lo - o) * 2^100 -- (-huge, +huge) when o lies inside [lo, hi], entirely beyond any t_max
// otherwise (|lo|, |o| < 2^27 keep it finite).  The fp64 path keeps the reference's
// (lo - o) * (1/d) (aabb.h:35-53), which has no inf - inf.
__device__ __forceinline__ float slab_rcp(float x) { return rcp(x + copysignf(0x1p-100f, x)); }
__device__ __forceinline__ double slab_rcp(double x) { return rcp(x); }

template <class R>
struct V3 {
    R x, y, z;
};
template <class R> __device__ __forceinline__ V3<R> mk(R x, R y, R z) { return V3<R>{x, y, z}; }
template <class R> __device__ __forceinline__ V3<R> operator+(V3<R> a, V3<R> b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
template <class R> __device__ __forceinline__ V3<R> operator-(V3<R> a, V3<R> b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
template <class R> __device__ __forceinline__ V3<R> operator*(V3<R> a, V3<R> b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
template <class R> __device__ __forceinline__ V3<R> operator-(V3<R> a) { return {-a.x, -a.y, -a.z}; }
template <class R> __device__ __forceinline__ V3<R> scl(R t, V3<R> v) { return {t * v.x, t * v.y, t * v.z}; }       // vec3.h:93-99
template <class R> __device__ __forceinline__ V3<R> dvs(V3<R> v, R t) { return scl(rcp(t), v); }                   // vec3.h:101-103
// c + t v: one explicit FMA per component on the fp32 path (the fp32 unit fuses only within
// one expression, -ffp-contract=on, so fusions that span these helpers are spelled out);
// the fp64 path keeps the reference's separate rounding.
__device__ __forceinline__ V3<float> madd(float t, V3<float> v, V3<float> c) {
    return {__builtin_fmaf(t, v.x, c.x), __builtin_fmaf(t, v.y, c.y), __builtin_fmaf(t, v.z, c.z)};
}
__device__ __forceinline__ V3<double> madd(double t, V3<double> v, V3<double> c) { return c + scl(t, v); }
template <class R> __device__ __forceinline__ R dot(V3<R> a, V3<R> b) { return a.x * b.x + a.y * b.y + a.z * b.z; } // vec3.h:105-109
template <class R> __device__ __forceinline__ V3<R> cross(V3<R> u, V3<R> v) {                                  // vec3.h:111-115
    return {u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x};
}
template <class R> __device__ __forceinline__ R len2(V3<R> v) { return v.x * v.x + v.y * v.y + v.z * v.z; }         // vec3.h:46-48
template <class R> __device__ __forceinline__ V3<R> unit(V3<R> v) { return dvs(v, (R)sqrt(len2(v))); }            // vec3.h:117-119
template <class R> __device__ __forceinline__ V3<R> reflect(V3<R> v, V3<R> n) {                                   // vec3.h:149-151
    if constexpr (sizeof(R) == 4) return madd(-2.f * dot(v, n), n, v);
    return v - scl((R)2 * dot(v, n), n);
}
template <class R>
__device__ __forceinline__ V3<R> refract(V3<R> uv, V3<R> n, R e) {                                                  // vec3.h:153-157
    R cos_theta = fmin(dot(-uv, n), (R)1.0);
    V3<R> perp = scl(e, madd(cos_theta, n, uv));
    V3<R> par = scl(-(R)sqrt(fabs((R)1.0 - len2(perp))), n);
    return perp + par;
}
template <class R, class S> __device__ __forceinline__ V3<R> cvt(V3<S> v) { return {(R)v.x, (R)v.y, (R)v.z}; }
template <class R> __device__ __forceinline__ V3<R> ld3(const double* p) { return {(R)p[0], (R)p[1], (R)p[2]}; }
template <class R> __device__ __forceinline__ V3<R> ld3(const float* p) { return {(R)p[0], (R)p[1], (R)p[2]}; }

// ---------------------------------------------------------------------------------
// Kernel parameters (one struct, passed by value).
// ---------------------------------------------------------------------------------
constexpr int MAX_PHASES = 8;
struct RenderParams {
    int W, H, spp, max_depth;      // spp = samples rendered by THIS launch
    int sample_begin;              // global index of its first sample (RNG key, progressive)
    int accumulate;                // 1: continue the sums already in out_sums / out_segs
    int shard, nshards, tiles_x, shard_tiles;
    uint32_t seed32;
    int n_nodes, n_spheres, n_mats, n_big;
    int n_front;   // spheres [0, n_front) of `spheres` are tested before the BVH (not in it)
    int stack_size;
    int defocus;  // camera.h:94: defocus_angle > 0
    double cam_center[3], p00[3], du[3], dv[3], ddu[3], ddv[3];
    float f_center[3], f_p00[3], f_du[3], f_dv[3], f_ddu[3], f_ddv[3];  // the same, rounded once
    const Node* nodes;
    const void* spheres;   // SphereF or SphereD by precision
    const void* mats;      // MatF or MatD by precision
    const SphereD* big;
    const BigF* bigf;      // fp32 kernels: the same big spheres relative to their near point
    const Node4* mnodes;   // mesh BVH (4-wide, HBM-resident, 32-bit refs); n_mnodes == 0: no mesh
    const void* tris;      // TriF or TriD by precision, BVH leaf order
    const uint32_t* tmeta; // fp32: the triangles' meta words (TriF carries none)
    int n_mnodes;
    int mstack;            // mesh traversal stack entries per lane kept in LDS (rest: scratch)
    void* out_sums;        // shard_tiles*64*3 R
    uint32_t* out_segs;    // shard_tiles*64 (may be null)
    unsigned long long* diag;  // DIAG builds: DIAG_SLOTS counters (rt_render_diag)
    // fp64 persistent lanes: each sample's radiance goes to `samples`
    // ([s - sample_begin][pixel][3]); reduce_kernel then sums them per pixel in sample
    // order -- the reference's additions in the reference's order, bit-identical for any
    // split of the work.
    void* samples;
    // fp32 path (!EXACT): pixel sums in fixed point.  Each sample's radiance is rounded to
    // a multiple of 2^-FIX_SAMPLE_SHIFT and summed exactly, so sums do not depend on how a
    // pixel's samples are split over work items, launches (progressive ranges) or shards:
    // a lane sums one item's samples (<= FIX_ITEM_SAMPLES) in fp32 -- exact for radiance
    // in [0, 1], which every material with albedo <= 1 keeps -- then adds the sum to
    // accum[pixel][3] (64-bit integers in units of 2^-FIX_SHIFT) with one integer atomic
    // per channel; non-finite / overflowing sums set accum_flags[pixel] bits.
    // finalize_kernel turns accum into the fp32 out_sums.  No per-sample buffer.
    long long* accum;
    uint32_t* accum_flags;
    // this launch's sums in units of 2^-FIX_SAMPLE_SHIFT, packed: accp[2p] = R | G << 32,
    // accp[2p + 1] = B (each < 2^32 for <= FIX_LAUNCH_SAMPLES samples of radiance <= 1);
    // finalize_kernel adds them to accum.  Two atomics per flush instead of three.
    unsigned long long* accp;
    // fp32 persistent lanes: the work queue's control block (QUEUE_CTRL_BYTES, zeroed
    // before the launch: per-XCD heads, fetch_item); the grid is capped at max_wgs
    // workgroups (what the device keeps resident)
    uint32_t* queue;
    int max_wgs;
    // ...whose items come in nph phases: phase p covers samples [sample_begin + ph_s0[p],
    // + ph_k[p] * ph_c[p]) of every tile in ph_k[p] chunks of ph_c[p] samples (items
    // tile-major within a phase); chunk sizes shrink from phase to phase
    int nph;
    int ph_s0[MAX_PHASES], ph_c[MAX_PHASES], ph_k[MAX_PHASES];
    // coherent primaries (TRAV_COH): another shade round runs while at least this many
    // lanes of the wave hold no ray
    int coh_refill;
    // TRAV_F32BOX (fp64 kernels): a bound of |coordinate| over every sphere- and mesh-BVH
    // node box (cons_slabs)
    float box_extent;
    float mbox[6];         // the mesh's box (lo xyz, hi xyz): the union of the root's child boxes
    GridHdr grid;          // TRAV_GRID: the sphere grid's header (its cells are `nodes`)
    // RN(1 / tiles_x) and half of it: render_coherent's pop finds a tile's row as
    // floor((t + 0.5) / tiles_x) = (int)fma(t, inv, inv / 2) in fp64 -- exact for every
    // t < 2^51 (the quotient lies >= 0.5 / tiles_x from an integer, its error is <=
    // (t + 0.5) 2^-52 / tiles_x), and three VALU instead of a 32-bit integer division's ~20
    double tiles_x_inv, tiles_x_inv_half;
};
constexpr size_t QUEUE_CTRL_BYTES = 4096;   // RenderParams::queue: 8 heads x 128 B (+ room)
constexpr int FIX_SHIFT = 28;          // accum: 64-bit integers in units of 2^-28
constexpr int FIX_SAMPLE_SHIFT = 19;   // each sample's radiance rounded to a multiple of 2^-19
constexpr int FIX_ITEM_SAMPLES = 32;         // <= 32 such values in [0, 1] sum exactly in fp32
constexpr int FIX_LAUNCH_SAMPLES = 8191;     // a launch's packed sums stay below 2^32 per channel
// accum_flags bits, per channel c at bit 3c: NaN, +overflow (+inf), -overflow (-inf)
constexpr uint32_t FIX_NAN = 1u, FIX_POS = 2u, FIX_NEG = 4u;
constexpr int DIAG_SLOTS = 32;   // rt_render_diag_ex (RT_DIAG_SLOTS)

// Coherent primaries (TRAV_COH, render_coherent): per wave, a FIFO of primary hits that
// wait for a lane to shade them, then the current work item's pixel sums (64 x 3 floats).
constexpr int COH_FIFO = 128;
template <bool MESH>
struct CohEntryT {
    float t;        // hit distance
    uint32_t pix;   // pixel of the shard (local tile * 64 + pixel of the tile)
    uint32_t sid;   // sample - sample_begin (bits 0-15) | (hit id + 16) << 16 (spheres, bits 16-27)
                    // | the defocus rejections (fp32, bits 28-31)
};
template <>
struct CohEntryT<true> {   // scenes with a mesh: triangle ids need the full word
    float t;
    uint32_t pix;
    uint32_t sid;   // sample - sample_begin | the defocus rejections << 28 (fp32)
    int32_t id;
};
using CohEntry = CohEntryT<false>;
static_assert(sizeof(CohEntryT<false>) == 12 && sizeof(CohEntryT<true>) == 16, "CohEntry");
// fp64 coherent kernel (f64_kernel 4): the exact fp64 hit distance
template <bool MESH>
struct CohEntryD {
    double t;
    uint32_t pix;
    uint32_t sid;   // as CohEntryT
};
template <>
struct CohEntryD<true> {
    double t;
    uint32_t pix;
    uint32_t sid;
    int32_t id;
    uint32_t pad;
};
static_assert(sizeof(CohEntryD<false>) == 16 && sizeof(CohEntryD<true>) == 24, "CohEntryD");
template <class R, bool MESH> struct CohEntrySel { using type = CohEntryT<MESH>; };
template <bool MESH> struct CohEntrySel<double, MESH> { using type = CohEntryD<MESH>; };
template <class R, bool MESH> using CohEntryX = typename CohEntrySel<R, MESH>::type;
constexpr size_t COH_SUM_BYTES = 64 * 3 * sizeof(float);   // the wave's item pixel sums
// each lane's path throughput and scatter count, parked in LDS across the trace by the fp32
// mixed-scene kernels (coh_parks)
constexpr size_t COH_PARK_BYTES = 64 * 4 * sizeof(float);
// LDS per wave of the coherent kernel: the FIFO, then (unless TRAV_NOSUM, or fp64) the item
// sums, then (coh_parks) the parked path state
constexpr size_t coh_wave_bytes(bool mesh, bool sums, int fifo = COH_FIFO, bool f64 = false, bool park = false) {
    return (size_t)fifo * (f64 ? (mesh ? sizeof(CohEntryD<true>) : sizeof(CohEntryD<false>))
                               : (mesh ? sizeof(CohEntryT<true>) : sizeof(CohEntryT<false>))) +
           (sums && !f64 ? COH_SUM_BYTES : 0) + (park ? COH_PARK_BYTES : 0);
}
constexpr size_t COH_WAVE_BYTES = coh_wave_bytes(false, true);
// per workgroup: the kernel's rarely read constants (camera vectors, work-queue phases),
// read from LDS so that the persistent kernel does not hold them in scalar registers
struct CohConst {
    float cam[18];   // f_center, f_p00, f_du, f_dv, f_ddu, f_ddv (camera_ray_lds)
    int nph;
    int ph_s0[MAX_PHASES], ph_c[MAX_PHASES], ph_k[MAX_PHASES];
    int pad;
};
static_assert(sizeof(CohConst) % 16 == 0, "CohConst");
constexpr size_t COH_CAM_BYTES = sizeof(CohConst);


template <class R> struct Prec;
template <> struct Prec<float> { using Sph = SphereF; using Mat = MatF; using Tri = TriF; };
template <> struct Prec<double> { using Sph = SphereD; using Mat = MatD; using Tri = TriD; };

// Scene view: pointers into LDS (spheres) and HBM (mesh).
template <class R>
struct SceneView {
    const Node* nodes;
    const typename Prec<R>::Sph* sph;
    const typename Prec<R>::Mat* mat;
    const SphereD* big;
    const BigF* bigf;
    int n_nodes, n_big, n_front;
    const Node4* mnodes;   // HBM
    const typename Prec<R>::Tri* tris;
    const uint32_t* tmeta; // fp32: triangle meta words (RenderParams::tmeta)
    int n_mnodes;
    uint32_t* mstack;      // this lane's LDS stack column (entry k at mstack[k * stride])
    int n_mstack;
    float mbox[6];         // RenderParams::mbox
    GridHdr grid;          // RenderParams::grid (uniform: scalar registers)
    // RenderParams::grid in the kernel-argument segment (constant address space: scalar
    // loads), for the sphere-only grid walks
    const __attribute__((address_space(4))) GridHdr* gridp;
    float box_extent;      // TRAV_F32BOX: bound of |coordinate| over every node box (RenderParams)
};

template <class R>
struct Ray {
    V3<R> o, d;
    R time;
};

// ---------------------------------------------------------------------------------
// sphere::hit (sphere.h:30-57), root selection only: the nearest root in the strict
// interval (tmin, tmax) (interval.h:33-35).  The hit record is rebuilt once for the
// closest sphere (shade_sphere), which yields the same values as the reference's
// per-candidate record (they are pure functions of ray, sphere and root).
// ---------------------------------------------------------------------------------
template <class T, bool EXACT, bool SELECT = false>
__device__ __forceinline__ bool sphere_root(V3<T> c, T r, V3<T> cv, bool moving, V3<T> o, V3<T> d, T a, T inv_a,
                                            T time, T tmin, T tmax, bool self, T& t) {
    V3<T> center = c;
    if (EXACT) {
        if (moving) center = c + scl(time, cv);                 // sphere.h:31, 68-72
    } else {
        center = madd(time, cv, c);                             // cv == 0 when stationary
    }
    if (EXACT) {
        // sphere.h:32-48 verbatim (half-b quadratic): fp64 rounds as the reference.
        V3<T> oc = o - center;
        T half_b = dot(oc, d);
        T cc = len2(oc) - r * r;
        T disc = half_b * half_b - a * cc;
        if (disc < 0) return false;
        T sq = (T)sqrt(disc);
        T root = (-half_b - sq) / a;
        if (!(tmin < root && root < tmax)) {
            root = (-half_b + sq) / a;
            if (!(tmin < root && root < tmax)) return false;
        }
        t = root;
        return true;
    }
    // fp32: the same roots, computed without the two cancellations that make the
    // half-b form unusable in single precision (SURVEY.md §7 "fp32 precision"):
    //  * discriminant from the closest-approach vector l = f + (b/a) d:
    //    (half_b^2 - a c)/a = r^2 - |l|^2  (Ray Tracing Gems ch. 7), so a small sphere
    //    seen from afar keeps ~1e-6 accuracy instead of ~1e-4;
    //  * the root pair as c/q and q/a with q = b + sign(b) sqrt(a disc) (no b - sqrt(..)).
    //  * self: the ray starts on this sphere (its previous hit), so one root is the
    //    origin itself (t = 0, always < tmin in the reference's fp64); only the other,
    //    t = -2 (f.d)/a, can be a hit.  Without this, fp32 rounding of the hit point
    //    turns short scattered directions (|d| << 1, material.h:21 has no near_zero
    //    guard) into false self-hits above tmin = 0.001.
    const V3<T> f = o - center;
    const T b = -dot(f, d);
    T root;
    if (self) {
        root = (T)2 * b * inv_a;
        if (!(tmin < root && root < tmax)) return false;
        t = root;
        return true;
    }
    const V3<T> l = madd(b * inv_a, d, f);
    const T r2 = r * r;
    const T disc = r2 - len2(l);
    if (disc < 0) return false;
    const T cc = len2(f) - r2;
    const T q = b + copysign((T)sqrt(a * disc), b);
    const T ta = cc * rcp(q), tb = q * inv_a;
    const T t0 = fmin(ta, tb), t1 = fmax(ta, tb);
    if (SELECT) {
        root = (tmin < t0 && t0 < tmax) ? t0 : t1;   // nearest root inside (tmin, tmax)
        t = root;
        return tmin < root && root < tmax;
    }
    root = t0;
    if (!(tmin < root && root < tmax)) {
        root = t1;
        if (!(tmin < root && root < tmax)) return false;
    }
    t = root;
    return true;
}

// Triangle (mesh path): Moller-Trumbore, two-sided, no epsilon beyond
// the shared (tmin, tmax) interval.  Operation order is the oracle's (rt_oracle.c
// tri_hit), so the fp64 instantiation is bit-identical to it.  e1 = v1 - v0 and
// e2 = v2 - v0 are precomputed on the host in fp64.
// (The fp32 path used this test with the barycentric bounds widened by 2^-20 until r04;
// it now runs the watertight tri_wt below.)
template <class T>
__device__ __forceinline__ bool tri_root(V3<T> v0, V3<T> e1, V3<T> e2, V3<T> o, V3<T> d, T tmin, T tmax, T& t) {
    constexpr T EPS = (T)0;
    const V3<T> pv = cross(d, e2);
    const T det = dot(e1, pv);
    if (det == (T)0) return false;
    const T inv_det = rcp(det);
    const V3<T> tv = o - v0;
    const T u = dot(tv, pv) * inv_det;
    if (u < -EPS || u > (T)1 + EPS) return false;
    const V3<T> qv = cross(tv, e1);
    const T v = dot(d, qv) * inv_det;
    if (v < -EPS || u + v > (T)1 + EPS) return false;
    const T tt = dot(e2, qv) * inv_det;
    if (!(tmin < tt && tt < tmax)) return false;
    t = tt;
    return true;
}

// fp32 triangle test, watertight (r05).  Moller-Trumbore in fp32
// computes each triangle's barycentrics on its own, so a ray through the edge two
// triangles share can fall outside both (|o - v0| ~ 100 edge lengths makes u wrong by
// ~3e-6 > the 2^-20 widening: 39 of 33.5M rays from inside the C4 blob leaked,
// tools/leak_probe.py).  Here each edge has ONE value, computed identically by both
// triangles that share it: with the vertices relative to the ray origin (A = v0 - o, ...,
// the same fp32 numbers in every triangle: TriF keeps the shared vertices), the edge
// function of edge (P, Q) is d . (P x Q), evaluated without fused multiply-adds, so that
// Q x P is bit for bit -(P x Q) (rounded products commute; a - b = -(b - a)) and the other
// triangle sees exactly the negated value.  A ray is inside when the three edge values
// do not have opposite signs (zero -- exactly on an edge -- counts for both sides), so
// the triangles around any edge or vertex of a closed mesh leave no gap.  Two-sided like
// the oracle's test.
// The edge values lose accuracy as (|A| / edge length)^2 (a far camera assigns a ray near
// a facet boundary to the neighbouring facet -- consistently, so still without a gap),
// but t must not: it is the distance to the facet's plane, n . A / n . d with n = (v1 -
// v0) x (v2 - v0) from the nearby vertices, as accurate as Moller-Trumbore's (measured on
// the C5 blob from the C5 camera: median 5e-8, 99th percentile 6e-7 relative, against
// 6e-4 / 0.09 for the triple product A . (B x C) / (sum of the edge values)).
// (fence: keep a value in a register at this point -- orders the edge computations so that
// the three relative vertices are not all live alongside every intermediate)
__device__ __forceinline__ void vfence(float& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ bool tri_wt(V3<float> p0, V3<float> p1, V3<float> p2, V3<float> n, V3<float> o,
                                       V3<float> d, float tmin, float tmax, float& t) {
    // the facet's plane (n = (v1 - v0) x (v2 - v0) from the record): t = n . (v0 - o) / n . d
    const float nd = dot(n, d);
    float Ax, Ay, Az;
    {
#pragma clang fp contract(off)
        Ax = p0.x - o.x, Ay = p0.y - o.y, Az = p0.z - o.z;
    }
    const float tt = dot(n, mk(Ax, Ay, Az)) * rcp(nd);
    if (!(tmin < tt && tt < tmax)) return false;   // (nd == 0: never in range)
    // inside: every edge value has the sign of their sum, d . n = nd (or is 0); each is
    // checked as soon as it is known (most misses leave after one or two edges)
    auto outside = [nd](float e) { return nd > 0.f ? e < 0.f : e > 0.f; };
    {
#pragma clang fp contract(off)
        const float Bx = p1.x - o.x, By = p1.y - o.y, Bz = p1.z - o.z;
        float ec = d.x * (Ay * Bz - Az * By) + d.y * (Az * Bx - Ax * Bz) + d.z * (Ax * By - Ay * Bx);   // (v0, v1)
        vfence(ec);
        if (outside(ec)) return false;
        const float Cx = p2.x - o.x, Cy = p2.y - o.y, Cz = p2.z - o.z;
        float ea = d.x * (By * Cz - Bz * Cy) + d.y * (Bz * Cx - Bx * Cz) + d.z * (Bx * Cy - By * Cx);   // (v1, v2)
        vfence(ea);
        if (outside(ea)) return false;
        const float eb = d.x * (Cy * Az - Cz * Ay) + d.y * (Cz * Ax - Cx * Az) + d.z * (Cx * Ay - Cy * Ax);   // (v2, v0)
        if (outside(eb)) return false;
    }
    t = tt;
    return true;
}
// one triangle record: fp32 the watertight test on its vertices, fp64 Moller-Trumbore in
// the oracle's order (bit-exact)
__device__ __forceinline__ bool tri_hit(const TriF& q, V3<float> o, V3<float> d, float tmin, float tmax, float& t) {
    return tri_wt(mk(q.v0[0], q.v0[1], q.v0[2]), mk(q.v1[0], q.v1[1], q.v1[2]), mk(q.v2[0], q.v2[1], q.v2[2]),
                  mk(q.n[0], q.n[1], q.n[2]), o, d, tmin, tmax, t);
}
__device__ __forceinline__ bool tri_hit(const TriD& q, V3<double> o, V3<double> d, double tmin, double tmax,
                                        double& t) {
    return tri_root<double>(mk(q.v0[0], q.v0[1], q.v0[2]), mk(q.e1[0], q.e1[1], q.e1[2]),
                            mk(q.e2[0], q.e2[1], q.e2[2]), o, d, tmin, tmax, t);
}

// Diagnostic counters (DIAG builds only, rt_render_diag): wave-level loop iterations and
// the active lanes summed over them, counted by the first active lane of each iteration.
struct DiagCounters {
    unsigned long long inner_it = 0, inner_act = 0, leaf_it = 0, leaf_act = 0;
    unsigned long long mnode_it = 0, mnode_act = 0, mtri_it = 0, mtri_act = 0;   // mesh BVH
    uint32_t steps = 0;   // this lane's node visits + sphere tests in the current closest_hit
    __device__ __forceinline__ static void count(unsigned long long& it, unsigned long long& act) {
        const unsigned long long e = __builtin_amdgcn_read_exec();
        if ((int)(threadIdx.x & 63) == __builtin_ctzll(e)) {
            ++it;
            act += (unsigned long long)__builtin_popcountll(e);
        }
    }
};

template <class R>
struct Hit {
    R t;         // closest root (R)
    double td;   // closest root in fp64 when a big sphere won (fp64 path only)
    int id;      // >= 0 BVH sphere (LDS index), <= -2 big sphere (-2 - k), -1 none,
                 // MESH_HIT_BASE | k triangle k (BVH leaf order)
};

__device__ __forceinline__ bool box_hit(const float lo[3], const float hi[3], V3<float> inv, V3<float> oi, float tmin,
                                        float tmax, float& tnear) {
    float t0x = fmaf(lo[0], inv.x, -oi.x), t1x = fmaf(hi[0], inv.x, -oi.x);
    float t0y = fmaf(lo[1], inv.y, -oi.y), t1y = fmaf(hi[1], inv.y, -oi.y);
    float t0z = fmaf(lo[2], inv.z, -oi.z), t1z = fmaf(hi[2], inv.z, -oi.z);
    float tn = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fmaxf(fminf(t0z, t1z), tmin));
    // tn <= min(tf, tmax) as two compares: tmax (a loop-carried value) then needs no
    // re-canonicalising v_max per node for fminf (same result: fminf ignores a NaN slab)
    float tf = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
    tnear = tn;
    return tn <= tf && tn <= tmax;
}
__device__ __forceinline__ bool box_hit(const float lo[3], const float hi[3], V3<double> inv, V3<double> o,
                                        double tmin, double tmax, double& tnear) {
    double t0x = ((double)lo[0] - o.x) * inv.x, t1x = ((double)hi[0] - o.x) * inv.x;
    double t0y = ((double)lo[1] - o.y) * inv.y, t1y = ((double)hi[1] - o.y) * inv.y;
    double t0z = ((double)lo[2] - o.z) * inv.z, t1z = ((double)hi[2] - o.z) * inv.z;
    double tn = fmax(fmax(fmin(t0x, t1x), fmin(t0y, t1y)), fmax(fmin(t0z, t1z), tmin));
    double tf = fmin(fmin(fmax(t0x, t1x), fmax(t0y, t1y)), fmin(fmax(t0z, t1z), tmax));
    tnear = tn;
    return tn <= tf;
}

// Conservative fp32 slabs for the fp64 path (TRAV_F32BOX).  Per ray and axis (cons_slabs):
// f = fl32(1/d), and the slab of plane x is fma(x, f, c) with c = fl32(-fl32(o) f) moved by
// m = 2^-21 (|o| + E) |f| (E: the scene's coordinate bound, RenderParams::box_extent)
// towards the outside of the slab -- down for the entry plane, up for the exit plane.
// The rounding of fl32(o), of f, of the product and of the FMA together stay below
// 2^-24 (5 |o| + 2 E) |1/d| (1 + 2^-23) < m, so each computed slab contains the exact one
// and the box test can only pass boxes the exact test would reject, never the reverse.  An
// axis with |d| < 2^-60 is not tested at all (slab (-inf, inf)).
struct ConsSlabs {
    float f[3], clo[3], chi[3];
};
__device__ __forceinline__ ConsSlabs cons_slabs(V3<double> o, V3<double> d, float extent) {
    ConsSlabs s;
    const double oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        if (fabs(dd[a]) < 0x1p-60) {
            s.f[a] = 0.f;
            s.clo[a] = -__builtin_huge_valf();
            s.chi[a] = __builtin_huge_valf();
            continue;
        }
        const float f = (float)(1.0 / dd[a]);
        const float m = (float)((fabs(oo[a]) + (double)extent) * 0x1p-21 * fabs((double)f));
        const float c = -((float)oo[a] * f);
        s.f[a] = f;
        s.clo[a] = f > 0.f ? c - m : c + m;   // the lo plane is the entry plane when f > 0
        s.chi[a] = f > 0.f ? c + m : c - m;
    }
    return s;
}
__device__ __forceinline__ bool box_hit_cons(const float lo[3], const float hi[3], const ConsSlabs& s, float tmin,
                                             float tmax, float& tnear) {
    const float t0x = __builtin_fmaf(lo[0], s.f[0], s.clo[0]), t1x = __builtin_fmaf(hi[0], s.f[0], s.chi[0]);
    const float t0y = __builtin_fmaf(lo[1], s.f[1], s.clo[1]), t1y = __builtin_fmaf(hi[1], s.f[1], s.chi[1]);
    const float t0z = __builtin_fmaf(lo[2], s.f[2], s.clo[2]), t1z = __builtin_fmaf(hi[2], s.f[2], s.chi[2]);
    const float tn = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fmaxf(fminf(t0z, t1z), tmin));
    const float tf = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
    tnear = tn;
    return tn <= tf && tn <= tmax;
}
// fp32 bounds of the fp64 interval (0.001, tmax): below 0.001, and tmax rounded up
constexpr float CONS_TMIN = 0.0009f;
__device__ __forceinline__ float cons_tmax(double tmax) { return (float)tmax * (1.f + 0x1p-22f); }

// hittable_list::hit (hittable_list.h:25-39) over {big spheres} + BVH (bvh.h:16-24):
// closest root in (0.001, inf).  The BVH visits the nearer child first and pushes the
// other onto this lane's LDS stack (stack[k * stride]).
// TRAV bit flags (all give identical pixels; they only trade instructions for divergence):
//   8 select-based root choice
//   16 whole-record LDS reads: nodes and spheres as ds_read_b128 only (the compiler
//      otherwise narrows reads whose last word is unused to ds_read_b96, which costs the
//      LDS twice the cycles of a b128 read, MI355X_MICROARCH.md §LDS)
//   64 coherent primaries (fp32, render_coherent): camera rays are traced in batches of
//      one sample of all 64 pixels of a tile, secondaries in the bounce loop
//   128 (with 64) no LDS pixel sums: every sample goes straight to the fixed-point sums
//      (chosen by the C ABI when the sums would not fit the LDS of two workgroups per CU)
//   512 pop culling: the register stack top keeps its entry distance, and a popped top
//      whose box starts beyond the closest hit found since it was pushed is dropped
//      without a visit (its children's boxes start no nearer: child lo/hi lie inside the
//      parent's and the slab FMAs round monotonically, so the visit would hit neither)
//   32 (fp64 kernels) conservative fp32 slab tests: the fp64 path's box tests run in fp32
//      on the unmodified fp32 node boxes, each slab widened by a per-ray bound of the
//      rounding (box_hit_cons) so that no box the exact ray enters is rejected; boxes only
//      prune the search (the spheres are still tested in the reference's fp64), so the
//      closest hit -- and every pixel -- is the fp64 slab test's
// (1 speculative while-while, 2 paired leaf tests, 4 branch-light node step, the ray pool,
// 1024 a drain pool and 2048 a 64-entry FIFO were measured slower and removed in r03,
// DESIGN.md §5; 256 time-binned sphere trees (+0.7 % only without the LDS item sums) and
// 4096 an LDS copy of the mesh tree top (-2.8 % on C4) were removed in r04 and are refused
// by rt_set_tuning.)
//   2048 (fp64 kernels) persistent lanes over the work queue (render_lanes<EXACT>), each
//      sample's radiance stored for the ordered reduction
//   8192 (fp32 coherent mesh kernels; added by the C ABI unless 16384 is asked for) the
//      if-if mesh loop: a lane visits one node or tests one leaf per iteration, node and
//      triangle loads leaving through the same instructions (C4 52.0 -> 45.0 ms)
//   16384 (tuning only, never in a kernel key) keep the while-while mesh loop
//   (32768, quantised 64-B mesh nodes -- 8-bit child planes on a per-node grid -- measured
//   C4 +12 % / C5 +7 % in r05 and removed; the number stays refused)
//   65536 (fp32 sphere kernels) the uniform sphere grid (rt_scene.h GridHdr) instead of the
//      sphere BVH: the ray's cells in order, each cell's listed spheres tested, until the
//      closest hit lies before the cell's exit (no traversal stack)
//   131072 (with 65536; added by the C ABI where the grid is one cell tall in y, unless 262144
//      is asked for) the walk steps in x and z only (r06: C3 -6 %, the same frame)
//   (262144, tuning only, never in a kernel key: keep the 3-D walk on such a grid)
enum { TRAV_SELROOT = 8, TRAV_B128 = 16, TRAV_F32BOX = 32, TRAV_COH = 64, TRAV_NOSUM = 128, TRAV_TBIN = 256,
       TRAV_CULL = 512, TRAV_PERSIST = 2048, TRAV_MTOP = 4096, TRAV_MIFIF = 8192, TRAV_MWHILE = 16384,
       TRAV_MQ = 32768, TRAV_GRID = 65536, TRAV_GFLAT = 131072,
       TRAV_G3D = 262144 };
constexpr int TRAV_REMOVED = TRAV_TBIN | TRAV_MTOP;   // refused (r04)
// FIFO entries per wave (r03: a 64-entry FIFO, where a batch waits until the FIFO is
// empty, freed 12 KB of LDS per workgroup but ran 3.5 % slower on C3)
constexpr int coh_fifo_entries(int) { return COH_FIFO; }
// r06: the fp32 mixed-scene kernels (meshes over the sphere grid) park each lane's path
// throughput and scatter count in LDS (COH_PARK_BYTES) instead of holding them across the
// trace, where the 6-wave register budget spilled them to scratch around every bounce: the
// C5 geometry at 4K @ 1024 1,525.4-1,526.3 -> 1,506.0-1,507.1 ms, frames identical
// (profiles/r06/r06p).  Mesh-only C4 keeps them in registers: parked it ran 42.9-44.9 ms
// against 39.8-40.0 at every block and LDS stack depth tried (r06q).
constexpr bool coh_parks(bool mesh, int tr, bool f64) { return mesh && !f64 && (tr & TRAV_GRID) != 0; }
// LDS views by 32-bit LDS byte address (the sphere grid's flat walk and record reads)
typedef __attribute__((address_space(3))) const uint32_t lds_cu32;
typedef __attribute__((address_space(3))) const float4 lds_cf4;
// Keep a loaded word live without an instruction (forces the full-width LDS read).
__device__ __forceinline__ void keep_live(uint32_t v) { asm volatile("" ::"v"(v)); }
template <class R, bool EXACT, bool DIAG = false, int TRAV = 0, bool MESH = false>
__device__ __forceinline__ Hit<R> closest_hit(const SceneView<R>& sc, const Ray<R>& ray, uint16_t* stack, int stride,
                                              int self_id, DiagCounters* dg = nullptr) {
    constexpr R TMIN = (R)0.001;
    Hit<R> h;
    h.id = -1;
    h.td = __builtin_huge_val();
    R tmax = (R)__builtin_huge_valf();
    const V3<R> o = ray.o, d = ray.d;
    const R a = len2(d);
    const R inv_a = rcp(a);

    // big spheres (rt_scene.h BIG_RADIUS)
    if (EXACT) {
        // reference arithmetic, fp64 (sphere.h:30-57)
        const V3<double> od = cvt<double>(o), dd = cvt<double>(d);
        double tmaxd = __builtin_huge_val();
        for (int k = 0; k < sc.n_big; ++k) {
            const SphereD& s = sc.big[k];
            double t;
            if (sphere_root<double, true>(mk(s.c[0], s.c[1], s.c[2]), s.r, mk(s.cv[0], s.cv[1], s.cv[2]),
                                          (s.meta >> 30) & 1u, od, dd, (double)a, 0.0, (double)ray.time, 0.001,
                                          tmaxd, false, t)) {
                tmaxd = t;
                h.id = -2 - k;
                h.td = t;
            }
        }
        if (h.id != -1) tmax = (R)h.td;
    } else {
        // fp32 path: relative to the sphere's near point p0 (BigF), f = o - c = q + r n:
        // b = -f.d = -(q.d + r n.d), c = |f|^2 - r^2 = q.q + 2 r n.q, without the
        // cancellation of |f| ~ r ~ 1000; the roots then follow from the stable pair c/q,
        // q/a (see sphere_root).
        for (int k = 0; k < sc.n_big; ++k) {
            const BigF& s = sc.bigf[k];
            V3<R> p0 = mk((R)s.p0[0], (R)s.p0[1], (R)s.p0[2]);
            if ((s.meta >> 30) & 1u) p0 = madd((R)ray.time, mk((R)s.cv[0], (R)s.cv[1], (R)s.cv[2]), p0);
            const V3<R> q = o - p0, nn = mk((R)s.n[0], (R)s.n[1], (R)s.n[2]);
            const R b = -fma((R)s.r, dot(nn, d), dot(q, d));
            R t;
            if ((-2 - k) == self_id) {
                t = (R)2 * b * inv_a;
                if (!(TMIN < t && t < tmax)) continue;
            } else {
                const R cc = fma((R)2 * (R)s.r, dot(nn, q), dot(q, q));
                const R disc = b * b - a * cc;
                if (disc < 0) continue;
                const R qq = b + copysign((R)sqrt(disc), b);
                const R ta = cc * rcp(qq), tb = qq * inv_a;
                const R t0 = fmin(ta, tb), t1 = fmax(ta, tb);
                t = t0;
                if (!(TMIN < t && t < tmax)) {
                    t = t1;
                    if (!(TMIN < t && t < tmax)) continue;
                }
            }
            tmax = t;
            h.id = -2 - k;
        }
    }

    // one sphere of the LDS array (the tree's leaves and the front list share it)
    using Sph = typename Prec<R>::Sph;
    auto test_rec = [&](const Sph* rec, bool is_self, R tlim, R& tk) -> bool {
        if constexpr (!EXACT && (TRAV & TRAV_B128) != 0) {
            const float4* q = (const float4*)rec;
            const float4 s0 = q[0], s1 = q[1];   // c, r | cv, meta
            keep_live(__float_as_uint(s0.w));
            keep_live(__float_as_uint(s1.w));
            return sphere_root<R, false, (TRAV & TRAV_SELROOT) != 0>(
                mk((R)s0.x, (R)s0.y, (R)s0.z), (R)s0.w, mk((R)s1.x, (R)s1.y, (R)s1.z), false, o, d, a, inv_a,
                ray.time, TMIN, tlim, is_self, tk);
        }
        const auto& s = *rec;
        return sphere_root<R, EXACT, (TRAV & TRAV_SELROOT) != 0>(mk((R)s.c[0], (R)s.c[1], (R)s.c[2]), (R)s.r,
                                     mk((R)s.cv[0], (R)s.cv[1], (R)s.cv[2]), (s.meta >> 30) & 1u, o, d, a, inv_a,
                                     ray.time, TMIN, tlim, !EXACT && is_self, tk);
    };
    auto test_one = [&](int k, R tlim, R& tk) -> bool { return test_rec(sc.sph + k, k == self_id, tlim, tk); };
    // front list (rt_tuning.front_spheres): the largest spheres, tested by every lane
    // before the tree; the closest hit is the same in any test order
    for (int k = 0; k < sc.n_front; ++k) {
        R t;
        if (test_one(k, tmax, t)) {
            tmax = t;
            h.id = k;
        }
    }

    if constexpr ((TRAV & TRAV_GRID) != 0) {
        // Uniform grid (GridHdr; in LDS where the tree's nodes go): the cells the ray crosses
        // in order, each cell's listed spheres tested (one sphere or one cell step per lane
        // and iteration), until the closest hit so far lies before the current cell's exit
        // (a sphere hit further on is listed in the cell it is reached in: rt_bvh.cpp pads
        // the listed boxes beyond the rounding of these plane distances).
        // The fp64 kernel (EXACT, f64_kernel 5) walks the same cells with the ray rounded to
        // fp32 and tests the listed spheres in fp64: the cells only choose which spheres are
        // tested, and the padding of the listed boxes covers that rounding too.
        if (sc.n_nodes > 0) {
            // TRAV_GFLAT (r06): the grid is one cell tall in y (GridHdr::res[1] == 1, a field of
            // spheres on a ground plane, main.cpp:18-44): the walk steps in x and z only.  Its
            // one layer spans the grid box's height, which clips the ray (tn, tf), so a step in
            // y could only come within the rounding of the exit (the 3-D walk's last step):
            // the same cells, the same frame (C3 -6 %, profiles/r06/r06w)
            constexpr bool FLAT = (TRAV & TRAV_GFLAT) != 0;
            // Sphere-only kernels re-read the header from the kernel arguments per walk (scalar
            // loads through a pointer the compiler cannot see through), instead of holding its
            // 20 words in SGPRs across the whole kernel, where the allocator spilled them to
            // VGPR lanes and read them back with a VALU v_readlane each (24 -> 5 in a walk's set-up;
            // SGPR spills 88 -> 72): C3 -1.0 %.  The mixed-scene kernels keep the copy (+1.2 %
            // with the pointer; profiles/r06/r06ab).
            const GridHdr g = [&]() {
                if constexpr (!MESH) {
                    auto gp = sc.gridp;
                    asm volatile("" : "+s"(gp));
                    return *(const GridHdr*)gp;
                } else {
                    return sc.grid;
                }
            }();
            const uint32_t pad = (uint32_t)g.res[0] * (uint32_t)g.res[1];   // empty layers (rt_bvh.cpp)
            // cell words and list entries are both indexed from `cells` (rt_scene.h GridHdr:
            // the lists follow the cells and the trailing pad layer), so one base register
            // serves the walk and the tests; the entries hold each sphere record's byte offset
            // from the grid's LDS base (the records follow the grid there)
            const uint32_t* cells = (const uint32_t*)sc.nodes + pad;
            const unsigned char* lbase = (const unsigned char*)sc.nodes;
            const uint32_t sph0 = (uint32_t)sc.n_nodes * (uint32_t)sizeof(Node);
            // (only a sphere of the array can be the ray's origin here: big spheres have negative
            // ids, triangles MESH_HIT_BASE | k, whose scaled offset would alias sphere k's)
            const uint32_t self_off = self_id >= 0 && self_id < MESH_HIT_BASE
                                          ? sph0 + (uint32_t)self_id * (uint32_t)sizeof(Sph)
                                          : 0xffffffffu;
            uint32_t hit_off = 0xffffffffu;
            const float INF = __builtin_huge_valf();
            const V3<float> of = cvt<float>(o), df = cvt<float>(d);
            float tn, tf, nx, ny = INF, nz, dtx, dty = 0.f, dtz;
            int ci;
            {
                const V3<float> inv = mk(slab_rcp(df.x), slab_rcp(df.y), slab_rcp(df.z));
                const V3<float> oi = of * inv;
                // clipped to the box of the spheres at the ray's time slab (rt_scene.h GridHdr;
                // a time outside [0, 1], or NaN: the grid box, the last one)
                const float tm = (float)ray.time;
                const int sk = tm >= 0.f && tm <= 1.f ? min((int)(tm * g.slab_k), g.n_slab - 1) : g.n_slab;
                // ((lo, hi) pairs per axis: lanes of different slabs read different banks)
                const float2* sbx = (const float2*)(lbase + g.slab_off) + sk;
                const int sst = g.n_slab + 1;
                const float2 bx = sbx[0], by = sbx[sst], bz = sbx[2 * sst];
                const float t0x = fmaf(bx.x, inv.x, -oi.x), t1x = fmaf(bx.y, inv.x, -oi.x);
                const float t0y = fmaf(by.x, inv.y, -oi.y), t1y = fmaf(by.y, inv.y, -oi.y);
                const float t0z = fmaf(bz.x, inv.z, -oi.z), t1z = fmaf(bz.y, inv.z, -oi.z);
                tn = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fmaxf(fminf(t0z, t1z), (float)TMIN));
                tf = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fminf(fmaxf(t0z, t1z), (float)tmax));
                // the entry cell, and per axis the distance to its exit plane and the step
                // between planes (never along a zero direction component)
                auto axis = [&](int a, float oa, float da, float iv, float oia, float& n, float& dt) {
                    int i = (int)((fmaf(tn, da, oa) - g.lo[a]) * g.inv_cs[a]);
                    i = i < 0 ? 0 : (i >= g.res[a] ? g.res[a] - 1 : i);
                    const float plane = fmaf((float)(da > 0.f ? i + 1 : i), g.cs[a], g.lo[a]);
                    n = da != 0.f ? fmaf(plane, iv, -oia) : INF;
                    dt = g.cs[a] * fabsf(iv);
                    return i;
                };
                const int ix = axis(0, of.x, df.x, inv.x, oi.x, nx, dtx);
                const int iz = axis(2, of.z, df.z, inv.z, oi.z, nz, dtz);
                if constexpr (FLAT) {
                    ci = iz * g.res[0] + ix;
                } else {
                    const int iy = axis(1, of.y, df.y, inv.y, oi.y, ny, dty);
                    ci = (iz * g.res[1] + iy) * g.res[0] + ix;
                }
            }
            // Termination (r06): every ray origin a launch can produce lies within +-GridHdr::
            // far_o (rt_abi.cpp grid_reach_ok decides per launch, from the camera and the
            // scene's bounds; otherwise the launch runs the tree).  There each step moves its
            // axis's plane distance by at least 15/16 of a cell (2^-24 (|o| + ext) stays below
            // cs / 16), so a walk takes at most res[0] + res[1] + res[2] + 2 steps before its
            // exit distance passes tf, and the fp32 rounding of the plane distances stays within
            // the listed boxes' padding.  No check in the loop: a cell-range test per step, or any
            // far-origin path in this function, measured +1.4 .. +9 % on C3 (r06c / r06d).
            if (tn <= tf) {
                const int sy = g.res[0], sz = g.res[1] * sy;
                const int stx = df.x > 0.f ? 1 : -1, sty = df.y > 0.f ? sy : -sy, stz = df.z > 0.f ? sz : -sz;
                // a cell word: its list's first and end entries (GRID_POS_BITS each)
                // (flat walk: the cell as its LDS byte address, stepped by 4 x the index steps --
                // no scaling per step)
                [[maybe_unused]] uint32_t ca = (uint32_t)(uintptr_t)(cells + ci);
                [[maybe_unused]] const int sx4 = stx * 4, sz4 = stz * 4;
                uint32_t w = FLAT ? *(const lds_cu32*)(uintptr_t)ca : cells[ci];
                uint32_t cur = w & GRID_POS_MASK, end = w >> GRID_POS_BITS;
                // one iteration: a lane whose cell is done steps to the next cell (stopping
                // once the closest hit so far lies before the cell's exit, or the ray leaves
                // the grid or passes the front / big spheres' hit), then tests one sphere of
                // its cell -- a single loop, so that lanes stepping through empty cells and
                // lanes testing spheres share every iteration
                for (;;) {
                    if (cur >= end) {
                        if (DIAG) DiagCounters::count(dg->inner_it, dg->inner_act), ++dg->steps;
                        // (a step out of the grid happens only within the rounding of its exit,
                        // the ray's last step: past the first or last layer it reads an empty
                        // pad cell, past a row's or slab's end the neighbouring row's cell --
                        // tests the exact sphere test settles, never a different hit -- and the
                        // next exit ends the loop)
                        if constexpr (FLAT) {
                            // (a compare and a select: fminf's NaN rules cost two more VALU)
                            const bool bx = nx <= nz;
                            const float te = bx ? nx : nz;
                            if (!(te < (float)tmax && te < tf)) break;
                            ca += bx ? sx4 : sz4;
                            nx = bx ? nx + dtx : nx;
                            nz = bx ? nz : nz + dtz;
                        } else {
                            const float te = fminf(fminf(nx, ny), nz);
                            if (!(te < (float)tmax && te < tf)) break;
                            const bool bx = nx == te, by = !bx && ny == te, bz = !bx && !by;
                            ci += bx ? stx : (by ? sty : stz);
                            nx = bx ? nx + dtx : nx;
                            ny = by ? ny + dty : ny;
                            nz = bz ? nz + dtz : nz;
                        }
                        w = FLAT ? *(const lds_cu32*)(uintptr_t)ca : cells[ci];
                        cur = w & GRID_POS_MASK;
                        end = w >> GRID_POS_BITS;
                    }
                    if (cur < end) {
                        if (DIAG) DiagCounters::count(dg->leaf_it, dg->leaf_act), ++dg->steps;
                        const uint32_t off = *(const lds_cu32*)(uintptr_t)cur;   // (cur: an LDS byte address)
                        cur += 4u;
                        R t;
                        // the record straight from its LDS byte address: the grid buffer is the
                        // first thing in the kernel's dynamic LDS, which starts at address 0 (the
                        // render kernels have no static LDS: rt_abi.cpp checks it per launch),
                        // saving the add of a base the compiler only learns to be 0 after ISel
                        const Sph* rec = (const Sph*)(const float4*)(const lds_cf4*)(uintptr_t)off;
                        if (test_rec(rec, off == self_off, tmax, t)) {
                            tmax = t;
                            hit_off = off;
                        }
                    }
                }
            }
            if (hit_off != 0xffffffffu) h.id = (int)((hit_off - sph0) / (uint32_t)sizeof(Sph));
        }
    } else if (sc.n_nodes > 0) {
        const Node* nodes = sc.nodes;
        constexpr bool CONS = EXACT && (TRAV & TRAV_F32BOX) != 0;
        using BT = std::conditional_t<CONS, float, R>;   // box-test distances
        const V3<R> inv = mk(slab_rcp(d.x), slab_rcp(d.y), slab_rcp(d.z));
        const V3<R> oi = EXACT ? o : o * inv;   // fp32: t = lo*inv - o*inv as one FMA
        ConsSlabs cs;
        if constexpr (CONS) cs = cons_slabs(cvt<double>(o), cvt<double>(d), sc.box_extent);
        // Stack: the most recently pushed ref stays in a register (`top`); older ones go
        // to this lane's LDS column.  Most pops follow a push, so most pops cost no LDS
        // round trip.
        uint32_t ref = 0, top = REF_NONE;
        BT top_tn = (BT)0;   // TRAV_CULL: entry distance of `top`'s box
        int sp = 0;
        auto pop = [&]() -> uint32_t {
            if (top != REF_NONE) {
                const uint32_t r = top;
                top = REF_NONE;
                if (!(TRAV & TRAV_CULL) || top_tn <= tmax) return r;
            }
            if (sp > 0) {
                --sp;
                return stack[sp * stride];
            }
            return REF_NONE;
        };
        // One node: test both children, continue with the nearer hit child, remember the
        // other (register top, older entries to LDS), or pop.
        auto visit = [&](uint32_t node) -> uint32_t {
            const uint4* q = (const uint4*)(nodes + node);
            const uint4 w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3];   // one 64-B node
            const float lo0[3] = {__uint_as_float(w0.x), __uint_as_float(w0.y), __uint_as_float(w0.z)};
            const float hi0[3] = {__uint_as_float(w1.x), __uint_as_float(w1.y), __uint_as_float(w1.z)};
            const float lo1[3] = {__uint_as_float(w2.x), __uint_as_float(w2.y), __uint_as_float(w2.z)};
            const float hi1[3] = {__uint_as_float(w3.x), __uint_as_float(w3.y), __uint_as_float(w3.z)};
            const uint32_t r0 = w0.w, r1 = w1.w;
            if (TRAV & TRAV_B128) {
                keep_live(w2.w);
                keep_live(w3.w);
            }
            BT tn0, tn1;
            bool h0, h1;
            if constexpr (CONS) {
                const float tmf = cons_tmax((double)tmax);
                h0 = box_hit_cons(lo0, hi0, cs, CONS_TMIN, tmf, tn0);
                h1 = box_hit_cons(lo1, hi1, cs, CONS_TMIN, tmf, tn1);
            } else {
                h0 = box_hit(lo0, hi0, inv, oi, TMIN, tmax, tn0);
                h1 = box_hit(lo1, hi1, inv, oi, TMIN, tmax, tn1);   // (no empty children: rt_bvh.cpp)
            }
            if (h0 && h1) {
                const bool first0 = tn0 <= tn1;
                if (top != REF_NONE) {
                    stack[sp * stride] = (uint16_t)top;
                    ++sp;
                }
                top = first0 ? r1 : r0;
                if (TRAV & TRAV_CULL) top_tn = first0 ? tn1 : tn0;
                return first0 ? r0 : r1;
            }
            if (h0 || h1) return h0 ? r0 : r1;
            return pop();
        };
        auto leaf_test = [&](uint32_t lref) {
            const int first = (int)(lref & 0x7ffu);
            const int last = first + (int)((lref >> 11) & 0xfu);
            for (int k = first; k <= last; ++k) {
                if (DIAG) DiagCounters::count(dg->leaf_it, dg->leaf_act), ++dg->steps;
                R t;
                if (test_one(k, tmax, t)) {
                    tmax = t;
                    h.id = k;
                }
            }
        };
        // while-while: descend until this lane reaches a leaf, test it, pop, repeat
        for (;;) {
            while (!(ref & REF_LEAF)) {
                if (DIAG) DiagCounters::count(dg->inner_it, dg->inner_act), ++dg->steps;
                ref = visit(ref);
            }
            if (ref == REF_NONE) break;
            leaf_test(ref);
            ref = pop();
            if (ref == REF_NONE) break;
        }
    }
    if (MESH && sc.n_mnodes > 0) {
        // Mesh BVH (4-wide): nodes and triangles stay in HBM (a mesh does not fit 160 KiB
        // of LDS; the working set of a frame lives in L2/MALL); an LDS copy of the tree's
        // top measured slower (r03am: the top is L1/L2-resident anyway) and was removed (r04).
        // Per node: the 4 child boxes, hit children ordered near to far (sorting network),
        // the nearest continued, the others pushed far-first.  Stack: the latest push in a
        // register (`top`), the next n_mstack entries in an LDS column, deeper ones in a
        // per-lane scratch array (scratch traffic shares the vector-memory counter with
        // the node loads, so an LDS stack keeps pushes off the node-load critical path).
        const V3<R> inv = mk(slab_rcp(d.x), slab_rcp(d.y), slab_rcp(d.z));
        const V3<R> oi = EXACT ? o : o * inv;
        ConsSlabs mcs;
        if constexpr (EXACT && (TRAV & TRAV_F32BOX) != 0) mcs = cons_slabs(cvt<double>(o), cvt<double>(d), sc.box_extent);
        uint32_t mstk[MESH_STACK_MAX];
        int sp = 0;
        uint32_t ref = 0, top = MREF_EMPTY;
        R mtop_tn = (R)0;   // TRAV_CULL: entry distance of `top`'s box
        // The LDS column through an LDS-typed pointer: written as `cond ? lds[i] : mstk[j]`
        // the compiler turned the pop into ONE flat load of a selected pointer, and a flat
        // load waits on both the vector-memory and the LDS counter (r03w)
        typedef __attribute__((address_space(3))) uint32_t lds_u32;
        lds_u32* const mlds = (lds_u32*)sc.mstack;
        auto mpop = [&]() -> uint32_t {
            if (top != MREF_EMPTY) {
                const uint32_t r = top;
                top = MREF_EMPTY;
                if (!(TRAV & TRAV_CULL) || mtop_tn <= tmax) return r;
            }
            if (sp <= 0) return MREF_EMPTY;
            --sp;
            if (sp < sc.n_mstack) return mlds[sp * stride];
            return mstk[sp - sc.n_mstack];
        };
        auto mpush = [&](uint32_t r, R tn) {
            if (top != MREF_EMPTY) {
                if (sp < sc.n_mstack)
                    mlds[sp * stride] = top;
                else
                    mstk[sp - sc.n_mstack] = top;
                ++sp;
            }
            top = r;
            if (TRAV & TRAV_CULL) mtop_tn = tn;
        };
        const R INF = (R)__builtin_huge_valf();
        typedef float nf4 __attribute__((ext_vector_type(4)));
        typedef uint32_t nu4 __attribute__((ext_vector_type(4)));
        typedef __attribute__((address_space(1))) const nu4 glb_u4;
        // One 4-wide node from its 7 loaded words: the child boxes, hit children ordered
        // near to far, the nearest returned, the others pushed (or a pop).
        auto mnode = [&](const nf4 v0, const nf4 v1, const nf4 v2, const nf4 v3, const nf4 v4, const nf4 v5,
                         const nu4 v6) -> uint32_t {
            const float4 lx = make_float4(v0.x, v0.y, v0.z, v0.w), ly = make_float4(v1.x, v1.y, v1.z, v1.w);
            const float4 lz = make_float4(v2.x, v2.y, v2.z, v2.w), hx = make_float4(v3.x, v3.y, v3.z, v3.w);
            const float4 hy = make_float4(v4.x, v4.y, v4.z, v4.w), hz = make_float4(v5.x, v5.y, v5.z, v5.w);
            const uint4 rr = make_uint4(v6.x, v6.y, v6.z, v6.w);
            R t[4];
            uint32_t r[4] = {rr.x, rr.y, rr.z, rr.w};
            if constexpr (!EXACT) {
                // the slab planes one child at a time (scalar FMAs: the same fused results as
                // the packed all-children form, v_pk_fma_f32, at the same issue cost -- but a
                // child's six plane distances die before the next child's are made: 94 -> 88
                // VGPRs, 80 with 6 spilled under the 6-wave budget; tools/vgpr_probes.py)
                const float LX[4] = {lx.x, lx.y, lx.z, lx.w}, LY[4] = {ly.x, ly.y, ly.z, ly.w};
                const float LZ[4] = {lz.x, lz.y, lz.z, lz.w}, HX[4] = {hx.x, hx.y, hx.z, hx.w};
                const float HY[4] = {hy.x, hy.y, hy.z, hy.w}, HZ[4] = {hz.x, hz.y, hz.z, hz.w};
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const float t0x = __builtin_fmaf(LX[c], inv.x, -oi.x), t1x = __builtin_fmaf(HX[c], inv.x, -oi.x);
                    const float t0y = __builtin_fmaf(LY[c], inv.y, -oi.y), t1y = __builtin_fmaf(HY[c], inv.y, -oi.y);
                    const float t0z = __builtin_fmaf(LZ[c], inv.z, -oi.z), t1z = __builtin_fmaf(HZ[c], inv.z, -oi.z);
                    const float tn = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fmaxf(fminf(t0z, t1z), (float)TMIN));
                    const float tf = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fminf(fmaxf(t0z, t1z), (float)tmax));
                    t[c] = tn <= tf && r[c] != MREF_EMPTY ? (R)tn : INF;
                }
            } else {
                const float lo[4][3] = {{lx.x, ly.x, lz.x}, {lx.y, ly.y, lz.y}, {lx.z, ly.z, lz.z}, {lx.w, ly.w, lz.w}};
                const float hi[4][3] = {{hx.x, hy.x, hz.x}, {hx.y, hy.y, hz.y}, {hx.z, hy.z, hz.z}, {hx.w, hy.w, hz.w}};
                [[maybe_unused]] const float tmf = cons_tmax((double)tmax);
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    bool hc;
                    R tn;
                    if constexpr ((TRAV & TRAV_F32BOX) != 0) {
                        float tf32;
                        hc = box_hit_cons(lo[c], hi[c], mcs, CONS_TMIN, tmf, tf32);
                        tn = (R)tf32;
                    } else {
                        hc = box_hit(lo[c], hi[c], inv, oi, TMIN, tmax, tn);
                    }
                    t[c] = hc && r[c] != MREF_EMPTY ? tn : INF;
                }
            }
            auto cswap = [&](int i, int j) {
                const bool sw = t[j] < t[i];
                const R ti = t[i];
                const uint32_t ri = r[i];
                t[i] = sw ? t[j] : ti;
                r[i] = sw ? r[j] : ri;
                t[j] = sw ? ti : t[j];
                r[j] = sw ? ri : r[j];
            };
            cswap(0, 1);
            cswap(2, 3);
            cswap(0, 2);
            cswap(1, 3);
            cswap(1, 2);
            if (t[3] < INF) mpush(r[3], t[3]);
            if (t[2] < INF) mpush(r[2], t[2]);
            if (t[1] < INF) mpush(r[1], t[1]);
            return t[0] < INF ? r[0] : mpop();
        };
        if constexpr (!EXACT && (TRAV & TRAV_MIFIF) != 0) {
            // one fp32 triangle k of the leaf order from its 9 vertex words (not the
            // triangle the ray starts on: a flat primitive cannot be re-hit at t > 0)
            auto mtri = [&](const V3<float> p0, const V3<float> p1, const V3<float> p2, const V3<float> nn, int k) {
                float t;
                if ((MESH_HIT_BASE | k) != self_id && tri_wt(p0, p1, p2, nn, o, d, TMIN, tmax, t)) {
                    tmax = t;
                    h.id = MESH_HIT_BASE | k;
                }
            };
            // if-if (TRAV_MIFIF): every iteration a lane either visits one node or tests
            // one leaf, and both kinds of load leave through the same instructions (a
            // node's 112 B, or a leaf's first two 48-B triangles), so the wave waits for
            // one memory round trip per iteration where while-while waits once per node
            // level and once more per leaf round.  Each lane's own sequence of visits,
            // tests and pops is while-while's, so the closest hit is the same bit for bit.
            const TriF* tris = (const TriF*)sc.tris;
            typedef __attribute__((address_space(1))) const nu4 glb_u4a;
            {
                // a ray that misses the mesh's box (the union of the root's child boxes, so
                // a ray entering any child enters it) or enters it beyond the closest hit
                // so far skips the mesh without a load (C4 +0.8 %, C5 +1.5 %, r03bf)
                const float blo[3] = {sc.mbox[0], sc.mbox[1], sc.mbox[2]};
                const float bhi[3] = {sc.mbox[3], sc.mbox[4], sc.mbox[5]};
                R tb;
                if (!box_hit(blo, bhi, inv, oi, TMIN, tmax, tb)) ref = MREF_EMPTY;
            }
            for (;;) {
                if (ref == MREF_EMPTY) break;
                const bool leaf = (ref & MREF_LEAF) != 0;
                const int first = (int)(ref & 0xffffffu);
                const int last = first + (int)((ref >> 24) & 0x7fu);
                // node: its 7 words of 16 B; leaf: its first two 48-B records (6 words), the
                // 7th load repeating the leaf's first address
                const glb_u4a* q = leaf ? (const glb_u4a*)(tris + first) : (const glb_u4a*)(sc.mnodes + ref);
                const glb_u4a* q6 = leaf ? q : q + 6;
                const nu4 w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3], w4 = q[4], w5 = q[5], w6 = q6[0];
                if (!leaf) {
                    if (DIAG) DiagCounters::count(dg->mnode_it, dg->mnode_act);
                    ref = mnode(__builtin_bit_cast(nf4, w0), __builtin_bit_cast(nf4, w1), __builtin_bit_cast(nf4, w2),
                                __builtin_bit_cast(nf4, w3), __builtin_bit_cast(nf4, w4), __builtin_bit_cast(nf4, w5), w6);
                    continue;
                }
                // words: tri A v0.xyz v1.x | v1.yz v2.xy | v2.z n.xyz, tri B in w3..w5 likewise
                auto fw = [](uint32_t u) { return __uint_as_float(u); };
                if (DIAG) DiagCounters::count(dg->mtri_it, dg->mtri_act);
                mtri(mk(fw(w0.x), fw(w0.y), fw(w0.z)), mk(fw(w0.w), fw(w1.x), fw(w1.y)), mk(fw(w1.z), fw(w1.w), fw(w2.x)),
                     mk(fw(w2.y), fw(w2.z), fw(w2.w)), first);
                if (last > first) {
                    if (DIAG) DiagCounters::count(dg->mtri_it, dg->mtri_act);
                    mtri(mk(fw(w3.x), fw(w3.y), fw(w3.z)), mk(fw(w3.w), fw(w4.x), fw(w4.y)),
                         mk(fw(w4.z), fw(w4.w), fw(w5.x)), mk(fw(w5.y), fw(w5.z), fw(w5.w)), first + 1);
                    // leaves beyond two triangles (mesh_max_leaf > 2): the rest one by one
                    for (int k = first + 2; k <= last; ++k) {
                        if (DIAG) DiagCounters::count(dg->mtri_it, dg->mtri_act);
                        const TriF& r = tris[k];
                        mtri(mk(r.v0[0], r.v0[1], r.v0[2]), mk(r.v1[0], r.v1[1], r.v1[2]), mk(r.v2[0], r.v2[1], r.v2[2]),
                             mk(r.n[0], r.n[1], r.n[2]), k);
                    }
                }
                ref = mpop();
            }
        } else {
            for (;;) {
                while (!(ref & MREF_LEAF)) {
                    if (DIAG) DiagCounters::count(dg->mnode_it, dg->mnode_act);
                    const glb_u4* q = (const glb_u4*)(sc.mnodes + ref);
                    const nu4 w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3], w4 = q[4], w5 = q[5], w6 = q[6];
                    ref = mnode(__builtin_bit_cast(nf4, w0), __builtin_bit_cast(nf4, w1), __builtin_bit_cast(nf4, w2),
                                __builtin_bit_cast(nf4, w3), __builtin_bit_cast(nf4, w4), __builtin_bit_cast(nf4, w5), w6);
                }
                if (ref == MREF_EMPTY) break;
                const int first = (int)(ref & 0xffffffu);
                const int last = first + (int)((ref >> 24) & 0x7fu);
                // software-pipelined: the next triangle's load is issued before this one's
                // test, so a leaf costs about one memory round trip instead of one per triangle
                typename Prec<R>::Tri tr = sc.tris[first];
                for (int k = first; k <= last; ++k) {
                    if (DIAG) DiagCounters::count(dg->mtri_it, dg->mtri_act);
                    const typename Prec<R>::Tri nx = sc.tris[k < last ? k + 1 : last];
                    R t;
                    if ((EXACT || (MESH_HIT_BASE | k) != self_id) &&   // flat: no re-hit of the origin triangle
                        tri_hit(tr, o, d, TMIN, tmax, t)) {
                        tmax = t;
                        h.id = MESH_HIT_BASE | k;
                    }
                    tr = nx;
                }
                ref = mpop();
                if (ref == MREF_EMPTY) break;
            }
        }
    }
    // every hit lowers tmax to its own t (fp64 big spheres: (R)td), so the winner's t is
    // tmax: h.t is not carried through the traversal (one VGPR, and fp32 keeps no td)
    h.t = tmax;
    return h;
}

// Hit record of the winner: p = r.at(t) (ray.h:19-21), outward normal (p - c)/r
// (sphere.h:51-53), face orientation (hittable.h:15-21).
template <class R>
struct Shade {
    V3<R> p, normal;
    bool front_face;
    uint32_t meta;
};

template <class T>
__device__ __forceinline__ void shade_sphere(V3<T> c, T r, V3<T> cv, bool moving, V3<T> o, V3<T> d, T time, T t,
                                             V3<T>& p, V3<T>& normal, bool& front) {
    V3<T> center = moving ? madd(time, cv, c) : c;
    p = madd(t, d, o);
    V3<T> outward = dvs(p - center, r);
    front = dot(d, outward) < 0;
    normal = front ? outward : -outward;
}

template <class R, bool MESH = false>
__device__ __forceinline__ Shade<R> shade(const SceneView<R>& sc, const Ray<R>& ray, const Hit<R>& h) {
    Shade<R> s;
    if (MESH && h.id >= MESH_HIT_BASE) {
        // triangle record: p = r.at(t), outward normal unit(e1 x e2), face orientation
        // (hittable.h:15-21); the oracle's tri_hit order (fp32: e1, e2 from the fp32
        // vertices, the meta word from the side array)
        const int k = h.id & (MESH_HIT_BASE - 1);
        const auto& q = sc.tris[k];
        s.p = madd(h.t, ray.d, ray.o);
        V3<R> outward;
        if constexpr (sizeof(R) == 4) {
            outward = unit(mk(q.n[0], q.n[1], q.n[2]));   // (e1 x e2 in fp64, rounded: TriF::n)
            s.meta = sc.tmeta[k];
        } else {
            outward = unit(cross(mk((R)q.e1[0], (R)q.e1[1], (R)q.e1[2]), mk((R)q.e2[0], (R)q.e2[1], (R)q.e2[2])));
            s.meta = q.meta;
        }
        s.front_face = dot(ray.d, outward) < 0;
        s.normal = s.front_face ? outward : -outward;
        return s;
    }
    if (h.id >= 0) {
        const auto& q = sc.sph[h.id];
        shade_sphere<R>(mk((R)q.c[0], (R)q.c[1], (R)q.c[2]), (R)q.r, mk((R)q.cv[0], (R)q.cv[1], (R)q.cv[2]),
                        (q.meta >> 30) & 1u, ray.o, ray.d, ray.time, h.t, s.p, s.normal, s.front_face);
        s.meta = q.meta;
    } else {
        const SphereD& q = sc.big[-2 - h.id];
        if (sizeof(R) == 8) {
            // fp64 path: the reference's record (sphere.h:50-54)
            V3<double> p, n;
            bool front;
            shade_sphere<double>(mk(q.c[0], q.c[1], q.c[2]), q.r, mk(q.cv[0], q.cv[1], q.cv[2]), (q.meta >> 30) & 1u,
                                 cvt<double>(ray.o), cvt<double>(ray.d), (double)ray.time, h.td, p, n, front);
            s.p = cvt<R>(p);
            s.normal = cvt<R>(n);
            s.front_face = front;
        } else {
            // fp32 path: p = o + t d; (p - c) / r = (p - p0) / r + n (BigF: no cancellation)
            const BigF& g = sc.bigf[-2 - h.id];
            s.p = madd(h.t, ray.d, ray.o);
            V3<R> p0 = mk((R)g.p0[0], (R)g.p0[1], (R)g.p0[2]);
            if ((g.meta >> 30) & 1u) p0 = madd((R)ray.time, mk((R)g.cv[0], (R)g.cv[1], (R)g.cv[2]), p0);
            const V3<R> outward = madd((R)g.inv_r, s.p - p0, mk((R)g.n[0], (R)g.n[1], (R)g.n[2]));
            s.front_face = dot(ray.d, outward) < 0;
            s.normal = s.front_face ? outward : -outward;
        }
        s.meta = q.meta;
    }
    return s;
}

// random_in_unit_sphere (vec3.h:129-135) with vec3::random(-1,1) (vec3.h:67-69): the
// reference's g++ build evaluates the three constructor arguments right to left, so z
// takes the first draw.
template <class R, class Rng>
__device__ __forceinline__ V3<R> random_in_unit_sphere(Rng& rng) {
    for (;;) {
        R z = rng.template next_affine<R>((R)2, (R)-1);
        R y = rng.template next_affine<R>((R)2, (R)-1);
        R x = rng.template next_affine<R>((R)2, (R)-1);
        V3<R> p = mk(x, y, z);
        if (len2(p) < (R)1) return p;
    }
}

// material::scatter (material.h:15-82).  Returns false when absorbed.
template <class R, bool EXACT, class Rng>
__device__ __forceinline__ bool scatter(const typename Prec<R>::Mat& m, uint32_t type, const V3<R>& din,
                                        const Shade<R>& s, Rng& rng, V3<R>& att, V3<R>& dir) {
    if (type != MAT_DIELECTRIC) {
        // lambertian (material.h:19-25) and metal (:35-41) both draw ONE
        // random_in_unit_sphere; drawing it on a shared path keeps the wave's rejection
        // loop converged across the two material types (same draws per lane).
        const V3<R> p = random_in_unit_sphere<R>(rng);
        att = mk((R)m.p[0], (R)m.p[1], (R)m.p[2]);
        if (type == MAT_LAMBERTIAN) {
            dir = s.normal + unit(p);                                  // no near_zero guard (vec3.h:50-54 unused)
            return true;
        }
        dir = madd((R)m.p[3], p, reflect(unit(din), s.normal));
        return dot(dir, s.normal) > 0;
    }
    // dielectric, material.h:52-71
    att = mk((R)1.0, (R)1.0, (R)1.0);
    const R ir = (R)m.p[3];
    const R ratio = s.front_face ? rcp(ir) : ir;
    const V3<R> ud = unit(din);
    const R cos_theta = fmin(dot(-ud, s.normal), (R)1.0);
    const R sin_theta = (R)sqrt((R)1.0 - cos_theta * cos_theta);
    const bool cannot_refract = ratio * sin_theta > (R)1.0;
    bool refl = cannot_refract;
    if (!refl) {                                                       // short-circuit ||: no draw on TIR
        R r0 = ((R)1 - ratio) / ((R)1 + ratio);                         // material.h:76-80
        r0 = r0 * r0;
        const R x = (R)1 - cos_theta;
        R x5;
        if (EXACT) {
            x5 = (R)pow((double)x, 5.0);
        } else {
            const R x2 = x * x;
            x5 = x2 * x2 * x;
        }
        refl = r0 + ((R)1 - r0) * x5 > rng.template next<R>();
    }
    dir = refl ? reflect(ud, s.normal) : refract(ud, s.normal, ratio);
    return true;
}

// Background (camera_cpu.h:23-25).
template <class R>
__device__ __forceinline__ V3<R> sky(const V3<R>& d) {
    const V3<R> ud = unit(d);
    const R a = (R)0.5 * (ud.y + (R)1.0);
    return madd(a, mk((R)0.5, (R)0.7, (R)1.0), scl((R)1.0 - a, mk((R)1.0, (R)1.0, (R)1.0)));
}

// camera::get_ray for the fp32 path with the camera vectors read from an LDS copy
// (cam: center, pixel00, du, dv, ddu, ddv as 18 floats = RenderParams::f_*): the
// persistent coherent kernel would otherwise keep them in scalar registers throughout.
// Same operations as camera_ray<float>.
// kdef (render_coherent's FIFO entries): in, >= 0: the defocus disk's rejected candidates, known (the ray is
// regenerated: the loop is skipped, its draws jumped over); -1: draw as usual and, if kout,
// store how many candidates were rejected there
template <class Rng>
__device__ __forceinline__ Ray<float> camera_ray_lds(const float* cam, int defocus, int i, int j, Rng& rng,
                                                     int kdef = -1, int* kout = nullptr) {
    auto v = [&](int k) { return mk(cam[3 * k], cam[3 * k + 1], cam[3 * k + 2]); };
    const V3<float> du = v(2), dv = v(3);
    const V3<float> pixel_center = madd((float)j, dv, madd((float)i, du, v(1)));
    const float px = rng.template next_affine<float>(1.f, -0.5f);
    const float py = rng.template next_affine<float>(1.f, -0.5f);
    const V3<float> pixel_sample = pixel_center + madd(px, du, scl(py, dv));
    V3<float> origin = v(0);
    if (defocus) {
        float x, y;
        if (kdef >= 0) {   // (counter RNG only: the rejected candidates' two draws each, skipped)
            rng.skip(2u * (uint32_t)kdef);
            y = rng.template next_affine<float>(2.f, -1.f);
            x = rng.template next_affine<float>(2.f, -1.f);
        } else {
            int k = 0;
            for (;;) {                                                 // vec3.h:121-127, y drawn first
                y = rng.template next_affine<float>(2.f, -1.f);
                x = rng.template next_affine<float>(2.f, -1.f);
                if (x * x + y * y + 0.f * 0.f < 1.f) break;
                ++k;
            }
            if (kout) *kout = k;
        }
        origin = madd(y, v(5), madd(x, v(4), origin));
    }
    Ray<float> r;
    r.o = origin;
    r.d = pixel_sample - origin;
    r.time = rng.template next<float>();
    return r;
}

// camera::get_ray (camera.h:87-113).
template <class R, class Rng>
__device__ __forceinline__ Ray<R> camera_ray(const RenderParams& P, int i, int j, Rng& rng, int kdef = -1,
                                             int* kout = nullptr) {
    const bool f = sizeof(R) == 4;  // fp32 path reads the pre-rounded copies
    const V3<R> du = f ? ld3<R>(P.f_du) : ld3<R>(P.du), dv = f ? ld3<R>(P.f_dv) : ld3<R>(P.dv);
    const V3<R> pixel_center = madd((R)j, dv, madd((R)i, du, f ? ld3<R>(P.f_p00) : ld3<R>(P.p00)));
    const R px = rng.template next_affine<R>((R)1, (R)-0.5);
    const R py = rng.template next_affine<R>((R)1, (R)-0.5);
    const V3<R> pixel_sample = pixel_center + madd(px, du, scl(py, dv));   // + is commutative: fp64 as camera.h:92
    V3<R> origin = f ? ld3<R>(P.f_center) : ld3<R>(P.cam_center);
    if (P.defocus) {
        R x, y;
        if (kdef >= 0) {   // (as camera_ray_lds)
            rng.skip(2u * (uint32_t)kdef);
            y = rng.template next_affine<R>((R)2, (R)-1);
            x = rng.template next_affine<R>((R)2, (R)-1);
        } else {
            int k = 0;
            for (;;) {                                                 // vec3.h:121-127, y drawn first
                y = rng.template next_affine<R>((R)2, (R)-1);
                x = rng.template next_affine<R>((R)2, (R)-1);
                if (x * x + y * y + (R)0 * (R)0 < (R)1) break;
                ++k;
            }
            if (kout) *kout = k;
        }
        origin = madd(y, f ? ld3<R>(P.f_ddv) : ld3<R>(P.ddv), madd(x, f ? ld3<R>(P.f_ddu) : ld3<R>(P.ddu), origin));
    }
    Ray<R> r;
    r.o = origin;
    r.d = pixel_sample - origin;
    r.time = rng.template next<R>();
    return r;
}

}  // namespace rtx

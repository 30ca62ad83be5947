// rt_lbvh.hip -- GPU BVH build for meshes ("a GPU BVH build
// (LBVH/Morton) for large meshes"), selected by rt_tuning.mesh_builder (RT_MESH_BUILD_GPU:
// with treelet restructuring, r06; RT_MESH_BUILD_GPU_LBVH: the plain Morton tree).
//
//   1. tri_keys    : 30-bit Morton code of each triangle centroid (bounds from the host's
//                    validation pass), value = triangle index
//   2. rocprim radix sort of (code, index)
//   3. leaf_boxes  : each sorted triangle's padded fp32 box, SAH cost and count
//   4. karras      : binary radix tree over the sorted codes (Karras 2012; equal codes
//                    are ordered by index), child refs, parent links
//   5. node_depth  : depth of every internal node (parent walk); then one level_box
//                    launch per depth, deepest first, unions the children's boxes, costs
//                    and counts (kernel boundaries order the levels: no cross-workgroup
//                    hand-off inside a launch, which per-XCD L2s would make fragile)
//   6. treelets    : (RT_MESH_BUILD_GPU) rounds of treelet restructuring (rt_treelet.h,
//                    Karras & Aila 2013): per round the depths again, then one launch per
//                    depth, deepest first, re-optimising the topology of the 7-leaf treelet
//                    under every node of that depth by SAH (disjoint within a launch)
//   7. leaf_offsets: the leaves' positions in depth-first order (one launch per depth, top
//                    down), so that every subtree's triangles are contiguous, and each node's
//                    range of them
//   8. tri_pack    : triangles to their positions -> TriF (+ meta) / TriD records, and the
//                    input index of each position (rt_trace_rays' remap)
//   9. classify    : internal nodes with <= max_leaf triangles become leaves; the
//                    4-wide tree keeps the live inner nodes at even depth (each adopts its
//                    grandchildren); an exclusive scan numbers them (root = 0)
//  10. emit_node4  : Node4 records in the layout the render kernel traverses
// The triangle records are produced exactly as the host path produces them (fp64: e1 =
// v1 - v0 in fp64; fp32: each vertex rounded once, the normal from fp64), so only the tree differs: closest hits
// -- and pixels -- are the same as with the host SAH tree.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>   // before rocprim: its texture iterator calls memset unqualified

#include <rocprim/rocprim.hpp>

#include "../../include/rt_hip.h"
#include "rt_lbvh.h"
#include "rt_scene.h"
#include "rt_treelet.h"

namespace rtx {
namespace {

__device__ __forceinline__ uint32_t expand10(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

__global__ void tri_keys(const rt_triangle* __restrict__ tri, int n, double lo0, double lo1, double lo2,
                         double inv0, double inv1, double inv2, uint32_t* __restrict__ keys,
                         uint32_t* __restrict__ vals) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const rt_triangle& t = tri[k];
    const double lo[3] = {lo0, lo1, lo2}, inv[3] = {inv0, inv1, inv2};
    uint32_t q[3];
    for (int a = 0; a < 3; ++a) {
        const double mn = fmin(t.v0[a], fmin(t.v1[a], t.v2[a])), mx = fmax(t.v0[a], fmax(t.v1[a], t.v2[a]));
        double u = (0.5 * (mn + mx) - lo[a]) * inv[a];
        u = u < 0 ? 0 : (u > 1 ? 1 : u);
        q[a] = (uint32_t)fmin(u * 1024.0, 1023.0);
    }
    keys[k] = (expand10(q[0]) << 2) | (expand10(q[1]) << 1) | expand10(q[2]);
    vals[k] = (uint32_t)k;
}

__device__ __forceinline__ int delta(const uint32_t* __restrict__ code, int n, int a, int b) {
    if (b < 0 || b >= n) return -1;
    const uint32_t ka = code[a], kb = code[b];
    if (ka == kb) return 32 + __clz((int)((uint32_t)a ^ (uint32_t)b));
    return __clz((int)(ka ^ kb));
}

// Binary node ids: internal i in [0, n-2] (root 0), leaf k = (n-1) + k.
__global__ void karras(const uint32_t* __restrict__ code, int n, uint32_t* __restrict__ child,
                       uint32_t* __restrict__ parent) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n - 1) return;
    const int d = (delta(code, n, i, i + 1) - delta(code, n, i, i - 1)) >= 0 ? 1 : -1;
    const int dmin = delta(code, n, i, i - d);
    int lmax = 2;
    while (delta(code, n, i, i + lmax * d) > dmin) lmax *= 2;
    int l = 0;
    for (int t = lmax / 2; t >= 1; t /= 2)
        if (delta(code, n, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = delta(code, n, i, j);
    int s = 0, t = l;
    do {
        t = (t + 1) >> 1;
        if (delta(code, n, i, i + (s + t) * d) > dnode) s += t;
    } while (t > 1);
    const int gamma = i + s * d + min(d, 0);
    const int lo = min(i, j), hi = max(i, j);
    const uint32_t left = (lo == gamma) ? (uint32_t)(n - 1 + gamma) : (uint32_t)gamma;
    const uint32_t right = (hi == gamma + 1) ? (uint32_t)(n - 1 + gamma + 1) : (uint32_t)(gamma + 1);
    child[2 * i] = left;
    child[2 * i + 1] = right;
    parent[left] = (uint32_t)i;
    parent[right] = (uint32_t)i;
}

// Outward-rounded fp32 box of an fp64 interval, the host builder's padding
// (rt_bvh.cpp to_float_box).
__device__ __forceinline__ void float_box(const double lo[3], const double hi[3], float* out) {
    for (int a = 0; a < 3; ++a) {
        const double pad = 1e-4 + 1e-5 * fmax(fabs(lo[a]), fabs(hi[a]));
        out[a] = nextafterf((float)(lo[a] - pad), -INFINITY);
        out[3 + a] = nextafterf((float)(hi[a] + pad), INFINITY);
    }
}

// each sorted triangle's box (the host builder's padding), SAH cost and count
__global__ void leaf_boxes(const rt_triangle* __restrict__ tri, const uint32_t* __restrict__ sorted_idx, int n,
                           float* __restrict__ box, float* __restrict__ cost, uint32_t* __restrict__ count) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const rt_triangle& t = tri[sorted_idx[k]];
    double lo[3], hi[3];
    for (int a = 0; a < 3; ++a) {
        lo[a] = fmin(t.v0[a], fmin(t.v1[a], t.v2[a]));
        hi[a] = fmax(t.v0[a], fmax(t.v1[a], t.v2[a]));
    }
    const size_t id = (size_t)(n - 1 + k);
    float_box(lo, hi, box + id * 6);
    cost[id] = TREELET_CT * half_area(box + id * 6);
    count[id] = 1u;
}

// fp64 records (TriD: v0, e1, e2 in fp64, meta inside) or fp32 records (TriF: the three
// vertices rounded once, meta to the side array), as the host path builds them, each at its
// leaf's depth-first position; lidx[position] = the input index
template <class Tri>
__global__ void tri_pack(const rt_triangle* __restrict__ tri, const uint32_t* __restrict__ sorted_idx, int n,
                         const uint32_t* __restrict__ mat_type, const uint32_t* __restrict__ off, Tri* __restrict__ out,
                         uint32_t* __restrict__ tmeta, uint32_t* __restrict__ lidx) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint32_t src = sorted_idx[k];
    const rt_triangle& t = tri[src];
    const uint32_t pos = off[n - 1 + k];
    Tri r{};
    double e1[3], e2[3];
    for (int a = 0; a < 3; ++a) {
        if constexpr (sizeof(Tri) == sizeof(TriD)) {
            r.v0[a] = t.v0[a];
            r.e1[a] = t.v1[a] - t.v0[a];
            r.e2[a] = t.v2[a] - t.v0[a];
        } else {
            r.v0[a] = (float)t.v0[a];
            r.v1[a] = (float)t.v1[a];
            r.v2[a] = (float)t.v2[a];
        }
        e1[a] = t.v1[a] - t.v0[a];
        e2[a] = t.v2[a] - t.v0[a];
    }
    const uint32_t meta = make_meta((uint32_t)t.mat, mat_type[t.mat], 0u);
    if constexpr (sizeof(Tri) == sizeof(TriD)) {
        r.meta = meta;
    } else {
        tmeta[pos] = meta;
        r.n[0] = (float)(e1[1] * e2[2] - e1[2] * e2[1]);   // the facet normal, fp64 (as the host path)
        r.n[1] = (float)(e1[2] * e2[0] - e1[0] * e2[2]);
        r.n[2] = (float)(e1[0] * e2[1] - e1[1] * e2[0]);
    }
    out[pos] = r;
    lidx[pos] = src;
}

__global__ void node_depth(const uint32_t* __restrict__ parent, int n, int* __restrict__ depth,
                           int* __restrict__ max_depth) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n - 1) return;
    int d = 0;
    for (uint32_t v = (uint32_t)i; v != 0; v = parent[v]) ++d;
    depth[i] = d;
    atomicMax(max_depth, d);
}

__global__ void level_box(const uint32_t* __restrict__ child, const int* __restrict__ depth, int n, int level,
                          float* __restrict__ box, float* __restrict__ cost, uint32_t* __restrict__ count) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n - 1 || depth[i] != level) return;
    const uint32_t ca = child[2 * i], cb = child[2 * i + 1];
    const float* a = box + (size_t)ca * 6;
    const float* b = box + (size_t)cb * 6;
    float* o = box + (size_t)i * 6;
    for (int c = 0; c < 3; ++c) {
        o[c] = fminf(a[c], b[c]);
        o[3 + c] = fmaxf(a[3 + c], b[3 + c]);
    }
    cost[i] = TREELET_CI * half_area(o) + cost[ca] + cost[cb];
    count[i] = count[ca] + count[cb];
}

// The treelet roots of each depth in one list (a counting sort by depth, per round): nodes
// of 3 or more triangles (fewer have one topology).  hist / cursor: TREELET_DEPTHS counters.
constexpr int TREELET_DEPTHS = 256;
__global__ void depth_hist(const int* __restrict__ depth, const uint32_t* __restrict__ count, int n,
                           uint32_t* __restrict__ hist) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n - 1 || count[i] < 3) return;
    atomicAdd(hist + depth[i], 1u);
}
__global__ void depth_scatter(const int* __restrict__ depth, const uint32_t* __restrict__ count, int n,
                              uint32_t* __restrict__ cursor, uint32_t* __restrict__ list) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n - 1 || count[i] < 3) return;
    list[atomicAdd(cursor + depth[i], 1u)] = (uint32_t)i;
}

// one depth of treelet restructuring, one wave per treelet root (the treelets under the
// nodes of one depth are disjoint)
__global__ __launch_bounds__(64) void treelet_wave(TreeView t, const uint32_t* __restrict__ roots) {
    __shared__ float copt[1 << TREELET_LEAVES];
    __shared__ uint8_t split[1 << TREELET_LEAVES];
    __shared__ uint32_t leaf[2 * TREELET_LEAVES];
    __shared__ int nl;
    optimize_treelet_wave(t, roots[blockIdx.x], copt, split, leaf, &nl);
}

// the leaves' depth-first positions, top down one depth per launch: a node's range starts
// at off[node], its left child's at the same place, its right child's after the left's
__global__ void leaf_offsets(const uint32_t* __restrict__ child, const int* __restrict__ depth,
                             const uint32_t* __restrict__ count, int n, int level, uint32_t* __restrict__ off) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n - 1 || depth[i] != level) return;
    const uint32_t a = child[2 * i], b = child[2 * i + 1];
    off[a] = off[i];
    off[b] = off[i] + count[a];
}

// every node's triangle range [first, last] in leaf positions
__global__ void node_ranges(const uint32_t* __restrict__ off, const uint32_t* __restrict__ count, int nn,
                            uint32_t* __restrict__ range) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nn) return;
    range[2 * i] = off[i];
    range[2 * i + 1] = off[i] + count[i] - 1u;
}

// Node kinds for the 4-wide tree: small (<= max_leaf triangles) internal nodes become
// leaves.  keep[i] = 1 for live inner nodes at even depth (the Node4s).
__global__ void classify(const uint32_t* __restrict__ parent, const uint32_t* __restrict__ range,
                         const int* __restrict__ depth, int n, int max_leaf, uint32_t* __restrict__ keep,
                         int* __restrict__ max_live_depth) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n - 1) return;
    const bool small = (int)(range[2 * i + 1] - range[2 * i]) + 1 <= max_leaf;
    bool live = !small;
    if (live && i != 0) {
        const uint32_t p = parent[i];
        live = (int)(range[2 * p + 1] - range[2 * p]) + 1 > max_leaf;
    }
    keep[i] = (live && (depth[i] & 1) == 0) ? 1u : 0u;
    if (live) atomicMax(max_live_depth, depth[i]);
}

__device__ __forceinline__ bool is_leafish(uint32_t id, const uint32_t* range, int max_leaf) {
    return (int)(range[2 * id + 1] - range[2 * id]) + 1 <= max_leaf;
}

__device__ __forceinline__ uint32_t leaf_ref(uint32_t id, const uint32_t* range) {
    const uint32_t lo = range[2 * id], hi = range[2 * id + 1];
    return MREF_LEAF | ((hi - lo) << 24) | lo;
}

__global__ void emit_node4(const uint32_t* __restrict__ child, const uint32_t* __restrict__ range,
                           const uint32_t* __restrict__ keep, const uint32_t* __restrict__ index, const float* __restrict__ box,
                           int n, int max_leaf, Node4* __restrict__ out, int* __restrict__ leaves) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n - 1 || !keep[i]) return;
    uint32_t kid[4];
    int m = 0;
    for (int c = 0; c < 2; ++c) {
        const uint32_t ch = child[2 * i + c];
        if (is_leafish(ch, range, max_leaf)) {
            kid[m++] = ch;
        } else {
            kid[m++] = child[2 * ch];
            kid[m++] = child[2 * ch + 1];
        }
    }
    Node4 nd;
    int nleaves = 0;
    for (int k = 0; k < 4; ++k) {
        if (k < m) {
            const float* b = box + (size_t)kid[k] * 6;
            nd.lox[k] = b[0];
            nd.loy[k] = b[1];
            nd.loz[k] = b[2];
            nd.hix[k] = b[3];
            nd.hiy[k] = b[4];
            nd.hiz[k] = b[5];
            if (is_leafish(kid[k], range, max_leaf)) {
                nd.ref[k] = leaf_ref(kid[k], range);
                ++nleaves;
            } else {
                nd.ref[k] = index[kid[k]];
            }
        } else {
            nd.lox[k] = nd.loy[k] = nd.loz[k] = INFINITY;
            nd.hix[k] = nd.hiy[k] = nd.hiz[k] = -INFINITY;
            nd.ref[k] = MREF_EMPTY;
        }
        nd.pad[k] = 0;
    }
    out[index[i]] = nd;
    if (nleaves) atomicAdd(leaves, nleaves);
}

// n == 1 or a root that is itself small: one Node4 with a single leaf child.
__global__ void emit_single(const float* __restrict__ box, int n, Node4* __restrict__ out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    Node4 nd;
    const float* b = box;   // binary id 0: the root (n > 1) or the only leaf (n == 1)
    for (int k = 0; k < 4; ++k) {
        nd.lox[k] = nd.loy[k] = nd.loz[k] = INFINITY;
        nd.hix[k] = nd.hiy[k] = nd.hiz[k] = -INFINITY;
        nd.ref[k] = MREF_EMPTY;
        nd.pad[k] = 0;
    }
    nd.lox[0] = b[0];
    nd.loy[0] = b[1];
    nd.loz[0] = b[2];
    nd.hix[0] = b[3];
    nd.hiy[0] = b[4];
    nd.hiz[0] = b[5];
    nd.ref[0] = MREF_LEAF | ((uint32_t)(n - 1) << 24);
    out[0] = nd;
}

#define CHK(x)                                  \
    do {                                        \
        hipError_t e_ = (x);                    \
        if (e_ != hipSuccess) return e_;        \
    } while (0)

}  // namespace

hipError_t lbvh_build(const LbvhInput& in, LbvhScratch& ws, LbvhOutput& out, hipStream_t st) {
    const int n = in.n;
    const unsigned B = 256, G = (unsigned)((n + B - 1) / B), Gi = (unsigned)((n > 1 ? n - 1 : 1) + B - 1) / B;
    // scratch (grown on demand, kept for rebuilds)
    auto need = [&](void** p, size_t* cap, size_t bytes) -> hipError_t {
        if (*cap >= bytes && *p) return hipSuccess;
        if (*p) CHK(hipFree(*p));
        *p = nullptr;
        *cap = 0;
        CHK(hipMalloc(p, bytes ? bytes : 16));
        *cap = bytes;
        return hipSuccess;
    };
    const size_t nn = (size_t)(n > 1 ? 2 * n - 1 : 1), ni = (size_t)(n > 1 ? n - 1 : 1);
    CHK(need(&ws.keys, &ws.keys_cap, (size_t)n * 4 * 4));
    CHK(need(&ws.child, &ws.child_cap, ni * 2 * 4 + nn * 2 * 4));
    CHK(need(&ws.box, &ws.box_cap, nn * 6 * 4 + nn * 4 * 4));
    CHK(need(&ws.index, &ws.index_cap, ni * 4 * 3 + 64 + 4 * 260));
    uint32_t* keys = (uint32_t*)ws.keys;
    uint32_t* keys_s = keys + n;
    uint32_t* vals = keys + 2 * (size_t)n;
    uint32_t* vals_s = keys + 3 * (size_t)n;
    uint32_t* lidx = keys;                                       // after the sort: input index by leaf position
    uint32_t* child = (uint32_t*)ws.child;                       // 2(n-1)
    uint32_t* range = child + 2 * ni;                            // 2(2n-1): every node's [first, last]
    float* box = (float*)ws.box;                                 // 6(2n-1)
    uint32_t* parent = (uint32_t*)(box + nn * 6);                // 2n-1
    float* cost = (float*)(parent + nn);                         // 2n-1
    uint32_t* count = (uint32_t*)(cost + nn);                    // 2n-1
    uint32_t* off = count + nn;                                  // 2n-1
    uint32_t* keep = (uint32_t*)ws.index;                        // n-1
    uint32_t* index = keep + ni;                                 // n-1
    int* depth = (int*)(index + ni);                             // n-1
    int* counters = depth + ni;   // [0] max live depth, [1] leaves, [2] max depth; [4..] treelet roots per depth
    // (keep[] doubles as the treelet roots' list before classify fills it)
    const TreeView tv{child, parent, box, cost, count, n};

    hipLaunchKernelGGL(tri_keys, dim3(G), dim3(B), 0, st, in.tris, n, in.lo[0], in.lo[1], in.lo[2], in.inv[0],
                       in.inv[1], in.inv[2], keys, vals);
    CHK(hipGetLastError());
    size_t tmp = 0;
    CHK(rocprim::radix_sort_pairs(nullptr, tmp, keys, keys_s, vals, vals_s, (size_t)n, 0, 30, st));
    CHK(need(&ws.sort_tmp, &ws.sort_tmp_cap, tmp));
    CHK(rocprim::radix_sort_pairs(ws.sort_tmp, tmp, keys, keys_s, vals, vals_s, (size_t)n, 0, 30, st));
    CHK(hipMemsetAsync(counters, 0, 16, st));
    CHK(hipMemsetAsync(off, 0, nn * 4, st));   // (the root's position: 0)
    hipLaunchKernelGGL(leaf_boxes, dim3(G), dim3(B), 0, st, in.tris, vals_s, n, box, cost, count);
    CHK(hipGetLastError());
    // depths of the internal nodes and the deepest (host), as each pass by depth needs them
    auto depths = [&](int& maxd) -> hipError_t {
        CHK(hipMemsetAsync(counters + 2, 0, 4, st));
        hipLaunchKernelGGL(node_depth, dim3(Gi), dim3(B), 0, st, parent, n, depth, counters + 2);
        CHK(hipGetLastError());
        CHK(hipMemcpyAsync(&maxd, counters + 2, 4, hipMemcpyDeviceToHost, st));
        return hipStreamSynchronize(st);
    };
    if (n > 1) {
        hipLaunchKernelGGL(karras, dim3(Gi), dim3(B), 0, st, keys_s, n, child, parent);
        CHK(hipGetLastError());
        int maxd = 0;
        CHK(depths(maxd));
        for (int level = maxd; level >= 0; --level) {
            hipLaunchKernelGGL(level_box, dim3(Gi), dim3(B), 0, st, child, depth, n, level, box, cost, count);
            CHK(hipGetLastError());
        }
        for (int round = 0; round < in.treelet_rounds; ++round) {
            CHK(depths(maxd));
            if (maxd >= TREELET_DEPTHS) break;   // (a degenerate tree: left as it is)
            uint32_t hist[TREELET_DEPTHS], start[TREELET_DEPTHS + 1];
            CHK(hipMemsetAsync(counters + 4, 0, TREELET_DEPTHS * 4, st));
            hipLaunchKernelGGL(depth_hist, dim3(Gi), dim3(B), 0, st, depth, count, n, (uint32_t*)(counters + 4));
            CHK(hipGetLastError());
            CHK(hipMemcpyAsync(hist, counters + 4, TREELET_DEPTHS * 4, hipMemcpyDeviceToHost, st));
            CHK(hipStreamSynchronize(st));
            start[0] = 0;
            for (int d = 0; d < TREELET_DEPTHS; ++d) start[d + 1] = start[d] + hist[d];
            CHK(hipMemcpyAsync(counters + 4, start, TREELET_DEPTHS * 4, hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(depth_scatter, dim3(Gi), dim3(B), 0, st, depth, count, n, (uint32_t*)(counters + 4),
                               keep);
            CHK(hipGetLastError());
            for (int level = maxd; level >= 0; --level) {
                if (hist[level] == 0) continue;
                hipLaunchKernelGGL(treelet_wave, dim3(hist[level]), dim3(64), 0, st, tv, keep + start[level]);
                CHK(hipGetLastError());
            }
        }
        CHK(depths(maxd));
        for (int level = 0; level <= maxd; ++level) {
            hipLaunchKernelGGL(leaf_offsets, dim3(Gi), dim3(B), 0, st, child, depth, count, n, level, off);
            CHK(hipGetLastError());
        }
    }
    hipLaunchKernelGGL(node_ranges, dim3((unsigned)((nn + B - 1) / B)), dim3(B), 0, st, off, count, (int)nn, range);
    CHK(hipGetLastError());
    if (in.f64)
        hipLaunchKernelGGL(tri_pack<TriD>, dim3(G), dim3(B), 0, st, in.tris, vals_s, n, in.mat_type, off,
                           (TriD*)out.tris, out.tmeta, lidx);
    else
        hipLaunchKernelGGL(tri_pack<TriF>, dim3(G), dim3(B), 0, st, in.tris, vals_s, n, in.mat_type, off,
                           (TriF*)out.tris, out.tmeta, lidx);
    CHK(hipGetLastError());
    const bool single = n <= in.max_leaf;
    int node4 = 0;
    if (single) {
        // the whole mesh fits one leaf: its box is the root's (or the only triangle's)
        hipLaunchKernelGGL(emit_single, dim3(1), dim3(64), 0, st, box, n, out.nodes);
        CHK(hipGetLastError());
        node4 = 1;
        out.depth4 = 1;
        out.leaves = 1;
    } else {
        hipLaunchKernelGGL(classify, dim3(Gi), dim3(B), 0, st, parent, range, depth, n, in.max_leaf, keep, counters);
        CHK(hipGetLastError());
        size_t stmp = 0;
        CHK(rocprim::exclusive_scan(nullptr, stmp, keep, index, 0u, (size_t)(n - 1), rocprim::plus<uint32_t>(), st));
        CHK(need(&ws.scan_tmp, &ws.scan_tmp_cap, stmp));
        CHK(rocprim::exclusive_scan(ws.scan_tmp, stmp, keep, index, 0u, (size_t)(n - 1), rocprim::plus<uint32_t>(),
                                    st));
        uint32_t last_keep = 0, last_index = 0;
        int cnt[2] = {0, 0};
        CHK(hipMemcpyAsync(&last_keep, keep + (n - 2), 4, hipMemcpyDeviceToHost, st));
        CHK(hipMemcpyAsync(&last_index, index + (n - 2), 4, hipMemcpyDeviceToHost, st));
        CHK(hipStreamSynchronize(st));
        node4 = (int)(last_index + last_keep);
        if (node4 > out.nodes_cap) return hipErrorOutOfMemory;   // caller sized nodes for n-1
        hipLaunchKernelGGL(emit_node4, dim3(Gi), dim3(B), 0, st, child, range, keep, index, box, n, in.max_leaf,
                           out.nodes, counters + 1);
        CHK(hipGetLastError());
        CHK(hipMemcpyAsync(cnt, counters, 8, hipMemcpyDeviceToHost, st));
        CHK(hipStreamSynchronize(st));
        out.depth4 = cnt[0] / 2 + 1;
        out.leaves = cnt[1];
    }
    out.node_count = node4;
    return hipStreamSynchronize(st);
}

}  // namespace rtx

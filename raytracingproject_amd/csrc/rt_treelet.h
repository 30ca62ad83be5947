// rt_treelet.h -- treelet restructuring of a binary BVH (r06; Karras & Aila, "Fast
// Parallel Construction of High-Quality Bounding Volume Hierarchies", HPG 2013), the
// quality pass of the GPU mesh builder (rt_lbvh.hip, RT_MESH_BUILD_GPU).
//
// A treelet is an internal node R and the part of its subtree found by repeatedly opening
// the treelet leaf with the largest surface area, up to TREELET_LEAVES leaves.  Its
// internal topology is then replaced by the one that minimises the SAH cost over those
// leaves -- a dynamic program over the 2^k subsets of the k leaves -- reusing the treelet's
// own internal node ids; R keeps its id, its box and the set of primitives below it, so
// the tree above R is unaffected and treelets rooted at distinct nodes of one depth are
// disjoint (rt_lbvh.hip processes one depth per launch, deepest first).
//
// Plain C++ usable on the host (tests/cpp/treelet_check.cpp) and the device.
#pragma once
#include <cstdint>

#ifdef __HIPCC__
#define RT_HD __host__ __device__
#else
#define RT_HD
#endif

namespace rtx {

constexpr int TREELET_LEAVES = 7;
constexpr float TREELET_CI = 1.0f;   // SAH cost of an internal node per unit of surface area
constexpr float TREELET_CT = 1.0f;   // ... of a primitive (leaf) per unit of surface area

// Binary tree in flat arrays: internal nodes [0, n - 1) (root 0), leaf k = (n - 1) + k.
//   child[2 i + c], parent[id], box[6 id] (lo xyz, hi xyz), cost[id] = subtree SAH cost
//   (leaf: TREELET_CT * area; internal: TREELET_CI * area + the children's costs),
//   count[id] = primitives below.
struct TreeView {
    uint32_t* child;
    uint32_t* parent;
    float* box;
    float* cost;
    uint32_t* count;
    int n;
};

RT_HD inline float half_area(const float* b) {
    const float dx = b[3] - b[0], dy = b[4] - b[1], dz = b[5] - b[2];
    return dx * dy + dy * dz + dz * dx;
}

// The treelet under internal node r: its leaves (opening the internal treelet leaf with the
// largest surface area until TREELET_LEAVES) and internal nodes (r first); returns the
// number of leaves.
RT_HD inline int form_treelet(const TreeView& t, uint32_t r, uint32_t* leaf, uint32_t* inner) {
    constexpr int K = TREELET_LEAVES;
    const uint32_t nint = (uint32_t)(t.n - 1);
    int nl = 2, ni = 1;
    leaf[0] = t.child[2 * r];
    leaf[1] = t.child[2 * r + 1];
    inner[0] = r;
    while (nl < K) {
        int best = -1;
        float ba = -1.f;
        for (int k = 0; k < nl; ++k) {
            if (leaf[k] >= nint) continue;   // a primitive
            const float a = half_area(t.box + 6 * (size_t)leaf[k]);
            if (a > ba) {
                ba = a;
                best = k;
            }
        }
        if (best < 0) break;
        const uint32_t v = leaf[best];
        inner[ni++] = v;
        leaf[best] = t.child[2 * v];
        leaf[nl++] = t.child[2 * v + 1];
    }
    return nl;
}

// Surface area of the union of the leaves in subset s.
RT_HD inline float subset_area(const TreeView& t, const uint32_t* leaf, int s) {
    float lo[3] = {3.4e38f, 3.4e38f, 3.4e38f}, hi[3] = {-3.4e38f, -3.4e38f, -3.4e38f};
    for (int m = s; m; m &= m - 1) {
        const float* b = t.box + 6 * (size_t)leaf[__builtin_ctz((unsigned)m)];
        for (int a = 0; a < 3; ++a) {
            lo[a] = lo[a] < b[a] ? lo[a] : b[a];
            hi[a] = hi[a] > b[3 + a] ? hi[a] : b[3 + a];
        }
    }
    const float bb[6] = {lo[0], lo[1], lo[2], hi[0], hi[1], hi[2]};
    return half_area(bb);
}

// The best split of subset s (>= 2 leaves) given every proper subset's optimal cost: the
// first partition in enumeration order of strictly least cost, p holding s's lowest leaf
// (each split counted once); returns its cost.
RT_HD inline float best_split(const float* copt, int s, int& bp) {
    float best = 3.4e38f;
    bp = 0;
    const int low = s & -s;
    for (int p = (s - 1) & s; p > 0; p = (p - 1) & s) {
        if (!(p & low)) continue;
        const float c = copt[p] + copt[s ^ p];
        if (c < best) {
            best = c;
            bp = p;
        }
    }
    return best;
}

// Rebuilds the treelet's topology from the optimal splits (node ids from `inner`, r first)
// and recomputes the boxes, costs and counts of its internal nodes, children first.
RT_HD inline void rebuild_treelet(const TreeView& t, uint32_t r, const uint32_t* leaf, const uint32_t* inner, int nl,
                                  const uint8_t* split) {
    constexpr int K = TREELET_LEAVES;
    int stack_s[K], stack_id[K], sp = 0, used = 1;
    uint32_t order[K - 1];
    int no = 0;
    const int full = (1 << nl) - 1;
    stack_s[sp] = full;
    stack_id[sp++] = (int)r;
    while (sp > 0) {
        --sp;
        const int s = stack_s[sp];
        const uint32_t id = (uint32_t)stack_id[sp];
        order[no++] = id;
        const int parts[2] = {split[s], s ^ split[s]};
        for (int c = 0; c < 2; ++c) {
            const int ps = parts[c];
            uint32_t cid;
            if ((ps & (ps - 1)) == 0) {
                cid = leaf[__builtin_ctz((unsigned)ps)];
            } else {
                cid = inner[used++];
                stack_s[sp] = ps;
                stack_id[sp++] = (int)cid;
            }
            t.child[2 * id + c] = cid;
            t.parent[cid] = id;
        }
    }
    for (int k = no - 1; k >= 0; --k) {
        const uint32_t id = order[k], a = t.child[2 * id], b = t.child[2 * id + 1];
        float* o = t.box + 6 * (size_t)id;
        const float* ba = t.box + 6 * (size_t)a;
        const float* bb = t.box + 6 * (size_t)b;
        for (int x = 0; x < 3; ++x) {
            o[x] = ba[x] < bb[x] ? ba[x] : bb[x];
            o[3 + x] = ba[3 + x] > bb[3 + x] ? ba[3 + x] : bb[3 + x];
        }
        t.cost[id] = TREELET_CI * half_area(o) + t.cost[a] + t.cost[b];
        t.count[id] = t.count[a] + t.count[b];
    }
}

// Restructures the treelet rooted at internal node r (one thread); returns true when its
// topology changed.  Subsets are solved in increasing numeric order: a proper subset of s
// is numerically smaller than s.
RT_HD inline bool optimize_treelet(const TreeView& t, uint32_t r) {
    constexpr int K = TREELET_LEAVES, S = 1 << K;
    uint32_t leaf[K], inner[K - 1];
    const int nl = form_treelet(t, r, leaf, inner);
    if (nl < 3) return false;   // two leaves: one topology
    float area[S], copt[S];
    uint8_t split[S];
    const int full = (1 << nl) - 1;
    for (int s = 1; s <= full; ++s) {
        split[s] = 0;
        if ((s & (s - 1)) == 0) {   // a single leaf: its own subtree cost
            copt[s] = t.cost[leaf[__builtin_ctz((unsigned)s)]];
            continue;
        }
        area[s] = subset_area(t, leaf, s);
        int bp;
        const float best = best_split(copt, s, bp);
        copt[s] = TREELET_CI * area[s] + best;
        split[s] = (uint8_t)bp;
    }
    if (!(copt[full] < t.cost[r] * (1.f - 1e-6f))) return false;   // (no gain beyond rounding)
    rebuild_treelet(t, r, leaf, inner, nl, split);
    return true;
}

#ifdef __HIPCC__
// The same, one wave per treelet (rt_lbvh.hip treelet_wave): lanes solve the subsets of one
// size at a time (a subset's proper subsets are all smaller), in LDS; lane 0 forms and
// rebuilds the treelet.  The same operations per subset as optimize_treelet: the same tree.
__device__ inline void optimize_treelet_wave(const TreeView& t, uint32_t r, float* copt, uint8_t* split,
                                             uint32_t* shared_leaf, int* shared_nl) {
    constexpr int K = TREELET_LEAVES;
    const int lane = (int)(threadIdx.x & 63);
    if (lane == 0) {
        uint32_t leaf[K], inner[K - 1];
        const int nl = form_treelet(t, r, leaf, inner);
        for (int k = 0; k < K; ++k) shared_leaf[k] = k < nl ? leaf[k] : 0u;
        for (int k = 0; k < K - 1; ++k) shared_leaf[K + k] = k < nl - 1 ? inner[k] : 0u;
        *shared_nl = nl;
    }
    __syncthreads();
    const int nl = *shared_nl;
    if (nl < 3) return;
    const int full = (1 << nl) - 1;
    uint32_t leaf[K];
    for (int k = 0; k < K; ++k) leaf[k] = shared_leaf[k];
    for (int s = lane + 1; s <= full; s += 64)
        if ((s & (s - 1)) == 0) copt[s] = t.cost[leaf[__builtin_ctz((unsigned)s)]];
    __syncthreads();
    for (int size = 2; size <= nl; ++size) {
        for (int s = lane + 1; s <= full; s += 64) {
            if (__builtin_popcount((unsigned)s) != size) continue;
            const float area = subset_area(t, leaf, s);
            int bp;
            const float best = best_split(copt, s, bp);
            copt[s] = TREELET_CI * area + best;
            split[s] = (uint8_t)bp;
        }
        __syncthreads();
    }
    if (lane == 0 && copt[full] < t.cost[r] * (1.f - 1e-6f)) {
        uint32_t inner[K - 1];
        for (int k = 0; k < K - 1; ++k) inner[k] = shared_leaf[K + k];
        rebuild_treelet(t, r, leaf, inner, nl, split);
    }
}
#endif

}  // namespace rtx

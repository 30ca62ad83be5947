// rt_bvh.cpp -- host SAH BVH builder (see rt_bvh.h).
#include "rt_bvh.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>

#include "../../include/rt_hip.h"

namespace rtx {
namespace {

struct Box {
    double lo[3] = {std::numeric_limits<double>::infinity(), std::numeric_limits<double>::infinity(),
                    std::numeric_limits<double>::infinity()};
    double hi[3] = {-std::numeric_limits<double>::infinity(), -std::numeric_limits<double>::infinity(),
                    -std::numeric_limits<double>::infinity()};
    void grow(const Box& b) {
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], b.lo[a]);
            hi[a] = std::max(hi[a], b.hi[a]);
        }
    }
    double area() const {
        double d0 = hi[0] - lo[0], d1 = hi[1] - lo[1], d2 = hi[2] - lo[2];
        if (!(d0 >= 0) || !(d1 >= 0) || !(d2 >= 0)) return 0.0;
        return 2.0 * (d0 * d1 + d1 * d2 + d2 * d0);
    }
};

Box exact_box(const rt_sphere& s) {
    Box b;
    for (int a = 0; a < 3; ++a) {
        double c0 = s.center[a], c1 = s.center[a] + (s.moving ? s.center_vec[a] : 0.0);
        b.lo[a] = std::min(c0, c1) - s.radius;
        b.hi[a] = std::max(c0, c1) + s.radius;
    }
    return b;
}

// Widen a double interval to fp32 so the slab test (relative error a few ulp of t)
// can never cull a sphere the exact test would hit.
void to_float_box(const Box& b, float lo[3], float hi[3]) {
    for (int a = 0; a < 3; ++a) {
        double pad = 1e-4 + 1e-5 * std::max(std::fabs(b.lo[a]), std::fabs(b.hi[a]));
        lo[a] = std::nextafter((float)(b.lo[a] - pad), -std::numeric_limits<float>::infinity());
        hi[a] = std::nextafter((float)(b.hi[a] + pad), std::numeric_limits<float>::infinity());
    }
}

struct Builder {
    const BvhParams& p;
    std::vector<Box> boxes;
    std::vector<double> cent[3];
    std::vector<int> idx;        // working permutation of BVH prims (input indices)
    BuiltBvh& out;
    int max_depth = 0;

    Builder(const BvhParams& params, BuiltBvh& o) : p(params), out(o) {}

    uint32_t make_leaf(int b, int e, Box& box) {
        int first = (int)out.order.size();
        for (int k = b; k < e; ++k) {
            out.order.push_back(idx[k]);
            box.grow(boxes[idx[k]]);
        }
        out.leaves++;
        return REF_LEAF | (uint32_t)(e - b - 1) << 11 | (uint32_t)first;
    }

    // Returns the ref of the subtree over idx[b, e) and its box.
    uint32_t build(int b, int e, int depth, Box& box) {
        const int n = e - b;
        Box nb;
        for (int k = b; k < e; ++k) nb.grow(boxes[idx[k]]);
        if (n == 1) return make_leaf(b, e, box);

        // full-sweep SAH over the three centroid orders; deep trees (degenerate inputs:
        // coincident centres make every split peel off one sphere) fall back to median
        // splits before the LDS stack limit, as the mesh builder does
        double best_cost = std::numeric_limits<double>::infinity();
        int best_axis = -1, best_split = -1;
        std::vector<double> right_area(n);
        for (int axis = 0; axis < 3 && depth < STACK_MAX - 8; ++axis) {
            std::stable_sort(idx.begin() + b, idx.begin() + e,
                             [&](int x, int y) { return cent[axis][x] < cent[axis][y]; });
            Box acc;
            for (int k = n - 1; k >= 1; --k) {
                acc.grow(boxes[idx[b + k]]);
                right_area[k] = acc.area();
            }
            Box lacc;
            for (int k = 1; k < n; ++k) {
                lacc.grow(boxes[idx[b + k - 1]]);
                double c = lacc.area() * k + right_area[k] * (n - k);
                if (c < best_cost) {
                    best_cost = c;
                    best_axis = axis;
                    best_split = k;
                }
            }
        }
        double area = nb.area();
        double split_cost = p.cost_traverse * area + p.cost_intersect * best_cost;
        double leaf_cost = p.cost_intersect * n * area;
        if (n <= p.max_leaf && (best_axis < 0 || leaf_cost <= split_cost)) return make_leaf(b, e, box);
        if (best_axis < 0) {   // no finite split cost (cannot happen within COORD_MAX): median on x
            best_axis = 0;
            best_split = n / 2;
        }

        std::stable_sort(idx.begin() + b, idx.begin() + e,
                         [&](int x, int y) { return cent[best_axis][x] < cent[best_axis][y]; });
        int node = (int)out.nodes.size();
        out.nodes.emplace_back();
        max_depth = std::max(max_depth, depth);
        Box b0, b1;
        uint32_t r0 = build(b, b + best_split, depth + 1, b0);
        uint32_t r1 = build(b + best_split, e, depth + 1, b1);
        Node& nd = out.nodes[node];
        to_float_box(b0, nd.lo0, nd.hi0);
        to_float_box(b1, nd.lo1, nd.hi1);
        nd.ref0 = r0;
        nd.ref1 = r1;
        nd.pad0 = nd.pad1 = 0;
        box.grow(b0);
        box.grow(b1);
        return (uint32_t)node;
    }
};

// ---- binned SAH over triangles ------------------------------------------------------
struct MeshBuilder {
    const std::vector<Box>& boxes;
    const std::vector<double>* cent;   // [3]
    std::vector<int>& idx;
    MeshBvh& out;
    int max_leaf;
    double cost_traverse;
    int max_depth = 0;
#ifndef RT_MESH_BINS
#define RT_MESH_BINS 32
#endif
    static constexpr int BINS = RT_MESH_BINS;   // SAH bins per axis

    MeshBuilder(const std::vector<Box>& b, const std::vector<double>* c, std::vector<int>& i, MeshBvh& o, int ml,
                double ct)
        : boxes(b), cent(c), idx(i), out(o), max_leaf(ml), cost_traverse(ct) {}

    uint32_t make_leaf(int b, int e, Box& box) {
        const int first = (int)out.order.size();
        for (int k = b; k < e; ++k) {
            out.order.push_back(idx[k]);
            box.grow(boxes[idx[k]]);
        }
        out.leaves++;
        return MREF_LEAF | (uint32_t)(e - b - 1) << 24 | (uint32_t)first;
    }

    uint32_t build(int b, int e, int depth, Box& box) {
        const int n = e - b;
        Box nb, cb;
        for (int k = b; k < e; ++k) {
            nb.grow(boxes[idx[k]]);
            Box c;
            for (int a = 0; a < 3; ++a) c.lo[a] = c.hi[a] = cent[a][idx[k]];
            cb.grow(c);
        }
        if (n <= 1) return make_leaf(b, e, box);
        // deep trees (degenerate inputs) fall back to median splits before the stack limit
        const bool force_median = depth >= MESH_STACK_MAX - 8;
        int best_axis = -1, best_bin = -1;
        double best_cost = std::numeric_limits<double>::infinity();
        if (!force_median) {
            for (int axis = 0; axis < 3; ++axis) {
                const double lo = cb.lo[axis], ext = cb.hi[axis] - cb.lo[axis];
                if (!(ext > 0)) continue;
                Box bbox[BINS];
                int cnt[BINS] = {0};
                for (int k = b; k < e; ++k) {
                    int bi = (int)((cent[axis][idx[k]] - lo) / ext * BINS);
                    bi = bi < 0 ? 0 : (bi >= BINS ? BINS - 1 : bi);
                    cnt[bi]++;
                    bbox[bi].grow(boxes[idx[k]]);
                }
                double right_area[BINS];
                int right_cnt[BINS];
                Box acc;
                int ac = 0;
                for (int bi = BINS - 1; bi >= 1; --bi) {
                    acc.grow(bbox[bi]);
                    ac += cnt[bi];
                    right_area[bi] = acc.area();
                    right_cnt[bi] = ac;
                }
                Box lacc;
                int lc = 0;
                for (int bi = 1; bi < BINS; ++bi) {
                    lacc.grow(bbox[bi - 1]);
                    lc += cnt[bi - 1];
                    if (lc == 0 || right_cnt[bi] == 0) continue;
                    const double c = lacc.area() * lc + right_area[bi] * right_cnt[bi];
                    if (c < best_cost) {
                        best_cost = c;
                        best_axis = axis;
                        best_bin = bi;
                    }
                }
            }
        }
        const double area = nb.area();
        const double leaf_cost = (double)n * area;
        const double split_cost = cost_traverse * area + best_cost;   // intersect cost 1
        if (n <= max_leaf && (best_axis < 0 || leaf_cost <= split_cost)) return make_leaf(b, e, box);

        int mid;
        if (best_axis >= 0) {
            const int axis = best_axis;
            const double lo = cb.lo[axis], ext = cb.hi[axis] - cb.lo[axis];
            auto it = std::partition(idx.begin() + b, idx.begin() + e, [&](int t) {
                int bi = (int)((cent[axis][t] - lo) / ext * BINS);
                bi = bi < 0 ? 0 : (bi >= BINS ? BINS - 1 : bi);
                return bi < best_bin;
            });
            mid = (int)(it - idx.begin());
        } else {
            mid = b;
        }
        if (mid <= b || mid >= e) {
            // no usable SAH split (all centroids in one bin): object median on the widest axis
            int axis = 0;
            for (int a = 1; a < 3; ++a)
                if (cb.hi[a] - cb.lo[a] > cb.hi[axis] - cb.lo[axis]) axis = a;
            mid = b + n / 2;
            std::nth_element(idx.begin() + b, idx.begin() + mid, idx.begin() + e,
                             [&](int x, int y) { return cent[axis][x] < cent[axis][y]; });
        }
        const int node = (int)out.nodes.size();
        out.nodes.emplace_back();
        max_depth = std::max(max_depth, depth);
        Box b0, b1;
        const uint32_t r0 = build(b, mid, depth + 1, b0);
        const uint32_t r1 = build(mid, e, depth + 1, b1);
        Node& nd = out.nodes[node];
        to_float_box(b0, nd.lo0, nd.hi0);
        to_float_box(b1, nd.lo1, nd.hi1);
        nd.ref0 = r0;
        nd.ref1 = r1;
        nd.pad0 = nd.pad1 = 0;
        box.grow(b0);
        box.grow(b1);
        return (uint32_t)node;
    }
};

}  // namespace

// Binary -> 4-wide: a node's children are its binary children, then repeatedly the inner
// child with the largest box is replaced by its two children until there are 4 (or only
// leaves).  Child boxes come from the binary nodes (already widened to fp32).
struct Collapse {
    const std::vector<Node>& bn;
    std::vector<Node4>& out;
    int max_depth = 0;
    struct Child {
        float lo[3], hi[3];
        uint32_t ref;
    };
    static double area(const Child& c) {
        const double d0 = (double)c.hi[0] - c.lo[0], d1 = (double)c.hi[1] - c.lo[1], d2 = (double)c.hi[2] - c.lo[2];
        return 2.0 * (d0 * d1 + d1 * d2 + d2 * d0);
    }
    void children_of(uint32_t b, Child* ch, int& n) const {
        const Node& nd = bn[b];
        Child c0, c1;
        for (int a = 0; a < 3; ++a) {
            c0.lo[a] = nd.lo0[a];
            c0.hi[a] = nd.hi0[a];
            c1.lo[a] = nd.lo1[a];
            c1.hi[a] = nd.hi1[a];
        }
        c0.ref = nd.ref0;
        c1.ref = nd.ref1;
        ch[n++] = c0;
        if (c1.ref != MREF_EMPTY) ch[n++] = c1;
    }
    uint32_t build(uint32_t b, int depth) {
        max_depth = std::max(max_depth, depth);
        Child ch[4];
        int n = 0;
        children_of(b, ch, n);
        while (n < 4) {
            int best = -1;
            double ba = -1.0;
            for (int k = 0; k < n; ++k)
                if (!(ch[k].ref & MREF_LEAF) && area(ch[k]) > ba) {
                    ba = area(ch[k]);
                    best = k;
                }
            if (best < 0) break;
            const uint32_t e = ch[best].ref;
            ch[best] = ch[n - 1];
            --n;
            children_of(e, ch, n);
        }
        const uint32_t idx = (uint32_t)out.size();
        out.emplace_back();
        Node4 nd{};
        for (int k = 0; k < 4; ++k) {
            if (k < n) {
                nd.lox[k] = ch[k].lo[0];
                nd.loy[k] = ch[k].lo[1];
                nd.loz[k] = ch[k].lo[2];
                nd.hix[k] = ch[k].hi[0];
                nd.hiy[k] = ch[k].hi[1];
                nd.hiz[k] = ch[k].hi[2];
                nd.ref[k] = (ch[k].ref & MREF_LEAF) ? ch[k].ref : build(ch[k].ref, depth + 1);
            } else {
                nd.lox[k] = nd.loy[k] = nd.loz[k] = std::numeric_limits<float>::infinity();
                nd.hix[k] = nd.hiy[k] = nd.hiz[k] = -std::numeric_limits<float>::infinity();
                nd.ref[k] = MREF_EMPTY;
            }
        }
        out[idx] = nd;
        return idx;
    }
};

// Relabel: the first min(MESH_TOP_MAX, n) nodes in breadth-first order, then the rest in
// their (depth-first) build order.
void mesh_top_first(std::vector<Node4>& nodes) {
    const size_t n = nodes.size();
    std::vector<uint32_t> newid(n, MREF_EMPTY);
    std::vector<uint32_t> bfs;
    bfs.push_back(0);
    for (size_t q = 0; q < bfs.size() && bfs.size() < (size_t)MESH_TOP_MAX; ++q) {
        const Node4& nd = nodes[bfs[q]];
        for (uint32_t r : nd.ref)
            if (!(r & MREF_LEAF) && bfs.size() < (size_t)MESH_TOP_MAX) bfs.push_back(r);
    }
    uint32_t next = 0;
    for (uint32_t k : bfs) newid[k] = next++;
    for (size_t k = 0; k < n; ++k)
        if (newid[k] == MREF_EMPTY) newid[k] = next++;
    std::vector<Node4> out(n);
    for (size_t k = 0; k < n; ++k) {
        Node4 nd = nodes[k];
        for (uint32_t& r : nd.ref)
            if (!(r & MREF_LEAF)) r = newid[r];
        out[newid[k]] = nd;
    }
    nodes.swap(out);
}

bool build_mesh_bvh(const rt_triangle* tris, int n, int max_leaf, double cost_traverse, MeshBvh& out,
                    std::string& err) {
    out = MeshBvh();
    if (n <= 0) return true;
    if (n > MESH_MAX_TRIS) {
        err = "mesh holds at most 2^24 triangles";
        return false;
    }
    max_leaf = std::max(1, std::min(max_leaf, MESH_LEAF_MAX));
    std::vector<Box> boxes(n);
    std::vector<double> cent[3];
    for (int a = 0; a < 3; ++a) cent[a].resize(n);
    std::vector<int> idx(n);
    for (int k = 0; k < n; ++k) {
        Box bx;
        for (int a = 0; a < 3; ++a) {
            const double x0 = tris[k].v0[a], x1 = tris[k].v1[a], x2 = tris[k].v2[a];
            if (!coord_ok(x0) || !coord_ok(x1) || !coord_ok(x2)) {
                err = "triangle " + std::to_string(k) + " has a vertex coordinate that is not finite or beyond +-1e30";
                return false;
            }
            bx.lo[a] = std::min(x0, std::min(x1, x2));
            bx.hi[a] = std::max(x0, std::max(x1, x2));
            cent[a][k] = 0.5 * (bx.lo[a] + bx.hi[a]);
        }
        boxes[k] = bx;
        idx[k] = k;
    }
    MeshBuilder B(boxes, cent, idx, out, max_leaf, cost_traverse > 0 ? cost_traverse : 1.0);
    Box root;
    const uint32_t r = B.build(0, n, 1, root);
    if (r & MREF_LEAF) {
        Node nd{};
        to_float_box(root, nd.lo0, nd.hi0);
        nd.ref0 = r;
        nd.ref1 = MREF_EMPTY;
        for (int a = 0; a < 3; ++a) {
            nd.lo1[a] = std::numeric_limits<float>::infinity();
            nd.hi1[a] = -std::numeric_limits<float>::infinity();
        }
        out.nodes.push_back(nd);
        B.max_depth = 1;
    }
    out.depth = B.max_depth;
    Collapse C{out.nodes, out.nodes4};
    C.build(0, 1);
    out.depth4 = C.max_depth;
    mesh_top_first(out.nodes4);
    // each 4-wide visit pushes at most 3 entries (one kept in a register)
    if (3 * out.depth4 + 1 > MESH_STACK_MAX) {
        err = "mesh BVH deeper than the traversal stack";
        return false;
    }
    return true;
}

void sphere_box(const rt_sphere& s, float lo[3], float hi[3]) { to_float_box(exact_box(s), lo, hi); }

bool build_bvh(const rt_sphere* spheres, int n, const BvhParams& p, BuiltBvh& out, std::string& err) {
    out = BuiltBvh();
    Builder B(p, out);
    B.boxes.resize(n);
    for (int a = 0; a < 3; ++a) B.cent[a].resize(n);
    for (int k = 0; k < n; ++k) {
        const rt_sphere& s = spheres[k];
        bool ok = coord_ok(s.radius);
        for (int a = 0; a < 3; ++a) ok = ok && coord_ok(s.center[a]) && coord_ok(s.center_vec[a]);
        if (!ok) {
            err = "sphere " + std::to_string(k) + " has a centre, motion or radius that is not finite or beyond +-1e30";
            return false;
        }
        // The reference keeps every sphere in one list; very large spheres (radius >=
        // BIG_RADIUS, the R=1000 ground) go to an fp64 side list instead of the BVH.
        if (std::fabs(s.radius) >= BIG_RADIUS) {
            out.big.push_back(k);
            continue;
        }
        B.boxes[k] = exact_box(s);
        for (int a = 0; a < 3; ++a) B.cent[a][k] = 0.5 * (B.boxes[k].lo[a] + B.boxes[k].hi[a]);
        B.idx.push_back(k);
    }
    if ((int)out.big.size() > MAX_BIG) {
        err = "more than " + std::to_string(MAX_BIG) + " spheres with radius >= " + std::to_string(BIG_RADIUS);
        return false;
    }
    int front = p.front;
    if (front < 0 && !B.idx.empty()) {
        // auto: the spheres at least 4x the median radius (main.cpp's three R = 1 spheres
        // among the R = 0.2 field), at most 8
        std::vector<double> r;
        for (int k : B.idx) r.push_back(std::fabs(spheres[k].radius));
        std::nth_element(r.begin(), r.begin() + r.size() / 2, r.end());
        const double med = r[r.size() / 2];
        front = 0;
        for (int k : B.idx)
            if (std::fabs(spheres[k].radius) >= 4 * med) ++front;
        front = std::min(front, 8);
    }
    if (front > 0 && !B.idx.empty()) {
        // the `front` largest spheres (ties: input order) leave the tree: every ray tests
        // them first (all lanes together), so a ray that hits one starts the traversal
        // with a short t_max and the tree's boxes are those of the small spheres only
        std::vector<int> by_r = B.idx;
        std::stable_sort(by_r.begin(), by_r.end(),
                         [&](int a, int b) { return std::fabs(spheres[a].radius) > std::fabs(spheres[b].radius); });
        by_r.resize(std::min<size_t>((size_t)front, by_r.size()));
        for (int k : by_r) out.order.push_back(k);
        out.front = (int)by_r.size();
        std::vector<int> rest;
        for (int k : B.idx)
            if (std::find(by_r.begin(), by_r.end(), k) == by_r.end()) rest.push_back(k);
        B.idx.swap(rest);
    }
    const int nb = (int)B.idx.size();
    if (nb + out.front > MAX_LEAF_FIRST) {
        err = "LDS-resident BVH holds at most " + std::to_string(MAX_LEAF_FIRST) + " spheres";
        return false;
    }
    if (nb > 0) {
        Box root;
        uint32_t r = B.build(0, nb, 1, root);
        if (r & REF_LEAF) {
            // single-leaf scene: a root with the leaf as BOTH children, so that the node
            // step needs no empty-child test.  The second visit cannot change the hit: it
            // recomputes the same roots, and only a root strictly below tmax (= the closest
            // root found by the first visit) would count.
            Node nd{};
            Box rb = root;
            to_float_box(rb, nd.lo0, nd.hi0);
            to_float_box(rb, nd.lo1, nd.hi1);
            nd.ref0 = nd.ref1 = r;
            out.nodes.push_back(nd);
            B.max_depth = 1;
        }
    }
    out.depth = B.max_depth;
    if ((int)out.nodes.size() > MAX_INNER) {
        err = "BVH has more than 32768 inner nodes";
        return false;
    }
    if (out.depth > STACK_MAX) {
        err = "BVH deeper than the LDS stack (" + std::to_string(STACK_MAX) + ")";
        return false;
    }
    return true;
}

// ---- uniform sphere grid (TRAV_GRID) ------------------------------------------------
// Cells of about 1 / density spheres each over the swept boxes' union; an axis thinner than
// a cell gets one cell (main.cpp's field is 22 x 0.9 x 22: a 29 x 1 x 29 grid at the default
// density 2, 23 x 1 x 23 at 1).
// Each box is padded by ~1e-4 of the grid's extent (plus 2^-16 of its largest coordinate)
// before it is listed, so that a sphere whose surface is reached within the fp32 rounding
// of a cell boundary -- the kernel's cell stepping and its stop test compare fp32 plane
// distances -- is listed in the cells on both sides of it.
bool build_sphere_grid(const SphereF* sph, int first, int n, double density, int slabs, int rec_bytes,
                       GridHdr& hdr, std::vector<unsigned char>& out) {
    out.clear();
    const int m = n - first;
    if (m <= 0 || !(density > 0) || slabs < 1 || slabs > GRID_SLAB_MAX) return false;
    const size_t slab_bytes = (size_t)(slabs + 1) * 24;
    std::vector<double> blo((size_t)m * 3), bhi((size_t)m * 3);
    double lo[3], hi[3];
    for (int a = 0; a < 3; ++a) {
        lo[a] = std::numeric_limits<double>::infinity();
        hi[a] = -std::numeric_limits<double>::infinity();
    }
    for (int k = 0; k < m; ++k) {
        const SphereF& q = sph[first + k];
        const double r = std::fabs((double)q.r);
        for (int a = 0; a < 3; ++a) {
            const double c0 = q.c[a], c1 = (double)q.c[a] + (double)q.cv[a];
            blo[(size_t)k * 3 + a] = std::min(c0, c1) - r;
            bhi[(size_t)k * 3 + a] = std::max(c0, c1) + r;
            lo[a] = std::min(lo[a], blo[(size_t)k * 3 + a]);
            hi[a] = std::max(hi[a], bhi[(size_t)k * 3 + a]);
        }
    }
    double ext = 0.0, span = 0.0;
    for (int a = 0; a < 3; ++a) {
        ext = std::max({ext, std::fabs(lo[a]), std::fabs(hi[a])});
        span = std::max(span, hi[a] - lo[a]);
    }
    if (!std::isfinite(ext) || !(span > 0)) return false;
    const double pad = 1e-4 * span + std::ldexp(ext, -16);
    double E[3];
    for (int a = 0; a < 3; ++a) {
        lo[a] -= pad;
        hi[a] += pad;
        E[a] = hi[a] - lo[a];
    }
    // cell edge for `density` cells per sphere over the box's volume (thin axes: one cell)
    double cell = std::cbrt(E[0] * E[1] * E[2] / (density * m));
    int res[3];
    size_t ncell = 0, nid = 0, bytes = 0;
    std::vector<uint32_t> cnt;
    auto word_of = [&](int x, int y, int z) { return ((size_t)z * res[1] + (size_t)y) * res[0] + (size_t)x; };
    // (an attempt stops counting once the lists pass 4 entries per sphere, where the grid is
    // refused anyway: a few large spheres over many small cells cost no more than that)
    const size_t max_ids = (size_t)4 * m;
    bool over = true;
    for (int attempt = 0; attempt < 64 && over; ++attempt) {
        ncell = 1;
        for (int a = 0; a < 3; ++a) {
            res[a] = (int)std::max(1.0, std::min(1024.0, std::round(E[a] / cell)));
            ncell *= (size_t)res[a];
        }
        cnt.assign(ncell, 0u);
        nid = 0;
        over = false;
        for (int k = 0; k < m && !over; ++k) {
            int c0[3], c1[3];
            size_t span_k = 1;
            for (int a = 0; a < 3; ++a) {
                const double s = res[a] / E[a];
                c0[a] = std::max(0, std::min(res[a] - 1, (int)std::floor((blo[(size_t)k * 3 + a] - pad - lo[a]) * s)));
                c1[a] = std::max(0, std::min(res[a] - 1, (int)std::floor((bhi[(size_t)k * 3 + a] + pad - lo[a]) * s)));
                span_k *= (size_t)(c1[a] - c0[a] + 1);
            }
            if (nid + span_k > max_ids) {
                over = true;
                break;
            }
            for (int z = c0[2]; z <= c1[2]; ++z)
                for (int y = c0[1]; y <= c1[1]; ++y)
                    for (int x = c0[0]; x <= c1[0]; ++x) ++cnt[word_of(x, y, z)];
            nid += span_k;
        }
        bytes = (ncell + 2 * (size_t)res[0] * res[1]) * 4 + nid * 4;
        over = over || ((bytes + 15) & ~(size_t)15) + slab_bytes > GRID_MAX_BYTES;
        cell *= 1.26;   // (for the next attempt) half the cells
    }
    if (over) return false;
    size_t empty = 0;
    for (uint32_t c : cnt) {
        if (c > (uint32_t)GRID_CELL_MAX) return false;
        empty += c == 0;
    }
    // spheres in clusters (most cells empty): a ray would walk empty cells the tree's boxes
    // skip; cells of more than 8 spheres on average (a coarse grid forced by large spheres):
    // a ray would test them all -- the tree serves both (C3's field: 11 % of the cells
    // empty, 1.5 spheres per occupied cell)
    if (empty * 2 > ncell || nid > 8 * (ncell - empty)) return false;
    if ((size_t)n * (size_t)rec_bytes + GRID_MAX_BYTES + sizeof(Node) > 0xffffffffu) return false;
    // The walk's reach (GridHdr::far_o, r06).  The kernel's cell decisions are off by at most
    // ~(k + 12) 2^-24 (|o| + ext) along an axis after k steps -- the rounding of o and d to
    // fp32 and of 1/d, o/d, each plane distance, each of the k step additions, the stop test's
    // (float)tmax and the entry point, every term bounded by |o_a| + |P_a| with P on the grid
    // box -- so with k <= res[0] + res[1] + res[2] + 2 and a factor of 2 to spare, origins
    // within +-far_o keep the error below the listed boxes' padding.  The same bound keeps
    // 2^-24 (|o| + ext) under a sixteenth of a cell, so a step always moves its plane distance
    // (by at least 15/16 of a cell): the walk ends.  A grid that not even rays from near its own
    // box could walk is refused.
    const int max_steps = res[0] + res[1] + res[2] + 2;
    double cs_min = std::numeric_limits<double>::infinity();
    for (int a = 0; a < 3; ++a) cs_min = std::min(cs_min, E[a] / res[a]);
    const double gext = ext + pad;
    const double far_o = std::min(std::ldexp(pad, 23) / (max_steps + 16), std::ldexp(cs_min, 20)) - gext;
    if (!(far_o > 2 * gext)) return false;
    GridHdr g{};
    g.far_o = (float)std::min(far_o, 1e30);
    for (int a = 0; a < 3; ++a) {
        g.lo[a] = (float)lo[a];
        g.hi[a] = (float)hi[a];
        g.cs[a] = (float)(E[a] / res[a]);
        g.inv_cs[a] = (float)(res[a] / E[a]);
        g.res[a] = res[a];
    }
    g.n_cells = (uint32_t)ncell;
    const size_t slab_off = (bytes + 15) & ~(size_t)15;
    bytes = slab_off + slab_bytes;
    g.slab_off = (uint32_t)slab_off;
    g.slab_k = (float)slabs;
    g.n_slab = slabs;
    std::vector<uint32_t> words(ncell), fill(ncell);
    // list positions as byte offsets from the buffer's start (= LDS byte addresses: the
    // kernels copy the buffer to LDS address 0): the lists follow the leading pad layer, the
    // cells and the trailing pad layer (rt_scene.h GridHdr); GRID_MAX_BYTES keeps every
    // position below 2^GRID_POS_BITS
    const uint32_t base = (uint32_t)(ncell + 2 * (size_t)res[0] * res[1]);
    static_assert(GRID_MAX_BYTES <= GRID_POS_MASK, "grid list positions");
    uint32_t run = 0;
    for (size_t c = 0; c < ncell; ++c) {
        words[c] = ((base + run) * 4u) | (((base + run + cnt[c]) * 4u) << GRID_POS_BITS);
        fill[c] = run;
        run += cnt[c];
    }
    const size_t total = (bytes + sizeof(Node) - 1) / sizeof(Node) * sizeof(Node);   // where the records start
    std::vector<uint32_t> ids(nid);
    for (int k = 0; k < m; ++k) {
        int c0[3], c1[3];
        for (int a = 0; a < 3; ++a) {
            const double s = res[a] / E[a];
            c0[a] = std::max(0, std::min(res[a] - 1, (int)std::floor((blo[(size_t)k * 3 + a] - pad - lo[a]) * s)));
            c1[a] = std::max(0, std::min(res[a] - 1, (int)std::floor((bhi[(size_t)k * 3 + a] + pad - lo[a]) * s)));
        }
        for (int z = c0[2]; z <= c1[2]; ++z)
            for (int y = c0[1]; y <= c1[1]; ++y)
                for (int x = c0[0]; x <= c1[0]; ++x)
                    ids[fill[word_of(x, y, z)]++] = (uint32_t)(total + (size_t)(first + k) * (size_t)rec_bytes);
    }
    // (an empty x-y layer of cells on either side of the grid: a step past its first or last
    // layer -- only ever within the rounding of the exit, the ray's last -- reads an empty
    // cell, so the kernel needs no bounds test)
    const size_t layer = (size_t)res[0] * res[1];
    out.assign(total, 0);
    std::memcpy(out.data() + layer * 4, words.data(), ncell * 4);
    if (nid) std::memcpy(out.data() + (ncell + 2 * layer) * 4, ids.data(), nid * 4);
    // the time slabs' boxes: slab k spans the times [k, k + 1) / slabs, widened by a margin
    // far beyond the kernel's rounding of t * slabs, and each sphere's box over it is padded
    // as the listed boxes (so a slab box holds every surface point the exact ray can reach at
    // a time of that slab), then clipped to the grid box; the last box is the grid box;
    // stored as (lo, hi) pairs per axis (rt_scene.h GridHdr)
    float* sb = (float*)(out.data() + slab_off);
    for (int k = 0; k <= slabs; ++k) {
        double slo[3], shi[3];
        for (int a = 0; a < 3; ++a) {
            slo[a] = lo[a];
            shi[a] = hi[a];
        }
        if (k < slabs) {
            const double t0 = (double)k / slabs - 1.0 / (1024.0 * slabs), t1 = (double)(k + 1) / slabs + 1.0 / (1024.0 * slabs);
            for (int a = 0; a < 3; ++a) {
                slo[a] = std::numeric_limits<double>::infinity();
                shi[a] = -std::numeric_limits<double>::infinity();
            }
            for (int q = 0; q < m; ++q) {
                const SphereF& s = sph[first + q];
                const double r = std::fabs((double)s.r);
                for (int a = 0; a < 3; ++a) {
                    const double c0 = (double)s.c[a] + t0 * (double)s.cv[a], c1 = (double)s.c[a] + t1 * (double)s.cv[a];
                    slo[a] = std::min(slo[a], std::min(c0, c1) - r);
                    shi[a] = std::max(shi[a], std::max(c0, c1) + r);
                }
            }
            for (int a = 0; a < 3; ++a) {
                slo[a] = std::max(slo[a] - pad, lo[a]);
                shi[a] = std::min(shi[a] + pad, hi[a]);
            }
        }
        for (int a = 0; a < 3; ++a) {   // (lo, hi) pairs per axis
            sb[((size_t)a * (slabs + 1) + k) * 2] = (float)slo[a];
            sb[((size_t)a * (slabs + 1) + k) * 2 + 1] = (float)shi[a];
        }
    }
    hdr = g;
    return true;
}

}  // namespace rtx

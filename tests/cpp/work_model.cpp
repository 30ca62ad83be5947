// Algorithmic work per primary ray ("re-derive with the same probe method
// once the mesh fixture is fixed"): the reference's path logic (the oracle's ray_color,
// scatter and counter RNG, oracle/rt_oracle.c) with world.hit answered by BVH traversals
// over the product's own host-built trees (csrc/rt_bvh.cpp: the SAH sphere tree and the
// 4-wide triangle tree with its default parameters), counting what a traversal must touch:
// node visits, box tests, sphere and triangle tests, world.hit calls and hits.  Test
// infrastructure (it links the oracle): tests/work_model.py drives it and writes the
// constants bench.py carries (raytracingproject_amd/measure.py).
//
// Traversal (both trees): nearest child first, the others pushed far-first with their
// entry distance; a popped entry whose box starts beyond the closest hit so far is dropped
// without a visit (the order the kernels use; rt_device.h closest_hit).  Box tests are the
// slab test in fp64 on the trees' fp32 boxes (outward-rounded and padded by the builder, so
// no primitive the exact ray hits is culled).  Big spheres (R >= 64, the ground) are tested
// by every ray before the tree, as in the kernels; the front list is not used (front = 0):
// every other sphere is in the tree.
//
//   work_model SPHERES MATERIALS TRIANGLES WIDTH NPIX SPP SEED [--frame OUT]
//     *.bin: rt_sphere / rt_material / rt_triangle records (TRIANGLES may be an empty file);
//     NPIX pixels drawn uniformly (a fixed LCG over the WIDTH x height frame of main.cpp's
//     camera) x SPP samples each (sample indices 0..SPP-1), counter RNG keyed by SEED.
//     Prints one JSON object of per-primary averages.  --frame OUT instead renders every
//     pixel at SPP and writes the fp64 sums (H*W*3 doubles) -- the probe's paths checked
//     against the linear-scan oracle by tests/test_work_model.py.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../oracle/rt_oracle.h"
#include "../../raytracingproject_amd/csrc/rt_bvh.h"

using namespace rtx;

namespace {

struct Counts {
    uint64_t sph_visits = 0, sph_boxes = 0, sph_tests = 0;
    uint64_t mesh_visits = 0, mesh_boxes = 0, tri_tests = 0;
    uint64_t calls = 0, sphere_hits = 0, tri_hits = 0, both = 0;   // both: a sphere found, then a nearer triangle
};

struct World {
    bool last_sphere = false;   // this world.hit call's sphere query found one
    std::vector<orc_sphere> os;
    std::vector<orc_triangle> ot;
    BuiltBvh sb;
    MeshBvh mb;
    Counts c;
};

// slab test of one fp32 box: entry distance in (tmin, tmax], or false
bool box(const float lo[3], const float hi[3], const double o[3], const double inv[3], double tmin, double tmax,
         double& tn) {
    double t0 = tmin, t1 = tmax;
    for (int a = 0; a < 3; ++a) {
        double a0 = ((double)lo[a] - o[a]) * inv[a], a1 = ((double)hi[a] - o[a]) * inv[a];
        if (std::isnan(a0)) a0 = -INFINITY;   // d = 0 with o on the plane: the slab is no constraint
        if (std::isnan(a1)) a1 = INFINITY;
        if (a0 > a1) std::swap(a0, a1);
        t0 = a0 > t0 ? a0 : t0;
        t1 = a1 < t1 ? a1 : t1;
    }
    tn = t0;
    return t0 <= t1;
}

int sphere_query(void* ctx, const double o[3], const double d[3], double tm, double tmin, double tmax) {
    World& w = *(World*)ctx;
    w.c.calls++;
    int best = -1;
    double closest = tmax, t;
    for (int k : w.sb.big) {
        w.c.sph_tests++;
        if (orc_sphere_root(&w.os[k], o, d, tm, tmin, closest, &t)) closest = t, best = k;
    }
    if (!w.sb.nodes.empty()) {
        const double inv[3] = {1.0 / d[0], 1.0 / d[1], 1.0 / d[2]};
        struct E { uint32_t ref; double tn; };
        E stack[64];
        int sp = 0;
        stack[sp++] = {0, tmin};
        while (sp > 0) {
            const E e = stack[--sp];
            if (e.tn > closest) continue;   // culled: its box starts beyond the closest hit
            if (e.ref & REF_LEAF) {
                const int first = (int)(e.ref & 0x7ffu), count = (int)((e.ref >> 11) & 0xfu) + 1;
                for (int k = first; k < first + count; ++k) {
                    w.c.sph_tests++;
                    const int s = w.sb.order[k];
                    if (orc_sphere_root(&w.os[s], o, d, tm, tmin, closest, &t)) closest = t, best = s;
                }
                continue;
            }
            const Node& n = w.sb.nodes[e.ref];
            w.c.sph_visits++;
            w.c.sph_boxes += 2;
            double t0, t1;
            const bool h0 = box(n.lo0, n.hi0, o, inv, tmin, closest, t0);
            const bool h1 = box(n.lo1, n.hi1, o, inv, tmin, closest, t1);
            if (h0 && h1) {
                const bool first0 = t0 <= t1;
                stack[sp++] = first0 ? E{n.ref1, t1} : E{n.ref0, t0};
                stack[sp++] = first0 ? E{n.ref0, t0} : E{n.ref1, t1};
            } else if (h0) {
                stack[sp++] = {n.ref0, t0};
            } else if (h1) {
                stack[sp++] = {n.ref1, t1};
            }
        }
    }
    if (best >= 0) w.c.sphere_hits++;
    w.last_sphere = best >= 0;
    return best;
}

int tri_query(void* ctx, const double o[3], const double d[3], double tmin, double tmax) {
    World& w = *(World*)ctx;
    if (w.mb.nodes4.empty()) return -1;
    const double inv[3] = {1.0 / d[0], 1.0 / d[1], 1.0 / d[2]};
    struct E { uint32_t ref; double tn; };
    E stack[3 * MESH_STACK_MAX];
    int sp = 0;
    stack[sp++] = {0, tmin};
    int best = -1;
    double closest = tmax, t;
    while (sp > 0) {
        const E e = stack[--sp];
        if (e.tn > closest) continue;
        if (e.ref & MREF_LEAF) {
            const int first = (int)(e.ref & 0xffffffu), count = (int)((e.ref >> 24) & 0x7fu) + 1;
            for (int k = first; k < first + count; ++k) {
                w.c.tri_tests++;
                const int tr = w.mb.order[k];
                if (orc_tri_root(&w.ot[tr], o, d, tmin, closest, &t)) closest = t, best = tr;
            }
            continue;
        }
        const Node4& n = w.mb.nodes4[e.ref];
        w.c.mesh_visits++;
        E hit[4];
        int nh = 0;
        for (int c = 0; c < 4; ++c) {
            if (n.ref[c] == MREF_EMPTY) continue;
            w.c.mesh_boxes++;
            const float lo[3] = {n.lox[c], n.loy[c], n.loz[c]}, hi[3] = {n.hix[c], n.hiy[c], n.hiz[c]};
            double tn;
            if (box(lo, hi, o, inv, tmin, closest, tn)) hit[nh++] = {n.ref[c], tn};
        }
        // far first onto the stack, so the nearest is popped next
        for (int a = 1; a < nh; ++a)
            for (int b = a; b > 0 && hit[b].tn > hit[b - 1].tn; --b) std::swap(hit[b], hit[b - 1]);
        for (int a = 0; a < nh; ++a) stack[sp++] = hit[a];
    }
    if (best >= 0) w.c.tri_hits++;
    if (best >= 0 && w.last_sphere) w.c.both++;
    return best;
}

template <class T>
std::vector<T> read_records(const char* path) {
    std::vector<T> v;
    FILE* f = std::fopen(path, "rb");
    if (!f) return v;
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    v.resize((size_t)n / sizeof(T));
    if (!v.empty() && std::fread(v.data(), sizeof(T), v.size(), f) != v.size()) v.clear();
    std::fclose(f);
    return v;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 8) {
        std::fprintf(stderr, "usage: work_model SPHERES MATERIALS TRIANGLES WIDTH NPIX SPP SEED [--frame OUT]\n");
        return 2;
    }
    const auto S = read_records<rt_sphere>(argv[1]);
    const auto M = read_records<rt_material>(argv[2]);
    const auto T = read_records<rt_triangle>(argv[3]);
    const int width = std::atoi(argv[4]), npix = std::atoi(argv[5]), spp = std::atoi(argv[6]);
    const uint64_t seed = std::strtoull(argv[7], nullptr, 0);
    const char* frame_out = argc >= 10 && std::string(argv[8]) == "--frame" ? argv[9] : nullptr;

    World w;
    // the oracle's records (one material per sphere in the oracle: index into M)
    std::vector<orc_material> om(M.size());
    for (size_t k = 0; k < M.size(); ++k) {
        om[k].type = M[k].type;
        om[k].pad = 0;
        for (int a = 0; a < 3; ++a) om[k].albedo[a] = M[k].albedo[a];
        om[k].fuzz = M[k].fuzz < 1 ? M[k].fuzz : 1;   // material.h:33
        om[k].ir = M[k].ir;
    }
    w.os.resize(S.size());
    for (size_t k = 0; k < S.size(); ++k) {
        for (int a = 0; a < 3; ++a) w.os[k].center[a] = S[k].center[a], w.os[k].center_vec[a] = S[k].center_vec[a];
        w.os[k].radius = S[k].radius;
        w.os[k].moving = S[k].moving;
        w.os[k].mat = S[k].mat;
    }
    w.ot.resize(T.size());
    for (size_t k = 0; k < T.size(); ++k) {
        for (int a = 0; a < 3; ++a)
            w.ot[k].v0[a] = T[k].v0[a], w.ot[k].v1[a] = T[k].v1[a], w.ot[k].v2[a] = T[k].v2[a];
        w.ot[k].mat = T[k].mat;
        w.ot[k].pad = 0;
    }
    // the product's trees with its default parameters (rt_ctx.h tuning: max_leaf 6,
    // cost_traverse 1, cost_intersect 0.25; mesh_max_leaf 2, mesh_cost_traverse 2)
    std::string err;
    BvhParams bp;
    bp.max_leaf = 6;
    bp.cost_traverse = 1.0;
    bp.cost_intersect = 0.25;
    bp.front = 0;
#ifndef WM_MESH_LEAF
#define WM_MESH_LEAF 2
#endif
    if (!build_bvh(S.data(), (int)S.size(), bp, w.sb, err) ||
        !build_mesh_bvh(T.data(), (int)T.size(), WM_MESH_LEAF, 2.0, w.mb, err)) {
        std::fprintf(stderr, "build: %s\n", err.c_str());
        return 1;
    }
#ifdef WM_QUANT_BITS
    // design probe: child boxes quantised to WM_QUANT_BITS-bit steps of a power-of-two
    // grid over the node's own box (rounded outwards), the compressed-node layout's loss
    // in culling (more node visits and triangle tests), not a product format
    for (Node4& n : w.mb.nodes4) {
        float* lo[3] = {n.lox, n.loy, n.loz};
        float* hi[3] = {n.hix, n.hiy, n.hiz};
        for (int a = 0; a < 3; ++a) {
            double plo = INFINITY, phi = -INFINITY;
            for (int c = 0; c < 4; ++c)
                if (n.ref[c] != MREF_EMPTY) plo = std::min(plo, (double)lo[a][c]), phi = std::max(phi, (double)hi[a][c]);
            if (!(phi > plo)) continue;
            const double steps = (double)((1 << WM_QUANT_BITS) - 1);
            const double s = std::ldexp(1.0, (int)std::ceil(std::log2((phi - plo) / steps)));
            for (int c = 0; c < 4; ++c) {
                if (n.ref[c] == MREF_EMPTY) continue;
                const double ql = std::floor(((double)lo[a][c] - plo) / s), qh = std::ceil(((double)hi[a][c] - plo) / s);
                lo[a][c] = std::nextafter((float)(plo + ql * s), -INFINITY);
                hi[a][c] = std::nextafter((float)(plo + qh * s), INFINITY);
            }
        }
    }
#endif
    orc_set_mesh(w.ot.data(), (int)w.ot.size());
    orc_accel acc = {sphere_query, tri_query, &w};
    orc_set_accel(&acc);

    orc_camera cam;
    orc_camera_defaults(&cam);
    cam.image_width = width;
    cam.samples_per_pixel = spp;
    orc_camera_initialize(&cam);
    const int W = cam.image_width, H = cam.image_height;
    std::vector<int32_t> pix;
    if (frame_out) {
        for (int j = 0; j < H; ++j)
            for (int i = 0; i < W; ++i) pix.push_back(i), pix.push_back(j);
    } else {
        uint64_t x = 0x9E3779B97F4A7C15ull ^ seed;
        for (int k = 0; k < npix; ++k) {
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            const uint64_t p = (x >> 17) % ((uint64_t)W * H);
            pix.push_back((int32_t)(p % W));
            pix.push_back((int32_t)(p / W));
        }
    }
    const int n = (int)pix.size() / 2;
    std::vector<double> sums((size_t)n * 3);
    std::vector<uint64_t> segs(n);
    orc_render_counter(w.os.data(), om.data(), (int)w.os.size(), &cam, seed, pix.data(), n, sums.data(), nullptr,
                       segs.data());
    orc_set_accel(nullptr);
    orc_set_mesh(nullptr, 0);
    if (frame_out) {
        FILE* f = std::fopen(frame_out, "wb");
        std::fwrite(sums.data(), sizeof(double), sums.size(), f);
        std::fclose(f);
    }
    uint64_t seg = 0;
    for (uint64_t s : segs) seg += s;
    const double P = (double)n * spp;
    const Counts& c = w.c;
    std::printf(
        "{\"primary_rays\": %.0f, \"width\": %d, \"height\": %d, \"segments\": %.6f, \"hits\": %.6f, "
        "\"sphere_hits\": %.6f, \"triangle_hits\": %.6f, \"sphere_node_visits\": %.6f, \"sphere_box_tests\": %.6f, "
        "\"sphere_tests\": %.6f, \"mesh_node_visits\": %.6f, \"mesh_box_tests\": %.6f, \"triangle_tests\": %.6f, "
        "\"world_hit_calls_check\": %.6f, \"sphere_nodes\": %zu, \"mesh_nodes\": %zu, \"triangles\": %zu}\n",
        P, W, H, seg / P, (double)(c.sphere_hits + c.tri_hits - c.both) / P, (double)(c.sphere_hits - c.both) / P,
        c.tri_hits / P,
        c.sph_visits / P, c.sph_boxes / P, c.sph_tests / P, c.mesh_visits / P, c.mesh_boxes / P, c.tri_tests / P,
        c.calls / P, w.sb.nodes.size(), w.mb.nodes4.size(), T.size());
    return 0;
}

// rt_abi.cpp -- implementation of the C ABI declared in include/rt_hip.h.
//
// Host-side responsibilities: validate arguments, build the BVH (rt_bvh.cpp), lay the
// scene out for the LDS-resident kernel, own device memory and the stream, launch the
// kernels (rt_render_f32.hip / rt_render_f64.hip) and time them with HIP events on the
// stream they run on.  Every failure is reported as a negative status + message; there
// is no CPU fallback anywhere in this library.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdarg>
#include <limits>
#include <map>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rt_hip.h"
#include "rt_bvh.h"
#include "rt_device.h"
#include "rt_launch.h"
#include "rt_lbvh.h"
#include "rt_ctx.h"

using namespace rtx;
using namespace rtx_abi;


namespace {

void free_scene(rt_ctx* c) {
    (void)hipFree(c->d_nodes);
    (void)hipFree(c->d_sph);
    (void)hipFree(c->d_mat);
    (void)hipFree(c->d_big);
    (void)hipFree(c->d_bigf);
    c->d_bigf = nullptr;
    (void)hipFree(c->d_mnodes);
    (void)hipFree(c->d_tris);
    (void)hipFree(c->d_tmeta);
    (void)hipFree(c->d_remap);
    c->d_remap = nullptr;
    (void)hipFree(c->d_grid);
    c->d_grid = nullptr;
    c->grid_nodes = c->grid_entries = 0;
    c->d_mnodes = nullptr;
    c->d_tris = nullptr;
    c->d_tmeta = nullptr;
    c->n_mnodes = c->n_tris = c->mdepth = c->mleaves = 0;
    c->d_nodes = nullptr;
    c->d_sph = c->d_mat = nullptr;
    c->d_big = nullptr;
    c->has_scene = false;
}

size_t elem_bytes(const rt_ctx* c) { return c->precision == RT_PREC_F64 ? 8 : 4; }

// LDS traversal-stack entries per lane.  A far child is pushed only at an inner node with
// both children hit, and each pending one belongs to a distinct ancestor of the node being
// visited, so at most `depth` (inner levels) are pending; the latest sits in a register
// (closest_hit's `top`), the rest in LDS.
int stack_entries(const rt_ctx* c) { return c->depth > 1 ? c->depth - 1 : 1; }

// The fp64 kernel (rt_tuning.f64_kernel; 0 = the measured best, rt_render_f64.hip)
// fp64 kernel: the tuning's, or (0) kernel 5 -- 4 over the sphere grid -- where the scene has
// a grid and the traversal flags ask for it, else 4; 5 without a grid runs as 4 (the same
// frame: the grid only picks which spheres are tested)
// (6, internal: kernel 5 with the flat walk, where the grid is one cell tall in y)
constexpr int F64_KERNEL_DEFAULT = 4, F64_KERNEL_GRID = 5, F64_KERNEL_GRID_FLAT = 6;
// the sphere grid serves the current launch: built, and every ray the launch can start lies
// within its walk's reach (grid_reach_ok; otherwise the tree, the same frame)
bool grid_usable(const rt_ctx* c) { return c->grid_nodes > 0 && !c->grid_blocked; }
// ...and is one cell tall in y, so that its walk steps in x and z only (TRAV_GFLAT, r06),
// unless the tuning keeps the 3-D walk (TRAV_G3D)
bool grid_flat(const rt_ctx* c) {
    return grid_usable(c) && c->grid_hdr.res[1] == 1 && !(c->tuning.traversal & TRAV_G3D);
}
int f64_kernel_of(const rt_ctx* c) {
    const int k = c->tuning.f64_kernel > 0 ? c->tuning.f64_kernel
                  : (c->tuning.traversal & TRAV_GRID) ? F64_KERNEL_GRID : F64_KERNEL_DEFAULT;
    if (k != F64_KERNEL_GRID) return k;
    return !grid_usable(c) ? F64_KERNEL_DEFAULT : grid_flat(c) ? F64_KERNEL_GRID_FLAT : k;
}

// The sphere grid's walk is exact and ends only for ray origins within +-GridHdr::far_o
// (rt_bvh.cpp build_sphere_grid); the kernel has no check for it (any such code in the walk
// cost C3 1.4 .. 9 %, r06), so each launch checks here, on the host, that no ray it can
// produce starts beyond it -- else it renders with the tree.  Rays start at the camera (its
// centre, within the defocus disk) or at hit points: on the geometry a ray can reach anywhere
// (reach_lo / reach_hi: small spheres swept over the shutter, triangles, big spheres that
// refract or move), or on a static opaque big sphere B, which a ray from O reaches only
// within the tangent distance sqrt(|O - C|^2 - R^2) of O (a point of B seen from O), and
// whose surface starts no ray that meets B again.  Hit regions on the big spheres are grown
// from each other to a fixed point (a ground sphere alone: one step).  The margin covers the
// fp32 rounding of hit points.
bool grid_reach_ok(const rt_ctx* c, const rt_camera* cam) {
    if (c->grid_nodes == 0) return true;
    using Box = std::array<double, 6>;
    auto empty = []() {
        const double inf = std::numeric_limits<double>::infinity();
        return Box{inf, inf, inf, -inf, -inf, -inf};
    };
    auto join = [](Box& a, const Box& b) {
        for (int k = 0; k < 3; ++k) {
            a[k] = std::min(a[k], b[k]);
            a[3 + k] = std::max(a[3 + k], b[3 + k]);
        }
    };
    Box u0 = empty();
    for (int k = 0; k < 3; ++k) {
        const double r = cam->defocus_angle > 0 ? std::fabs(cam->defocus_disk_u[k]) + std::fabs(cam->defocus_disk_v[k]) : 0;
        u0[k] = std::min(c->reach_lo[k], cam->center[k] - r);
        u0[3 + k] = std::max(c->reach_hi[k], cam->center[k] + r);
    }
    const size_t nb = c->reach_big.size();
    std::vector<Box> hit(nb, empty());
    bool changed = true;
    for (int it = 0; it < 16 && changed; ++it) {
        changed = false;
        for (size_t j = 0; j < nb; ++j) {
            Box from = u0;   // where a ray that meets B_j can start: anywhere but on B_j
            for (size_t k = 0; k < nb; ++k)
                if (k != j) join(from, hit[k]);
            const auto& b = c->reach_big[j];
            double d2 = 0, d2n = 0;   // the farthest corner of `from` from B_j's centre, and its nearest point
            for (int k = 0; k < 3; ++k) {
                const double e = std::max(std::fabs(from[k] - b[k]), std::fabs(from[3 + k] - b[k]));
                const double n = std::max({from[k] - b[k], b[k] - from[3 + k], 0.0});
                d2 += e * e;
                d2n += n * n;
            }
            // (a ray could start inside B_j -- geometry embedded in it, or a box too loose to
            // tell: then all of B_j)
            const double t = d2n < b[3] * b[3] ? std::numeric_limits<double>::infinity()
                                               : std::sqrt(std::max(d2 - b[3] * b[3], 0.0));
            Box h;
            for (int k = 0; k < 3; ++k) {
                h[k] = std::max(from[k] - t, b[k] - b[3]);
                h[3 + k] = std::min(from[3 + k] + t, b[k] + b[3]);
            }
            if (!(h[0] <= h[3] && h[1] <= h[4] && h[2] <= h[5])) continue;
            Box g = hit[j];
            join(g, h);
            if (g != hit[j]) {
                hit[j] = g;
                changed = true;
            }
        }
    }
    if (changed) return false;   // (no fixed point within 16 rounds: the tree)
    Box all = u0;
    for (const Box& h : hit) join(all, h);
    double m = 0;
    for (int k = 0; k < 6; ++k) m = std::max(m, std::fabs(all[k]));
    return m * (1.0 + 0x1p-10) <= (double)c->grid_hdr.far_o;   // (false for NaN)
}

// LDS of the sphere scene copy and the traversal stacks of one workgroup (kernel flags tr:
// TRAV_GRID kernels hold the grid where the tree's nodes go, and no traversal stack).
size_t lds_scene_bytes_at(const rt_ctx* c, int block, int tr = 0) {
    const bool grid = (tr & TRAV_GRID) != 0;
    const size_t sph = c->precision == RT_PREC_F64 ? sizeof(SphereD) : sizeof(SphereF);
    const size_t mat = c->precision == RT_PREC_F64 ? sizeof(MatD) : sizeof(MatF);
    const size_t stack = grid ? 0 : (size_t)block * (size_t)stack_entries(c) * 2;
    return (size_t)(grid ? c->grid_nodes : c->n_nodes) * sizeof(Node) + (size_t)c->n_sph * sph +
           (size_t)c->n_mat * mat + (size_t)c->n_big * (sizeof(SphereD) + sizeof(BigF)) + ((stack + 15) & ~(size_t)15);
}

// The render launch's view of the sphere scene for kernel flags tr: the grid in the nodes'
// place (RenderParams::nodes / n_nodes), no traversal stack.
void apply_grid(const rt_ctx* c, int tr, RenderParams& P) {
    if (!(tr & TRAV_GRID)) return;
    P.nodes = (const Node*)c->d_grid;
    P.n_nodes = c->grid_nodes;
    P.stack_size = 0;
    P.grid = c->grid_hdr;
}

// LDS of the sphere part of one workgroup at (block, kernel flags tr): the scene copy and
// stacks, plus the coherent kernel's per-wave FIFO (+ item sums) and constants block.
size_t lds_sphere_bytes_bt(const rt_ctx* c, int block, int tr) {
    const bool f32 = c->precision == RT_PREC_F32;
    const size_t nw = (size_t)(block / 64);
    const size_t coh = c->n_mnodes > 0 || !(tr & TRAV_COH)
                           ? 0
                           : nw * coh_wave_bytes(false, (tr & TRAV_NOSUM) == 0, coh_fifo_entries(tr), !f32) + COH_CAM_BYTES;
    return lds_scene_bytes_at(c, block, tr) + coh;
}

// LDS of a mesh scene's per-lane state beyond the sphere part, with `s` mesh traversal
// stack entries per lane in LDS (the rest in scratch).  fp32 mesh kernels also keep each
// lane's three item sums (floats) in LDS; the coherent kernel (fp32) puts its per-wave FIFO
// + item sums and the CohConst block there instead.
size_t lds_mesh_bytes_at(const rt_ctx* c, int block, int tr, int s) {
    if (c->n_mnodes == 0) return 0;
    const size_t stack = (size_t)block * (size_t)s * 4;
    const bool f64 = c->precision != RT_PREC_F32;
    if (tr & TRAV_COH)
        return stack +
               (size_t)(block / 64) *
                   coh_wave_bytes(true, (tr & TRAV_NOSUM) == 0, coh_fifo_entries(tr), f64, coh_parks(true, tr, f64)) +
               COH_CAM_BYTES;
    if (f64) return stack;
    return stack + (size_t)block * 3 * sizeof(float);
}

// VGPRs of an instantiated render kernel.  The plan weighs every candidate kernel, LDS
// stack depth and sum / no-sum choice on each call, several calls per render, and a kernel's
// register count never changes within a process: each is asked of HIP once (failed queries
// are not kept).
int kernel_vgprs(bool f64, bool mesh, int block, int wpe, int tr, int f64k) {
    static std::mutex mu;
    static std::map<std::array<int, 6>, int> known;
    const std::array<int, 6> key = f64 ? std::array<int, 6>{1, mesh, 0, 0, 0, f64k}
                                       : std::array<int, 6>{0, mesh, block, wpe, tr, 0};
    {
        std::lock_guard<std::mutex> g(mu);
        const auto it = known.find(key);
        if (it != known.end()) return it->second;
    }
    const int v = f64 ? render_f64_vgprs(mesh, f64k) : render_f32_vgprs(block, wpe, tr, mesh);
    if (v > 0) {
        std::lock_guard<std::mutex> g(mu);
        known[key] = v;
    }
    return v;
}

// Workgroups of the render kernel (block, traversal tr, waves_per_eu key wpe) that the
// register file lets share a CU (LDS aside): 512 VGPRs per SIMD lane, 8-register granules,
// at most 8 waves per SIMD, 4 SIMDs.
int wgs_per_cu_bt(const rt_ctx* c, int block, int tr, int wpe) {
    const bool mesh = c->n_mnodes > 0;
    const int v = kernel_vgprs(c->precision == RT_PREC_F64, mesh, block, wpe, tr, f64_kernel_of(c));
    int waves = v > 0 ? 512 / ((v + 7) & ~7) : 8;
    if (waves > 8) waves = 8;
    const int wgs = waves * 4 / (block / 64);
    return wgs > 0 ? wgs : 1;
}

// Workgroups per CU by registers and by the LDS a workgroup needs with s mesh stack
// entries per lane in LDS.
int occupancy_at(const rt_ctx* c, int block, int tr, int wpe, int s) {
    const int reg = wgs_per_cu_bt(c, block, tr, wpe);
    const size_t need = lds_sphere_bytes_bt(c, block, tr) + lds_mesh_bytes_at(c, block, tr, s);
    const int lds = need > 0 ? (int)(160 * 1024 / need) : 64;
    return reg < lds ? reg : lds;
}

// Mesh traversal stack entries per lane kept in LDS: the tuning's mesh_lds_stack, or (-1,
// the default) the most entries up to MESH_LDS_STACK_AUTO that cost no workgroup per CU.
// A mesh-only scene keeps all 12 at six 256-thread workgroups; the mixed scene's 512-thread
// workgroups carry the sphere scene as well and reach 3 per CU (6 waves per SIMD with the
// 6-wave kernel) only with the whole mesh stack in scratch: C5 geometry at 4K @ 32 takes
// 55.6 ms that way against 63.0 ms with 12 LDS entries at 2 per CU (r04f mw6c5).
constexpr int MESH_LDS_STACK_AUTO = 12;
// r06: none for the mixed-scene kernels over the sphere grid -- the C5 geometry at 4K @ 1024
// ran 1,525.6-1,528.5 ms with the whole mesh stack in scratch against 1,567.5-1,569.1 with the
// 5 LDS entries that cost no workgroup (2 entries: 1,565.4-1,566.8), frames identical, though
// its traffic per launch rises 32.6 -> 38.3 GB at 4K @ 32 (profiles/r06/r06h, r06i, r06j);
// mesh-only C4 keeps its 12 (none: +9 %).
int mesh_stack_bt(const rt_ctx* c, int block, int tr, int wpe) {
    if (c->n_mnodes == 0) return 0;
    if (c->tuning.mesh_lds_stack >= 0) return c->tuning.mesh_lds_stack;
    if (tr & TRAV_GRID) return 0;
    const int most = occupancy_at(c, block, tr, wpe, 0);
    for (int s = MESH_LDS_STACK_AUTO; s > 0; --s)
        if (occupancy_at(c, block, tr, wpe, s) >= most) return s;
    return 0;
}

size_t lds_mesh_stack_bytes_bt(const rt_ctx* c, int block, int tr, int wpe) {
    return lds_mesh_bytes_at(c, block, tr, mesh_stack_bt(c, block, tr, wpe));
}

// Workgroups per CU at (block, tr, wpe) by registers and by the LDS a workgroup needs.
int occupancy_bt(const rt_ctx* c, int block, int tr, int wpe) {
    return occupancy_at(c, block, tr, wpe, mesh_stack_bt(c, block, tr, wpe));
}

// The kernel the context's scene runs: threads per workgroup, traversal flags and the
// register-budget key (waves_per_eu) of its instantiation.
//  * fp64: the block of the f64_kernel (the flags are not used);
//  * fp32 spheres: the tuning's block and waves_per_eu; the coherent kernel drops its LDS
//    pixel sums (TRAV_NOSUM) where they would cost a workgroup per CU;
//  * fp32 meshes: mesh_block, or (0 = auto) whichever of 256 / 512 / 768 keeps more waves
//    resident per CU, counting registers and LDS: a mesh-only scene fits six 256-thread
//    workgroups with the 6-wave kernel (24 waves) against three of 512; with the sphere
//    scene also in LDS the bigger workgroups win (bench_mesh_block_r01al.jsonl), and of
//    those the 768-thread ones keep the item sums and two LDS stack entries (r05).  At
//    each block the coherent kernel keeps its LDS item sums unless they cost occupancy,
//    and mesh_waves_per_eu -1 (the default) weighs the 6-wave kernels (<= 80 VGPRs) against
//    the compiler's budget (0, 5 waves per SIMD) the same way -- equal occupancy keeps the
//    unspilled one.  The 6-wave kernels measured C4 37.7-37.9 ms against 39.7-40.0 and C5
//    geometry (with the mesh stack in scratch, above) 55.6 against 63.0 ms, frames identical
//    (profiles/r04/mw6_ab_r04f.txt).
struct KernelPlan {
    int block, trav, wpe;
};
KernelPlan plan_of(const rt_ctx* c) {
    int t = c->tuning.traversal;
    if (c->precision != RT_PREC_F32 || c->n_mnodes == 0) t &= ~TRAV_MIFIF;   // fp32 mesh kernels only
    // the if-if mesh loop is added wherever it is instantiated unless the while-while loop
    // (TRAV_MWHILE, never part of a kernel key) is asked for
    const bool want_mifif = (t & TRAV_MIFIF) || !(t & TRAV_MWHILE);
    t &= ~(TRAV_MWHILE | TRAV_MIFIF | TRAV_GFLAT | TRAV_G3D);
    if (c->precision == RT_PREC_F64)
        return {render_f64_block(f64_kernel_of(c)), render_f64_trav(f64_kernel_of(c)), 0};
    // the sphere grid wherever the scene has one (build_sphere_grid): the fp32 sphere kernels,
    // the fp32 mixed-scene mesh kernels (74328 / 74456, candidates below) and, through
    // f64_kernel 5, fp64 (handled above); else the tree
    if (!grid_usable(c)) t &= ~TRAV_GRID;
    // the flat walk (TRAV_GFLAT) wherever the grid is one cell tall in y and its kernel exists
    const bool flat = grid_flat(c);
    auto gflat = [&](int b, int w, int x, bool mesh) {
        return flat && (x & TRAV_GRID) && render_f32_supported(b, w, x | TRAV_GFLAT, mesh) ? x | TRAV_GFLAT : x;
    };
    if (c->n_mnodes == 0) {
        const int b = c->tuning.block, w = c->tuning.waves_per_eu;
        if ((t & TRAV_COH) && !(t & TRAV_NOSUM)) {
            const size_t base = lds_scene_bytes_at(c, b, t), nw = (size_t)(b / 64);
            const int fifo = coh_fifo_entries(t);
            const size_t with = base + nw * coh_wave_bytes(false, true, fifo) + COH_CAM_BYTES,
                         without = base + nw * coh_wave_bytes(false, false, fifo) + COH_CAM_BYTES;
            // (occupancy counts registers too: a small scene whose sums only lower a
            // workgroup count the registers never reach keeps them)
            const int reg = wgs_per_cu_bt(c, b, t, w);
            if (std::min<size_t>(reg, 160 * 1024 / with) < std::min<size_t>(reg, 160 * 1024 / without))
                t |= TRAV_NOSUM;
        }
        return {b, gflat(b, w, t, false), w};
    }
    if (!(t & TRAV_COH)) t &= ~TRAV_NOSUM;
    const int wt = c->tuning.mesh_waves_per_eu;
    const int t0 = t;
    KernelPlan cand[12];
    int nc = 0;
    for (int b : {256, 512, 768}) {
        if (c->tuning.mesh_block > 0 && b != c->tuning.mesh_block) continue;
        // (an explicit budget alone; auto weighs the compiler's against the 6-wave kernels)
        const int ws[2] = {wt >= 0 ? wt : 0, 6};
        for (int wi = 0; wi < (wt >= 0 ? 1 : 2); ++wi)
        for (int gi = 0; gi < ((t & TRAV_GRID) ? 2 : 1); ++gi) {   // (the sphere grid, then the tree)
            const int w = ws[wi];
            const int t = gi ? t0 & ~TRAV_GRID : t0;
            // (the if-if loop where its kernel exists, decided before the LDS sums are weighed)
            auto mifif = [&](int x) {
                return want_mifif && render_f32_supported(b, w, x | TRAV_MIFIF, true) ? x | TRAV_MIFIF : x;
            };
            int tb = mifif(t);
            if ((t & TRAV_COH) && !(t & TRAV_NOSUM)) {
                const int tn = mifif(t | TRAV_NOSUM);
                const bool ok_with = render_f32_supported(b, w, tb, true);
                const bool ok_without = render_f32_supported(b, w, tn, true);
                // (an uninstantiated kernel has no register count: only instantiated ones compete)
                if (!ok_with || (ok_without && occupancy_bt(c, b, tb, w) < occupancy_bt(c, b, tn, w))) tb = tn;
            }
            if (render_f32_supported(b, w, tb, true)) cand[nc++] = {b, gflat(b, w, tb, true), w};
        }
    }
    // the if-if loop wherever one of its kernels serves the request: the while-while kernels
    // that remain (equality references) run only when asked for
    bool any_mifif = false;
    for (int i = 0; i < nc; ++i) any_mifif = any_mifif || (cand[i].trav & TRAV_MIFIF) != 0;
    // ...and never in its place: a coherent request whose (block, budget) has no if-if
    // kernel (512 threads at the compiler's budget has only the while-while 728) is refused
    // by the render with its own key instead of silently running another loop
    if (want_mifif && (t & TRAV_COH) && !any_mifif) nc = 0;
    // nothing instantiated: the tuning's own key, which the render refuses with its name
    // The most waves resident per CU wins; at equal waves the plan with the LDS item sums
    // (no per-sample 64-bit atomics to HBM), then the sphere grid over the sphere tree (worth
    // more than any number of LDS mesh-stack entries: the grid's lists take less LDS than the
    // tree's nodes, and C5's geometry ran 9.5 % faster with it, r05), then the one with more
    // mesh-stack entries in LDS (less scratch traffic), then the smaller block (the order above).  The mixed scene:
    // 512 threads reach 24 waves per CU only with neither (3 x 8 waves); 768 threads reach
    // them with both (2 x 12 waves, sums and 2 LDS entries), and win (r05).
    KernelPlan best{c->tuning.mesh_block > 0 ? c->tuning.mesh_block : c->tuning.block, t, wt >= 0 ? wt : 0};
    long best_score = -1;
    for (int i = 0; i < nc; ++i) {
        if (any_mifif && !(cand[i].trav & TRAV_MIFIF)) continue;
        const int waves = occupancy_bt(c, cand[i].block, cand[i].trav, cand[i].wpe) * (cand[i].block / 64);
        const int sums = (cand[i].trav & TRAV_COH) && !(cand[i].trav & TRAV_NOSUM) ? 1 : 0;
        const int grid = (cand[i].trav & TRAV_GRID) ? 1 : 0;
        const long score = (long)waves * 4096 + sums * 1024 + grid * 512 +
                           mesh_stack_bt(c, cand[i].block, cand[i].trav, cand[i].wpe);
        if (score > best_score) {
            best = cand[i];
            best_score = score;
        }
    }
    return best;
}

int trav_of(const rt_ctx* c) { return plan_of(c).trav; }
int block_of(const rt_ctx* c) { return plan_of(c).block; }
size_t lds_sphere_bytes(const rt_ctx* c) {
    const KernelPlan k = plan_of(c);
    return lds_sphere_bytes_bt(c, k.block, k.trav);
}
size_t lds_mesh_stack_bytes(const rt_ctx* c) {
    const KernelPlan k = plan_of(c);
    return lds_mesh_stack_bytes_bt(c, k.block, k.trav, k.wpe);
}
int wgs_per_cu(const rt_ctx* c) {
    const KernelPlan k = plan_of(c);
    return wgs_per_cu_bt(c, k.block, k.trav, k.wpe);
}
// the mesh stack entries per lane in LDS of the kernel the scene runs (RenderParams.mstack)
int mesh_stack_of(const rt_ctx* c) {
    const KernelPlan k = plan_of(c);
    return mesh_stack_bt(c, k.block, k.trav, k.wpe);
}

size_t lds_bytes(const rt_ctx* c) { return lds_sphere_bytes(c) + lds_mesh_stack_bytes(c); }

int check_camera(rt_ctx* c, const rt_camera* cam) {
    if (!cam) return fail(c, RT_ERR_INVALID, "camera is NULL");
    if (cam->image_width <= 0 || cam->image_height <= 0)
        return fail(c, RT_ERR_INVALID, "image size %dx%d", cam->image_width, cam->image_height);
    if ((long long)cam->image_width * cam->image_height > (1ll << 31) / 4)
        return fail(c, RT_ERR_LIMIT, "image too large");
    return RT_OK;
}

void fill_params(const rt_ctx* c, const rt_camera* cam, int spp, int max_depth, RenderParams& P) {
    std::memset(&P, 0, sizeof(P));
    P.W = cam->image_width;
    P.H = cam->image_height;
    P.spp = spp;
    P.max_depth = max_depth;
    P.tiles_x = (P.W + 7) / 8;
    P.tiles_x_inv = 1.0 / P.tiles_x;
    P.tiles_x_inv_half = 0.5 * P.tiles_x_inv;
    P.seed32 = seed32_of(c->seed);
    P.n_nodes = c->n_nodes;
    P.n_spheres = c->n_sph;
    P.n_mats = c->n_mat;
    P.n_big = c->n_big;
    P.n_front = c->n_front;
    P.stack_size = stack_entries(c);
    P.defocus = cam->defocus_angle > 0;  // camera.h:94 tests defocus_angle <= 0
    for (int a = 0; a < 3; ++a) {
        P.f_center[a] = (float)cam->center[a];
        P.f_p00[a] = (float)cam->pixel00_loc[a];
        P.f_du[a] = (float)cam->pixel_delta_u[a];
        P.f_dv[a] = (float)cam->pixel_delta_v[a];
        P.f_ddu[a] = (float)cam->defocus_disk_u[a];
        P.f_ddv[a] = (float)cam->defocus_disk_v[a];
        P.cam_center[a] = cam->center[a];
        P.p00[a] = cam->pixel00_loc[a];
        P.du[a] = cam->pixel_delta_u[a];
        P.dv[a] = cam->pixel_delta_v[a];
        P.ddu[a] = cam->defocus_disk_u[a];
        P.ddv[a] = cam->defocus_disk_v[a];
    }
    P.nodes = c->d_nodes;
    P.spheres = c->d_sph;
    P.mats = c->d_mat;
    P.big = c->d_big;
    P.bigf = c->d_bigf;
    P.mnodes = c->d_mnodes;
    P.tris = c->d_tris;
    P.tmeta = c->d_tmeta;
    P.n_mnodes = c->n_mnodes;
    P.mstack = c->n_mnodes > 0 ? mesh_stack_of(c) : 0;
    P.box_extent = c->box_extent;
    std::copy(c->mbox, c->mbox + 6, P.mbox);
}

}  // namespace

extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }

int rt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char* rt_error_string(int code) {
    switch (code) {
        case RT_OK: return "ok";
        case RT_ERR_INVALID: return "invalid argument";
        case RT_ERR_HIP: return "HIP runtime error";
        case RT_ERR_NO_SCENE: return "no scene uploaded";
        case RT_ERR_LIMIT: return "scene or image exceeds kernel limits";
        case RT_ERR_COMM: return "RCCL error";
        default: return "unknown error";
    }
}

rt_ctx* rt_create(int device, uint64_t seed, int precision) {
    if (precision != RT_PREC_F32 && precision != RT_PREC_F64) return nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return nullptr;
    if (hipSetDevice(device) != hipSuccess) return nullptr;
    rt_ctx* c = new rt_ctx();
    c->device = device;
    c->seed = seed;
    c->precision = precision;
    if (hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) c->n_cu = 0;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
        hipMalloc((void**)&c->d_small, 16 * sizeof(double)) != hipSuccess ||
        hipMalloc((void**)&c->d_used, sizeof(int)) != hipSuccess) {
        rt_destroy(c);
        return nullptr;
    }
    return c;
}

void rt_destroy(rt_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    free_scene(c);
    (void)hipFree(c->d_shard);
    (void)hipFree(c->d_frame);
    (void)hipFree(c->d_segs);
    (void)hipFree(c->d_segs_frame);
    (void)hipFree(c->d_rgb);
    (void)hipFree(c->d_tape);
    (void)hipFree(c->d_small);
    (void)hipFree(c->d_used);
    (void)hipFree(c->d_samples);
    (void)hipFree(c->d_queue64);
    (void)hipFree(c->d_gather);
    for (auto& a : c->accum) {
        (void)hipFree(a.acc);
        (void)hipFree(a.accp);
        (void)hipFree(a.flags);
        (void)hipFree(a.queue);
    }
    (void)hipFree(c->d_rgb8);
    if (c->h_pinned) (void)hipHostFree(c->h_pinned);
    rt_comm_release(c);
    c->lbvh.release();
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char* rt_last_error(const rt_ctx* c) { return c ? c->err.c_str() : "null context"; }

int rt_set_seed(rt_ctx* c, uint64_t seed) {
    if (!c) return RT_ERR_INVALID;
    c->seed = seed;
    return RT_OK;
}

void* rt_stream(rt_ctx* c) { return c ? (void*)c->stream : nullptr; }

int rt_get_tuning(rt_ctx* c, rt_tuning* t) {
    if (!c || !t) return RT_ERR_INVALID;
    *t = c->tuning;
    return RT_OK;
}

int rt_set_tuning(rt_ctx* c, const rt_tuning* t) {
    if (!c || !t) return RT_ERR_INVALID;
    if (t->block != 256 && t->block != 448 && t->block != 512 && t->block != 768 && t->block != 1024)
        return fail(c, RT_ERR_INVALID, "block %d (256, 448, 512, 768 or 1024)", t->block);
    if (t->max_leaf < 1 || t->max_leaf > LEAF_MAX) return fail(c, RT_ERR_INVALID, "max_leaf %d", t->max_leaf);
    if (!(t->cost_traverse > 0) || !(t->cost_intersect > 0)) return fail(c, RT_ERR_INVALID, "SAH costs must be > 0");
    if (t->waves_per_eu != 0 && t->waves_per_eu != 4 && t->waves_per_eu != 6 && t->waves_per_eu != 8)
        return fail(c, RT_ERR_INVALID, "waves_per_eu 0, 4, 6 or 8");
    if (t->mesh_waves_per_eu != -1 && t->mesh_waves_per_eu != 0 && t->mesh_waves_per_eu != 6)
        return fail(c, RT_ERR_INVALID, "mesh_waves_per_eu -1 (auto: the instantiated kernel keeping more waves "
                                       "per CU), 0 (the compiler's register budget) or 6 (<= 80 VGPRs); 5 / 7 / 8 "
                                       "are not built (7 spilled inside the traversal loop: C4 +19 %)");
    if (t->coh_refill < 1 || t->coh_refill > 64) return fail(c, RT_ERR_INVALID, "coh_refill %d (1..64)", t->coh_refill);
    if (t->f64_kernel != 0 && (t->f64_kernel == F64_KERNEL_GRID_FLAT || render_f64_block(t->f64_kernel) < 0))
        return fail(c, RT_ERR_INVALID, "f64_kernel %d (0 = default, or an instantiated one)", t->f64_kernel);
    if (t->front_spheres < -1 || t->front_spheres > 16)
        return fail(c, RT_ERR_INVALID, "front_spheres %d (-1 = auto, 0..16)", t->front_spheres);
    if (!(t->sphere_grid_density >= 0 && t->sphere_grid_density <= 64))
        return fail(c, RT_ERR_INVALID, "sphere_grid_density %g (0 = no grid, up to 64 cells per sphere)",
                    t->sphere_grid_density);
    if (t->sphere_grid_time_slabs < 1 || t->sphere_grid_time_slabs > GRID_SLAB_MAX)
        return fail(c, RT_ERR_INVALID, "sphere_grid_time_slabs %d (1..%d)", t->sphere_grid_time_slabs, GRID_SLAB_MAX);
    if (t->grid_workgroups < 0 || t->grid_workgroups > (1 << 20))
        return fail(c, RT_ERR_INVALID, "grid_workgroups %d (0 = resident)", t->grid_workgroups);
    if (t->traversal < 0 || (t->traversal & ~(1023 | TRAV_MIFIF | TRAV_MWHILE | TRAV_GRID | TRAV_GFLAT | TRAV_G3D)) != 0 ||
        (t->traversal & TRAV_REMOVED) != 0 || (t->traversal & TRAV_MIFIF && t->traversal & TRAV_MWHILE) ||
        (t->traversal & TRAV_GFLAT && t->traversal & TRAV_G3D))
        return fail(c, RT_ERR_INVALID,
                    "traversal flags: 0..1023 without 256 (time-binned trees, removed in r04), + 8192 / 16384 (mesh "
                    "if-if / while-while loop, not both), + 65536 (sphere grid), + 131072 / 262144 (its flat / 3-D "
                    "walk, not both); 4096 (mesh LDS tree top, r04) and 32768 (quantised mesh nodes, r05) were "
                    "measured slower and removed");
    if (t->mesh_max_leaf < 1 || t->mesh_max_leaf > MESH_LEAF_MAX)
        return fail(c, RT_ERR_INVALID, "mesh_max_leaf %d (1..%d)", t->mesh_max_leaf, MESH_LEAF_MAX);
    if (t->mesh_lds_nodes < -1 || t->mesh_lds_nodes > MESH_TOP_MAX)
        return fail(c, RT_ERR_INVALID, "mesh_lds_nodes %d (-1 = auto, 0..%d)", t->mesh_lds_nodes, MESH_TOP_MAX);
    if (!(t->mesh_cost_traverse > 0)) return fail(c, RT_ERR_INVALID, "mesh_cost_traverse must be > 0");
    if (t->chunk_waves < 0) return fail(c, RT_ERR_INVALID, "chunk_waves %d (0 = off)", t->chunk_waves);
    if (t->sample_buffer_mb < 16) return fail(c, RT_ERR_INVALID, "sample_buffer_mb %d (>= 16)", t->sample_buffer_mb);
    if (t->mesh_block != 0 && t->mesh_block != 256 && t->mesh_block != 512 && t->mesh_block != 768)
        return fail(c, RT_ERR_INVALID, "mesh_block %d (0 = auto, 256, 512 or 768)", t->mesh_block);
    if (t->mesh_lds_stack < -1 || t->mesh_lds_stack > MESH_STACK_MAX)
        return fail(c, RT_ERR_INVALID, "mesh_lds_stack %d (-1 = auto, 0..%d)", t->mesh_lds_stack, MESH_STACK_MAX);
    if (t->item_samples < 1 || t->item_samples > FIX_ITEM_SAMPLES || !(t->item_balance >= 0) ||
        !(t->mesh_item_balance >= 0))
        return fail(c, RT_ERR_INVALID, "item_samples %d (1..%d), item_balance %g, mesh_item_balance %g (>= 0)",
                    t->item_samples, FIX_ITEM_SAMPLES, t->item_balance, t->mesh_item_balance);
    if (t->mesh_builder != RT_MESH_BUILD_HOST && t->mesh_builder != RT_MESH_BUILD_GPU &&
        t->mesh_builder != RT_MESH_BUILD_GPU_LBVH)
        return fail(c, RT_ERR_INVALID, "mesh_builder %d", t->mesh_builder);
    if (!render_f32_supported(t->block, t->waves_per_eu, t->traversal & ~(TRAV_MIFIF | TRAV_MWHILE | TRAV_GFLAT | TRAV_G3D),
                              false))
        return fail(c, RT_ERR_INVALID, "no fp32 kernel instantiated for block %d, waves_per_eu %d, traversal %d",
                    t->block, t->waves_per_eu, t->traversal);
    const rt_tuning old = c->tuning;
    c->tuning = *t;
    if (c->has_scene && lds_bytes(c) > 160 * 1024) {
        c->tuning = old;
        return fail(c, RT_ERR_LIMIT, "scene does not fit LDS at this block");
    }
    return RT_OK;
}

int rt_camera_initialize(const rt_camera_desc* d, rt_camera* cam) {
    if (!d || !cam) return RT_ERR_INVALID;
    // camera.h:52-85; vec3 ops as vec3.h (v / t is (1/t) * v; dot and length_squared
    // associate left to right).  Built with -ffp-contract=off.
    struct v3 { double x, y, z; };
    auto add = [](v3 a, v3 b) { return v3{a.x + b.x, a.y + b.y, a.z + b.z}; };
    auto sub = [](v3 a, v3 b) { return v3{a.x - b.x, a.y - b.y, a.z - b.z}; };
    auto scl = [](double t, v3 v) { return v3{t * v.x, t * v.y, t * v.z}; };
    auto dvs = [&](v3 v, double t) { return scl(1 / t, v); };
    auto cross = [](v3 u, v3 v) {
        return v3{u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x};
    };
    auto unit = [&](v3 v) { return dvs(v, std::sqrt(v.x * v.x + v.y * v.y + v.z * v.z)); };
    auto ld = [](const double* p) { return v3{p[0], p[1], p[2]}; };
    auto st = [](double* p, v3 v) { p[0] = v.x; p[1] = v.y; p[2] = v.z; };
    const double pi = 3.1415926535897932385;                    // rtweekend.h:17
    auto deg2rad = [&](double deg) { return deg * pi / 180.0; };  // rtweekend.h:21-23

    if (d->image_width <= 0 || !(d->aspect_ratio > 0)) return RT_ERR_INVALID;
    int H = static_cast<int>(d->image_width / d->aspect_ratio);
    H = (H < 1) ? 1 : H;
    const v3 center = ld(d->lookfrom);
    const double theta = deg2rad(d->vfov);
    const double h = std::tan(theta / 2);
    const double viewport_height = 2 * h * d->focus_dist;
    const double viewport_width = viewport_height * (static_cast<double>(d->image_width) / H);
    const v3 w = unit(sub(ld(d->lookfrom), ld(d->lookat)));
    const v3 u = unit(cross(ld(d->vup), w));
    const v3 v = cross(w, u);
    const v3 viewport_u = scl(viewport_width, u);
    const v3 viewport_v = scl(viewport_height, v3{-v.x, -v.y, -v.z});
    const v3 du = dvs(viewport_u, (double)d->image_width);
    const v3 dv = dvs(viewport_v, (double)H);
    const v3 upper_left = sub(sub(sub(center, scl(d->focus_dist, w)), dvs(viewport_u, 2)), dvs(viewport_v, 2));
    const v3 p00 = add(upper_left, scl(0.5, add(du, dv)));
    const double defocus_radius = d->focus_dist * std::tan(deg2rad(d->defocus_angle / 2));
    std::memset(cam, 0, sizeof(*cam));
    cam->image_width = d->image_width;
    cam->image_height = H;
    st(cam->center, center);
    st(cam->pixel00_loc, p00);
    st(cam->pixel_delta_u, du);
    st(cam->pixel_delta_v, dv);
    st(cam->defocus_disk_u, scl(defocus_radius, u));
    st(cam->defocus_disk_v, scl(defocus_radius, v));
    cam->defocus_angle = d->defocus_angle;
    return RT_OK;
}

int rt_upload_scene(rt_ctx* c, const rt_sphere* s, int n, const rt_material* m, int nm) {
    return rt_upload_scene_ex(c, s, n, m, nm, nullptr, 0);
}

int rt_upload_scene_ex(rt_ctx* c, const rt_sphere* s, int n, const rt_material* m, int nm, const rt_triangle* tri,
                       int ntri) {
    if (!c) return RT_ERR_INVALID;
    if (n < 0 || nm < 0 || ntri < 0 || (n > 0 && !s) || (nm > 0 && !m) || (ntri > 0 && !tri))
        return fail(c, RT_ERR_INVALID, "bad scene arrays (n=%d, nm=%d, ntri=%d)", n, nm, ntri);
    if (nm > (int)META_MAT_MASK) return fail(c, RT_ERR_LIMIT, "too many materials");
    for (int k = 0; k < nm; ++k)
        if (m[k].type < RT_LAMBERTIAN || m[k].type > RT_DIELECTRIC)
            return fail(c, RT_ERR_INVALID, "material %d has type %d", k, m[k].type);
    for (int k = 0; k < n; ++k) {
        if (s[k].mat < 0 || s[k].mat >= nm)
            return fail(c, RT_ERR_INVALID, "sphere %d references material %d of %d", k, s[k].mat, nm);
        if (!std::isfinite(s[k].radius)) return fail(c, RT_ERR_INVALID, "sphere %d radius not finite", k);
        bool ok = coord_ok(s[k].radius);
        for (int a = 0; a < 3; ++a) ok = ok && coord_ok(s[k].center[a]) && coord_ok(s[k].center_vec[a]);
        if (!ok) return fail(c, RT_ERR_LIMIT, "sphere %d: a coordinate is not finite or beyond +-1e30", k);
    }
    for (int k = 0; k < ntri; ++k) {
        if (tri[k].mat < 0 || tri[k].mat >= nm)
            return fail(c, RT_ERR_INVALID, "triangle %d references material %d of %d", k, tri[k].mat, nm);
        bool ok = true;
        for (int a = 0; a < 3; ++a) ok = ok && coord_ok(tri[k].v0[a]) && coord_ok(tri[k].v1[a]) && coord_ok(tri[k].v2[a]);
        if (!ok) return fail(c, RT_ERR_LIMIT, "triangle %d: a vertex coordinate is not finite or beyond +-1e30", k);
    }
    HIPCHK(c, hipSetDevice(c->device));

    BuiltBvh bvh;
    std::string err;
    BvhParams bp;
    bp.max_leaf = c->tuning.max_leaf;
    bp.cost_traverse = c->tuning.cost_traverse;
    bp.cost_intersect = c->tuning.cost_intersect;
    bp.front = c->tuning.front_spheres;
    if (!build_bvh(s, n, bp, bvh, err)) return fail(c, RT_ERR_LIMIT, "%s", err.c_str());
    MeshBvh mbvh;
    const bool gpu_build = ntri > 0 && c->tuning.mesh_builder != RT_MESH_BUILD_HOST;
    double clo[3] = {0, 0, 0}, chi[3] = {0, 0, 0};
    if (gpu_build) {
        // validation + centroid bounds for the Morton grid; the tree is built on the device
        if (ntri > MESH_MAX_TRIS) return fail(c, RT_ERR_LIMIT, "mesh holds at most 2^24 triangles");
        for (int a = 0; a < 3; ++a) {
            clo[a] = std::numeric_limits<double>::infinity();
            chi[a] = -std::numeric_limits<double>::infinity();
        }
        for (int k = 0; k < ntri; ++k)
            for (int a = 0; a < 3; ++a) {
                const double x0 = tri[k].v0[a], x1 = tri[k].v1[a], x2 = tri[k].v2[a];
                if (!std::isfinite(x0) || !std::isfinite(x1) || !std::isfinite(x2))
                    return fail(c, RT_ERR_LIMIT, "triangle %d has a non-finite vertex", k);
                const double cm = 0.5 * (std::fmin(x0, std::fmin(x1, x2)) + std::fmax(x0, std::fmax(x1, x2)));
                clo[a] = std::fmin(clo[a], cm);
                chi[a] = std::fmax(chi[a], cm);
            }
    } else if (!build_mesh_bvh(tri, ntri, c->tuning.mesh_max_leaf, c->tuning.mesh_cost_traverse, mbvh, err)) {
        return fail(c, RT_ERR_LIMIT, "%s", err.c_str());
    }

    const bool f64 = c->precision == RT_PREC_F64;
    const int nb = (int)bvh.order.size();
    auto meta_of = [&](const rt_sphere& q) {
        return make_meta((uint32_t)q.mat, (uint32_t)m[q.mat].type, q.moving ? 1u : 0u);
    };
    std::vector<SphereF> sf;
    std::vector<SphereD> sd;
    for (int k = 0; k < nb; ++k) {
        const rt_sphere& q = s[bvh.order[k]];
        if (f64) {
            SphereD r{};
            for (int a = 0; a < 3; ++a) {
                r.c[a] = q.center[a];
                r.cv[a] = q.moving ? q.center_vec[a] : 0.0;
            }
            r.r = q.radius;
            r.meta = meta_of(q);
            sd.push_back(r);
        } else {
            SphereF r{};
            for (int a = 0; a < 3; ++a) {
                r.c[a] = (float)q.center[a];
                r.cv[a] = q.moving ? (float)q.center_vec[a] : 0.0f;
            }
            r.r = (float)q.radius;
            r.meta = meta_of(q);
            sf.push_back(r);
        }
    }
    // the big spheres' near points (BigF): on each, the point nearest the centre of the
    // other spheres' bounding box (the origin without others), and the outward normal there
    double sc_lo[3] = {0, 0, 0}, sc_hi[3] = {0, 0, 0};
    {
        bool any = false;
        for (int k = 0; k < n; ++k) {
            if (std::find(bvh.big.begin(), bvh.big.end(), k) != bvh.big.end()) continue;
            for (int a = 0; a < 3; ++a) {
                const double lo = s[k].center[a] - std::fabs(s[k].radius), hi = s[k].center[a] + std::fabs(s[k].radius);
                sc_lo[a] = any ? std::min(sc_lo[a], lo) : lo;
                sc_hi[a] = any ? std::max(sc_hi[a], hi) : hi;
            }
            any = true;
        }
    }
    // where rays can start (r06, grid_reach_ok): everything but the static opaque big spheres
    // as boxes, those as (centre, radius)
    {
        const double inf = std::numeric_limits<double>::infinity();
        for (int a = 0; a < 3; ++a) {
            c->reach_lo[a] = inf;
            c->reach_hi[a] = -inf;
        }
        c->reach_big.clear();
        auto add = [&](const double* p, double r) {
            for (int a = 0; a < 3; ++a) {
                c->reach_lo[a] = std::min(c->reach_lo[a], p[a] - r);
                c->reach_hi[a] = std::max(c->reach_hi[a], p[a] + r);
            }
        };
        for (int k = 0; k < n; ++k) {
            const rt_sphere& q = s[k];
            const bool is_big = std::find(bvh.big.begin(), bvh.big.end(), k) != bvh.big.end();
            if (is_big && !q.moving && m[q.mat].type != RT_DIELECTRIC) {
                c->reach_big.push_back({q.center[0], q.center[1], q.center[2], std::fabs(q.radius)});
                continue;
            }
            double p1[3];
            for (int a = 0; a < 3; ++a) p1[a] = q.center[a] + (q.moving ? q.center_vec[a] : 0.0);
            add(q.center, std::fabs(q.radius));
            add(p1, std::fabs(q.radius));
        }
        for (int k = 0; k < ntri; ++k) {
            add(tri[k].v0, 0.0);
            add(tri[k].v1, 0.0);
            add(tri[k].v2, 0.0);
        }
    }
    c->grid_blocked = false;
    std::vector<BigF> bigf;
    std::vector<SphereD> big;
    for (int k : bvh.big) {
        const rt_sphere& q = s[k];
        SphereD r{};
        for (int a = 0; a < 3; ++a) {
            r.c[a] = q.center[a];
            r.cv[a] = q.moving ? q.center_vec[a] : 0.0;
        }
        r.r = q.radius;
        r.meta = meta_of(q);
        r.inv_r = (float)(1.0 / q.radius);
        big.push_back(r);
        BigF f{};
        double nv[3], len = 0;
        for (int a = 0; a < 3; ++a) {
            nv[a] = 0.5 * (sc_lo[a] + sc_hi[a]) - q.center[a];
            len += nv[a] * nv[a];
        }
        len = std::sqrt(len);
        for (int a = 0; a < 3; ++a) {
            const double na = len > 0 ? nv[a] / len : (a == 1 ? 1.0 : 0.0);
            f.n[a] = (float)na;
            f.p0[a] = (float)(q.center[a] + q.radius * na);
            f.cv[a] = q.moving ? (float)q.center_vec[a] : 0.0f;
        }
        f.r = (float)q.radius;
        f.inv_r = (float)(1.0 / q.radius);
        f.meta = r.meta;
        bigf.push_back(f);
    }
    std::vector<TriF> tf;
    std::vector<uint32_t> tmeta;
    std::vector<TriD> td;
    for (int k : mbvh.order) {
        const rt_triangle& q = tri[k];
        const uint32_t meta = make_meta((uint32_t)q.mat, (uint32_t)m[q.mat].type, 0u);
        if (f64) {
            TriD r{};
            for (int a = 0; a < 3; ++a) {
                r.v0[a] = q.v0[a];
                r.e1[a] = q.v1[a] - q.v0[a];
                r.e2[a] = q.v2[a] - q.v0[a];
            }
            r.meta = meta;
            td.push_back(r);
        } else {
            TriF r{};   // each vertex rounded once: shared vertices stay identical (watertight test)
            double e1[3], e2[3];
            for (int a = 0; a < 3; ++a) {
                r.v0[a] = (float)q.v0[a];
                r.v1[a] = (float)q.v1[a];
                r.v2[a] = (float)q.v2[a];
                e1[a] = q.v1[a] - q.v0[a];
                e2[a] = q.v2[a] - q.v0[a];
            }
            r.n[0] = (float)(e1[1] * e2[2] - e1[2] * e2[1]);   // the facet normal, fp64
            r.n[1] = (float)(e1[2] * e2[0] - e1[0] * e2[2]);
            r.n[2] = (float)(e1[0] * e2[1] - e1[1] * e2[0]);
            tf.push_back(r);
            tmeta.push_back(meta);
        }
    }
    std::vector<MatF> mf;
    std::vector<MatD> md;
    for (int k = 0; k < nm; ++k) {
        double p[4] = {m[k].albedo[0], m[k].albedo[1], m[k].albedo[2], 0.0};
        if (m[k].type == RT_METAL) p[3] = m[k].fuzz < 1 ? m[k].fuzz : 1;  // material.h:33
        if (m[k].type == RT_DIELECTRIC) p[3] = m[k].ir;
        if (f64) {
            MatD r;
            for (int a = 0; a < 4; ++a) r.p[a] = p[a];
            md.push_back(r);
        } else {
            MatF r;
            for (int a = 0; a < 4; ++a) r.p[a] = (float)p[a];
            mf.push_back(r);
        }
    }

    free_scene(c);
    auto upload = [&](void** dst, const void* src, size_t bytes) -> int {
        HIPCHK(c, hipMalloc(dst, bytes ? bytes : 16));
        if (bytes) HIPCHK(c, hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice));
        return RT_OK;
    };
    int rc;
    if ((rc = upload((void**)&c->d_nodes, bvh.nodes.data(), bvh.nodes.size() * sizeof(Node))) != RT_OK) return rc;
    if (f64) {
        if ((rc = upload(&c->d_sph, sd.data(), sd.size() * sizeof(SphereD))) != RT_OK) return rc;
        if ((rc = upload(&c->d_mat, md.data(), md.size() * sizeof(MatD))) != RT_OK) return rc;
    } else {
        if ((rc = upload(&c->d_sph, sf.data(), sf.size() * sizeof(SphereF))) != RT_OK) return rc;
        if ((rc = upload(&c->d_mat, mf.data(), mf.size() * sizeof(MatF))) != RT_OK) return rc;
    }
    {
        // the uniform grid over the tree's spheres, where the scene suits one (TRAV_GRID);
        // fp64 scenes list their spheres from the records rounded to fp32 (the padding
        // covers the rounding: the cells only choose which spheres are tested)
        std::vector<SphereF> sg;
        if (f64)
            for (const SphereD& q : sd) {
                SphereF r{};
                for (int a = 0; a < 3; ++a) {
                    r.c[a] = (float)q.c[a];
                    r.cv[a] = (float)q.cv[a];
                }
                r.r = (float)q.r;
                r.meta = q.meta;
                sg.push_back(r);
            }
        std::vector<unsigned char> grid;
        if (c->tuning.sphere_grid_density > 0 &&
            build_sphere_grid(f64 ? sg.data() : sf.data(), bvh.front, nb, c->tuning.sphere_grid_density,
                              c->tuning.sphere_grid_time_slabs, f64 ? (int)sizeof(SphereD) : (int)sizeof(SphereF),
                              c->grid_hdr, grid)) {
            if ((rc = upload(&c->d_grid, grid.data(), grid.size())) != RT_OK) return rc;
            c->grid_nodes = (int)(grid.size() / sizeof(Node));
            c->grid_density = c->tuning.sphere_grid_density;
            const uint32_t last = ((const uint32_t*)grid.data())[c->grid_hdr.n_cells - 1 +
                                                                 (uint32_t)(c->grid_hdr.res[0] * c->grid_hdr.res[1])];
            // (the last cell's end position, in bytes, less the pad layers and the cells)
            c->grid_entries = (int)((last >> GRID_POS_BITS) / 4u - c->grid_hdr.n_cells -
                                    2u * (uint32_t)(c->grid_hdr.res[0] * c->grid_hdr.res[1]));
        }
    }
    if ((rc = upload((void**)&c->d_big, big.data(), big.size() * sizeof(SphereD))) != RT_OK) return rc;
    if ((rc = upload((void**)&c->d_bigf, bigf.data(), bigf.size() * sizeof(BigF))) != RT_OK) return rc;
    if (gpu_build) {
        rt_triangle* d_in = nullptr;
        uint32_t* d_types = nullptr;
        std::vector<uint32_t> types(nm);
        for (int k = 0; k < nm; ++k) types[k] = (uint32_t)m[k].type;
        if ((rc = upload((void**)&d_in, tri, (size_t)ntri * sizeof(rt_triangle))) != RT_OK) return rc;
        if ((rc = upload((void**)&d_types, types.data(), types.size() * 4)) != RT_OK) {
            (void)hipFree(d_in);
            return rc;
        }
        const int cap = ntri > 1 ? ntri - 1 : 1;
        hipError_t e = hipMalloc((void**)&c->d_mnodes, (size_t)cap * sizeof(Node4));
        if (e == hipSuccess) e = hipMalloc(&c->d_tris, f64 ? (size_t)ntri * sizeof(TriD) : (size_t)ntri * sizeof(TriF) + TRIF_SLACK);
        if (e == hipSuccess && !f64) e = hipMalloc((void**)&c->d_tmeta, (size_t)ntri * sizeof(uint32_t));
        if (e == hipSuccess && !f64) e = hipMemsetAsync((char*)c->d_tris + (size_t)ntri * sizeof(TriF), 0, TRIF_SLACK, c->stream);
        LbvhInput in{};
        in.tris = d_in;
        in.n = ntri;
        in.mat_type = d_types;
        for (int a = 0; a < 3; ++a) {
            in.lo[a] = clo[a];
            in.inv[a] = chi[a] > clo[a] ? 1.0 / (chi[a] - clo[a]) : 0.0;
        }
        in.max_leaf = std::max(1, std::min(c->tuning.mesh_max_leaf, MESH_LEAF_MAX));
        in.f64 = f64;
        // two rounds of treelet restructuring: the 4-wide SAH cost of the C4 blob's tree 28.56
        // -> 25.77 -> 25.41 (3: 25.32) against the host SAH tree's 24.7 (tests/cpp/treelet_check.cpp)
        in.treelet_rounds = c->tuning.mesh_builder == RT_MESH_BUILD_GPU ? 2 : 0;
        LbvhOutput out{c->d_mnodes, cap, c->d_tris, c->d_tmeta};
        if (e == hipSuccess) e = lbvh_build(in, c->lbvh, out, c->stream);
        (void)hipFree(d_in);
        (void)hipFree(d_types);
        if (e != hipSuccess) {
            free_scene(c);
            return fail(c, RT_ERR_HIP, "GPU mesh BVH build: %s", hipGetErrorString(e));
        }
        if (3 * out.depth4 + 1 > MESH_STACK_MAX) {
            free_scene(c);
            return fail(c, RT_ERR_LIMIT, "GPU mesh BVH depth %d exceeds the traversal stack (use the host builder)",
                        out.depth4);
        }
        c->n_mnodes = out.node_count;
        c->n_tris = ntri;
        c->mdepth = out.depth4;
        c->mleaves = out.leaves;
    } else if (ntri > 0) {
        if ((rc = upload((void**)&c->d_mnodes, mbvh.nodes4.data(), mbvh.nodes4.size() * sizeof(Node4))) != RT_OK)
            return rc;
        if (f64) {
            if ((rc = upload(&c->d_tris, td.data(), td.size() * sizeof(TriD))) != RT_OK) return rc;
        } else {
            // the records plus TRIF_SLACK zero bytes (the if-if loop's 80-B leaf reads)
            tf.resize(tf.size() + (TRIF_SLACK + sizeof(TriF) - 1) / sizeof(TriF), TriF{});
            if ((rc = upload(&c->d_tris, tf.data(), tf.size() * sizeof(TriF))) != RT_OK) return rc;
            if ((rc = upload((void**)&c->d_tmeta, tmeta.data(), tmeta.size() * sizeof(uint32_t))) != RT_OK) return rc;
        }
        c->n_mnodes = (int)mbvh.nodes4.size();
        c->n_tris = ntri;
        c->mdepth = mbvh.depth4;
        c->mleaves = mbvh.leaves;
    }
    if (c->n_mnodes > 0) {
        // the mesh's box: the union of the root's child boxes, as the kernels test them
        // (read back from the device, so either builder's tree gives it)
        Node4 root;
        const hipError_t e = hipMemcpy(&root, c->d_mnodes, sizeof(Node4), hipMemcpyDeviceToHost);
        if (e != hipSuccess) {
            free_scene(c);
            return fail(c, RT_ERR_HIP, "mesh root read-back: %s", hipGetErrorString(e));
        }
        const float inf = std::numeric_limits<float>::infinity();
        float b[6] = {inf, inf, inf, -inf, -inf, -inf};
        for (int k = 0; k < 4; ++k) {
            if (root.ref[k] == MREF_EMPTY) continue;
            b[0] = std::min(b[0], root.lox[k]), b[1] = std::min(b[1], root.loy[k]), b[2] = std::min(b[2], root.loz[k]);
            b[3] = std::max(b[3], root.hix[k]), b[4] = std::max(b[4], root.hiy[k]), b[5] = std::max(b[5], root.hiz[k]);
        }
        std::copy(b, b + 6, c->mbox);
    }
    {
        // TRAV_F32BOX (fp64 kernels): a bound of |coordinate| over the sphere-tree boxes and
        // the triangles (the mesh boxes enclose them, rounded outward by an ulp)
        double ext = 0.0;
        for (const Node& nd : bvh.nodes)
            for (int a = 0; a < 3; ++a)
                ext = std::max({ext, (double)std::fabs(nd.lo0[a]), (double)std::fabs(nd.hi0[a]),
                                (double)std::fabs(nd.lo1[a]), (double)std::fabs(nd.hi1[a])});
        for (int k = 0; k < ntri; ++k)
            for (int a = 0; a < 3; ++a)
                ext = std::max({ext, std::fabs(tri[k].v0[a]), std::fabs(tri[k].v1[a]), std::fabs(tri[k].v2[a])});
        c->box_extent = std::isfinite(ext) ? (float)(ext * (1.0 + 0x1p-20)) : 3e38f;
    }
    c->n_nodes = (int)bvh.nodes.size();
    c->n_sph = nb;
    c->n_front = bvh.front;
    c->n_mat = nm;
    c->n_big = (int)big.size();
    c->depth = bvh.depth;
    c->leaves = bvh.leaves;
    c->n_input = n;
    {
        // rt_trace_rays' id map: BVH sphere position -> input index, then the big spheres,
        // then the triangles in leaf order (input index + n)
        std::vector<int> remap;
        remap.reserve((size_t)nb + big.size() + (size_t)ntri);
        for (int k = 0; k < nb; ++k) remap.push_back(bvh.order[k]);
        for (int k : bvh.big) remap.push_back(k);
        if (!gpu_build)
            for (int k : mbvh.order) remap.push_back(n + k);
        else if (ntri > 0) {
            std::vector<uint32_t> perm((size_t)ntri);
            HIPCHK(c, hipMemcpy(perm.data(), lbvh_sorted_index(c->lbvh, ntri), (size_t)ntri * 4, hipMemcpyDeviceToHost));
            for (uint32_t k : perm) remap.push_back(n + (int)k);
        }
        if ((rc = upload((void**)&c->d_remap, remap.data(), remap.size() * sizeof(int))) != RT_OK) return rc;
    }
    const size_t lds = lds_bytes(c);
    if (lds > 160 * 1024) {
        free_scene(c);
        return fail(c, RT_ERR_LIMIT, "scene needs %zu B of LDS per workgroup (> 160 KiB)", lds);
    }
    c->has_scene = true;
    return RT_OK;
}

int rt_scene_info_get(rt_ctx* c, rt_scene_info* info) {
    if (!c || !info) return RT_ERR_INVALID;
    if (!c->has_scene) return fail(c, RT_ERR_NO_SCENE, "no scene");
    info->num_spheres = c->n_input;
    info->num_materials = c->n_mat;
    info->bvh_nodes = c->n_nodes;
    info->bvh_depth = c->depth;
    info->bvh_leaves = c->leaves;
    info->big_spheres = c->n_big;
    // (the plan of a launch whose rays all start within the sphere grid's reach: rt_grid_reach)
    const bool blocked = c->grid_blocked;
    c->grid_blocked = false;
    info->lds_bytes = (int)lds_bytes(c);
    const KernelPlan plan = plan_of(c);
    c->grid_blocked = blocked;
    info->render_block = plan.block;
    info->render_traversal = plan.trav;
    info->render_waves_per_eu = c->precision == RT_PREC_F32 ? plan.wpe : 0;
    info->render_mesh_lds_stack = mesh_stack_of(c);
    for (int a = 0; a < 3; ++a) info->grid_res[a] = c->grid_nodes > 0 ? c->grid_hdr.res[a] : 0;
    info->grid_entries = c->grid_entries;
    info->grid_time_slabs = c->grid_nodes > 0 ? c->grid_hdr.n_slab : 0;
    info->grid_far_o = c->grid_nodes > 0 ? c->grid_hdr.far_o : 0.f;
    info->grid_density = c->grid_nodes > 0 ? c->grid_density : 0.0;
    info->precision = c->precision;
    info->num_triangles = c->n_tris;
    info->mesh_nodes = c->n_mnodes;
    info->mesh_depth = c->mdepth;
    info->mesh_leaves = c->mleaves;
    return RT_OK;
}

int rt_grid_reach(rt_ctx* c, const rt_camera* cam, int32_t* walks) {
    if (!c || !walks) return RT_ERR_INVALID;
    if (!c->has_scene) return fail(c, RT_ERR_NO_SCENE, "rt_grid_reach before rt_upload_scene");
    int rc = check_camera(c, cam);
    if (rc) return rc;
    *walks = c->grid_nodes > 0 && grid_reach_ok(c, cam) ? 1 : 0;
    return RT_OK;
}

int rt_shard_layout(int width, int height, int shard, int num_shards, rt_shard_info* info) {
    if (!info || width <= 0 || height <= 0 || num_shards <= 0 || shard < 0 || shard >= num_shards)
        return RT_ERR_INVALID;
    info->tile_w = 8;
    info->tile_h = 8;
    info->tiles_x = (width + 7) / 8;
    info->tiles_y = (height + 7) / 8;
    info->num_tiles = info->tiles_x * info->tiles_y;
    info->shard = shard;
    info->num_shards = num_shards;
    info->shard_tiles = (info->num_tiles - shard + num_shards - 1) / num_shards;
    info->max_shard_tiles = (info->num_tiles + num_shards - 1) / num_shards;
    return RT_OK;
}

// Largest work item (samples) of a persistent launch.  Coherent kernels: a work item
// belongs to one wave, so on small shards (many lanes per pixel) big items leave too few
// items per wave to even out; cap the item at the power of two <= 12 pixels per lane, but
// not below the power of two <= min(8, 24 pixels per lane) (C3 shards of 1 / 2 / 4 / 8
// GPUs: 32 / 16 / 8 / 8 -- measured 50.5 / 25.8 / 13.4 / 7.14 ms against 50.5 / 26.3 /
// 13.6 / 7.17 with the earlier 24-pixel cap (32 / 32 / 16 / 8),
// profiles/r02/item_cap_scaling_r02bn.log; 4 at 8 GPUs lost, item_size_sweep_r02ai.log)
static int item_cap(const rt_ctx* c, double lanes, double pixels) {
    int cmax = std::min(c->tuning.item_samples, FIX_ITEM_SAMPLES);
    if ((trav_of(c) & TRAV_COH) && c->n_mnodes == 0) {
        const double ppl = pixels / std::max(1.0, lanes);
        int cap = 1, floor_cap = 1;
        while (cap * 2 <= 12.0 * ppl && cap < FIX_ITEM_SAMPLES) cap *= 2;
        while (floor_cap * 2 <= 24.0 * ppl && floor_cap < 8) floor_cap *= 2;
        cmax = std::min(cmax, std::max(cap, floor_cap));
    }
    return cmax;
}

// Work-queue item phases of a persistent launch of spp samples, largest chunks first: a
// chunk of c samples is handed out only while the samples left after it keep every
// resident lane busy for `balance` chunks of that size, i.e. while
// left - c >= balance * c * lanes / pixels; single samples take the rest.
static void plan_phases(RenderParams& P, int spp, double lanes, double pixels, double balance, int cmax) {
    int left = spp, s0 = 0;
    P.nph = 0;
    for (int ch = 1 << 5; ch >= 1; ch >>= 1) {
        if (ch > cmax || left <= 0) continue;
        int k = left;   // single samples: the rest
        if (ch > 1) {
            const double keep = balance * ch * lanes / std::max(1.0, pixels);
            k = left - ch >= keep ? (int)((left - keep) / ch) : 0;
        }
        if (k <= 0) continue;
        P.ph_s0[P.nph] = s0;
        P.ph_c[P.nph] = ch;
        P.ph_k[P.nph] = k;
        ++P.nph;
        s0 += k * ch;
        left -= k * ch;
    }
}

// Item balance of an fp32 launch: the tuning's, doubled for a mesh scene whose shard has
// fewer pixels than the launch has resident lanes, so its single samples start earlier.
// On C4 at 8 GPUs that cuts the shard 6.25 -> 6.06 ms (predicted 5.94x -> 6.12x), and the
// 1-GPU frame (2.07 M pixels for 0.39 M lanes) is unchanged (profiles/r04/r04n/sc4c_ib*.log:
// mesh_item_balance 20 / 40 / 80 / 160 gave N = 8 shards of 6.25 / 6.06 / 6.12 / 6.10 ms and
// N = 1 frames of 37.14 / 37.22 / 37.67 / 37.99 ms).  Sphere scenes were not measured this
// way and keep item_balance.
static double item_balance_of(const rt_ctx* c, double lanes, double pixels) {
    if (c->n_mnodes == 0) return c->tuning.item_balance;
    return c->tuning.mesh_item_balance * (lanes > pixels ? 2.0 : 1.0);
}

int rt_render_range(rt_ctx* c, const rt_camera* cam, int sample_begin, int spp, int max_depth, int shard,
                    int num_shards, int accumulate, void* out_sums, uint32_t* out_segments, void* stream) {
    if (!c) return RT_ERR_INVALID;
    if (!c->has_scene) return fail(c, RT_ERR_NO_SCENE, "rt_render before rt_upload_scene");
    int rc = check_camera(c, cam);
    if (rc) return rc;
    if (spp < 0 || sample_begin < 0) return fail(c, RT_ERR_INVALID, "samples [%d, +%d)", sample_begin, spp);
    if (c->precision == RT_PREC_F64 && max_depth > 64)
        return fail(c, RT_ERR_LIMIT, "fp64 path keeps at most 64 bounces (max_depth %d)", max_depth);
    if (!out_sums) return fail(c, RT_ERR_INVALID, "out_sums is NULL");
    rt_shard_info si;
    if (rt_shard_layout(cam->image_width, cam->image_height, shard, num_shards, &si) != RT_OK)
        return fail(c, RT_ERR_INVALID, "bad shard %d of %d", shard, num_shards);
    HIPCHK(c, hipSetDevice(c->device));
    c->grid_blocked = !grid_reach_ok(c, cam);   // (before anything plans the launch)
    RenderParams P;
    fill_params(c, cam, spp, max_depth, P);
    P.sample_begin = sample_begin;
    P.accumulate = accumulate ? 1 : 0;
    P.shard = shard;
    P.nshards = num_shards;
    P.shard_tiles = si.shard_tiles;
    P.out_sums = out_sums;
    P.out_segs = out_segments;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    if (c->precision == RT_PREC_F32 && spp > FIX_LAUNCH_SAMPLES) {
        // packed per-launch sums hold <= FIX_LAUNCH_SAMPLES samples: consecutive ranges,
        // timed as one (rt_last_kernel_ms spans all of them)
        hipEvent_t start = nullptr;
        HIPCHK(c, hipEventCreate(&start));
        hipError_t er = hipEventRecord(start, st);
        for (int done = 0; done < spp && er == hipSuccess; done += FIX_LAUNCH_SAMPLES) {
            const int n = spp - done < FIX_LAUNCH_SAMPLES ? spp - done : FIX_LAUNCH_SAMPLES;
            if ((rc = rt_render_range(c, cam, sample_begin + done, n, max_depth, shard, num_shards,
                                      accumulate || done > 0, out_sums, out_segments, stream))) {
                (void)hipEventDestroy(start);
                return rc;
            }
        }
        std::swap(c->ev0, start);   // the first sub-range's start event is replaced by the whole call's
        (void)hipEventDestroy(start);
        if (er != hipSuccess) return fail(c, RT_ERR_HIP, "hipEventRecord: %s", hipGetErrorString(er));
        return RT_OK;
    }
    const size_t lds = lds_bytes(c);
    if (lds > 160 * 1024) return fail(c, RT_ERR_LIMIT, "render needs %zu B of LDS per workgroup", lds);
    const KernelPlan plan = plan_of(c);
    if (c->precision == RT_PREC_F32 && c->n_mnodes > 0 && !render_f32_supported(plan.block, plan.wpe, plan.trav, true))
        return fail(c, RT_ERR_INVALID, "no mesh kernel instantiated for block %d, mesh_waves_per_eu %d, traversal %d",
                    plan.block, plan.wpe, plan.trav);
    if (c->precision == RT_PREC_F32 && c->n_mnodes == 0 &&
        !render_f32_supported(block_of(c), c->tuning.waves_per_eu, trav_of(c), false))
        return fail(c, RT_ERR_INVALID,
                    "no fp32 kernel instantiated for block %d, waves_per_eu %d, traversal %d (tuning traversal %d; "
                    "128 = no LDS sums is added where they would cost occupancy)",
                    block_of(c), c->tuning.waves_per_eu, trav_of(c), c->tuning.traversal);
    if (c->precision == RT_PREC_F32 && c->diag_buf &&
        !render_f32_diag_supported(block_of(c), plan_of(c).wpe, trav_of(c), c->n_mnodes > 0))
        return fail(c, RT_ERR_INVALID, "no instrumented build of block %d, waves_per_eu %d, traversal %d (rt_render_diag)",
                    block_of(c), plan_of(c).wpe, trav_of(c));
    if (plan.trav & TRAV_GRID) {
        // the grid walk reads cells and records by LDS byte address, counting from 0: the
        // kernel's dynamic LDS must start there, i.e. the kernel has no static LDS (rt_device.h)
        const bool f64 = c->precision == RT_PREC_F64;
        const int s = f64 ? render_f64_static_lds(c->n_mnodes > 0, f64_kernel_of(c))
                          : render_f32_static_lds(plan.block, plan.wpe, plan.trav, c->n_mnodes > 0);
        if (s != 0) return fail(c, RT_ERR_HIP, "grid render kernel with %d B of static LDS (needs none)", s);
    }
    apply_grid(c, plan.trav, P);
    auto launch = [&](const RenderParams& q) {
        return c->precision == RT_PREC_F64
                   ? launch_render_f64(q, lds, st, f64_kernel_of(c))
                   : launch_render_f32(q, lds, st, plan.block, plan.wpe, plan.trav);
    };
    const size_t npx = (size_t)si.shard_tiles * 64, eb = elem_bytes(c);
    hipError_t e = hipSuccess;
    if (c->precision == RT_PREC_F32) {
        // fp32: lanes add their chunk's fixed-point sums into the context's accumulator
        // for this buffer (integer atomics: order-free), finalize_kernel writes out_sums.
        rt_ctx::Accum* slot = nullptr;
        for (auto& a : c->accum)
            if (a.out == out_sums && a.W == P.W && a.H == P.H && a.shard == shard && a.nshards == num_shards) slot = &a;
        const bool have = slot != nullptr;
        if (!slot) {
            slot = &c->accum[0];
            for (auto& a : c->accum)
                if (a.used < slot->used) slot = &a;
        }
        if ((rc = grow(c, (void**)&slot->acc, &slot->acc_cap, npx * 3 * sizeof(long long)))) return rc;
        if ((rc = grow(c, (void**)&slot->accp, &slot->accp_cap, npx * 2 * sizeof(unsigned long long)))) return rc;
        if ((rc = grow(c, (void**)&slot->flags, &slot->flags_cap, npx * sizeof(uint32_t)))) return rc;
        slot->out = out_sums;
        slot->W = P.W;
        slot->H = P.H;
        slot->shard = shard;
        slot->nshards = num_shards;
        slot->used = ++c->accum_clock;
        P.accum = slot->acc;
        P.accum_flags = slot->flags;
        P.accp = slot->accp;
        P.diag = c->diag_buf;
        P.coh_refill = c->tuning.coh_refill;
        // persistent lanes: no more workgroups than the device keeps resident
        if (!slot->queue) HIPCHK(c, hipMalloc((void**)&slot->queue, QUEUE_CTRL_BYTES));
        P.queue = slot->queue;
        {
            const int by_lds = lds > 0 ? (int)(160 * 1024 / lds) : 64;
            const int per_cu = std::min(wgs_per_cu(c), std::max(1, by_lds));
            P.max_wgs = std::max(1, per_cu * (c->n_cu > 0 ? c->n_cu : 256));
            if (c->tuning.grid_workgroups > 0) P.max_wgs = c->tuning.grid_workgroups;
        }
        {
            const double lanes = (double)P.max_wgs * block_of(c), pixels = (double)npx;
            plan_phases(P, spp, lanes, pixels, item_balance_of(c, lanes, pixels), item_cap(c, lanes, pixels));
        }
        HIPCHK(c, hipEventRecord(c->ev0, st));
        HIPCHK(c, hipMemsetAsync(slot->queue, 0, QUEUE_CTRL_BYTES, st));
        HIPCHK(c, hipMemsetAsync(slot->accp, 0, npx * 2 * sizeof(unsigned long long), st));
        if (!accumulate) {
            e = hipMemsetAsync(slot->acc, 0, npx * 3 * sizeof(long long), st);
            if (e == hipSuccess) e = hipMemsetAsync(slot->flags, 0, npx * sizeof(uint32_t), st);
            if (e == hipSuccess && out_segments) e = hipMemsetAsync(out_segments, 0, npx * sizeof(uint32_t), st);
        } else if (!have) {
            // no fixed-point state for this buffer: continue from its float values
            e = launch_seed_accum((const float*)out_sums, slot->acc, slot->flags, npx, st);
        } else {
            // state for this address: kept where out_sums still holds what it last
            // finalized to, restarted from the floats elsewhere (a reallocated buffer)
            e = launch_reconcile_accum((const float*)out_sums, slot->acc, slot->flags, npx, st);
        }
        if (e == hipSuccess && spp > 0)
            e = c->diag_buf ? launch_render_f32_diag(P, lds, st, trav_of(c), block_of(c), plan_of(c).wpe) : launch(P);
        if (e == hipSuccess) e = launch_finalize(slot->acc, slot->accp, slot->flags, (float*)out_sums, npx, st);
    } else {
        // fp64 on persistent lanes (TRAV_PERSIST): every sample's radiance goes to
        // d_samples, then the ordered reduction; passes bound the buffer to sample_buffer_mb
        // (a shard with no tiles has nothing to store: npx = 0)
        // The coherent kernel's FIFO entries carry a sample's index within the pass in 16
        // bits (CohEntryD::sid, the hit id above it): a pass holds at most 65535 samples.
        constexpr size_t MAX_PASS_SAMPLES = 0xffff;
        const size_t fit = std::min(MAX_PASS_SAMPLES, npx > 0 ? ((size_t)c->tuning.sample_buffer_mb << 20) /
                                                                    (npx * 3 * eb) : (size_t)spp);
        const int pass_spp = std::max(1, (size_t)spp < fit ? spp : (int)std::max<size_t>(1, fit));
        if ((rc = grow(c, &c->d_samples, &c->samples_cap, npx * 3 * eb * (size_t)std::max(1, pass_spp)))) return rc;
        if (!c->d_queue64) HIPCHK(c, hipMalloc((void**)&c->d_queue64, QUEUE_CTRL_BYTES));
        P.queue = c->d_queue64;
        P.coh_refill = c->tuning.coh_refill;   // (coherent fp64 kernel)
        {
            const int by_lds = lds > 0 ? (int)(160 * 1024 / lds) : 64;
            const int per_cu = std::min(wgs_per_cu(c), std::max(1, by_lds));
            P.max_wgs = std::max(1, per_cu * (c->n_cu > 0 ? c->n_cu : 256));
            if (c->tuning.grid_workgroups > 0) P.max_wgs = c->tuning.grid_workgroups;
        }
        const double balance = c->n_mnodes > 0 ? c->tuning.mesh_item_balance : c->tuning.item_balance;
        HIPCHK(c, hipEventRecord(c->ev0, st));
        if (out_segments && !accumulate) e = hipMemsetAsync(out_segments, 0, npx * sizeof(uint32_t), st);
        if (e == hipSuccess && spp == 0 && !accumulate) e = hipMemsetAsync(out_sums, 0, npx * 3 * eb, st);
        for (int done = 0; done < spp && npx > 0 && e == hipSuccess; done += pass_spp) {
            RenderParams Q = P;
            Q.sample_begin = sample_begin + done;
            Q.spp = spp - done < pass_spp ? spp - done : pass_spp;
            Q.samples = c->d_samples;
            const double lanes = (double)Q.max_wgs * block_of(c);
            plan_phases(Q, Q.spp, lanes, (double)npx, balance, item_cap(c, lanes, (double)npx));
            e = hipMemsetAsync(c->d_queue64, 0, QUEUE_CTRL_BYTES, st);
            if (e == hipSuccess) e = launch(Q);
            if (e == hipSuccess)
                e = launch_reduce(c->d_samples, out_sums, (int)eb, npx * 3, Q.spp, (accumulate || done > 0) ? 1 : 0, st);
        }
    }
    if (e != hipSuccess) return fail(c, RT_ERR_HIP, "render launch: %s", hipGetErrorString(e));
    HIPCHK(c, hipEventRecord(c->ev1, st));
    c->timed = true;
    return RT_OK;
}

int rt_render(rt_ctx* c, const rt_camera* cam, int spp, int max_depth, int shard, int num_shards, void* out_sums,
              uint32_t* out_segments, void* stream) {
    return rt_render_range(c, cam, 0, spp, max_depth, shard, num_shards, 0, out_sums, out_segments, stream);
}

int rt_last_kernel_ms(rt_ctx* c, float* ms) {
    if (!c || !ms) return RT_ERR_INVALID;
    if (!c->timed) return fail(c, RT_ERR_INVALID, "no kernel launched yet");
    HIPCHK(c, hipEventSynchronize(c->ev1));
    HIPCHK(c, hipEventElapsedTime(ms, c->ev0, c->ev1));
    return RT_OK;
}

int rt_unshard(rt_ctx* c, const void* gathered, int width, int height, int num_shards, void* frame, void* stream) {
    if (!c || !gathered || !frame || width <= 0 || height <= 0 || num_shards <= 0) return RT_ERR_INVALID;
    rt_shard_info si;
    rt_shard_layout(width, height, 0, num_shards, &si);
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, launch_unshard(gathered, frame, (int)elem_bytes(c), 3, width, height, si.tiles_x, num_shards,
                             si.max_shard_tiles, st));
    return RT_OK;
}

int rt_quantize(rt_ctx* c, const void* frame, int width, int height, int spp, int32_t* rgb, void* stream) {
    if (!c || !frame || !rgb || width <= 0 || height <= 0) return RT_ERR_INVALID;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, launch_quantize(frame, (int)elem_bytes(c), rgb, (size_t)width * height * 3, spp, st));
    return RT_OK;
}

int rt_render_frame(rt_ctx* c, const rt_camera* cam, int spp, int max_depth, void* sums_host, int32_t* rgb_host,
                    uint32_t* segments_host) {
    if (!c) return RT_ERR_INVALID;
    int rc = check_camera(c, cam);
    if (rc) return rc;
    HIPCHK(c, hipSetDevice(c->device));
    const int W = cam->image_width, H = cam->image_height;
    rt_shard_info si;
    rt_shard_layout(W, H, 0, 1, &si);
    const size_t npx_tiles = (size_t)si.num_tiles * 64, npx = (size_t)W * H, eb = elem_bytes(c);
    if ((rc = grow(c, &c->d_shard, &c->shard_cap, npx_tiles * 3 * eb))) return rc;
    if ((rc = grow(c, &c->d_frame, &c->frame_cap, npx * 3 * eb))) return rc;
    if ((rc = grow(c, (void**)&c->d_segs, &c->segs_cap, npx_tiles * 4))) return rc;
    if ((rc = grow(c, (void**)&c->d_segs_frame, &c->segs_frame_cap, npx * 4))) return rc;
    if ((rc = grow(c, (void**)&c->d_rgb, &c->rgb_cap, npx * 3 * 4))) return rc;
    if ((rc = rt_render(c, cam, spp, max_depth, 0, 1, c->d_shard, c->d_segs, nullptr))) return rc;
    HIPCHK(c, launch_unshard(c->d_shard, c->d_frame, (int)eb, 3, W, H, si.tiles_x, 1, si.max_shard_tiles, c->stream));
    if (segments_host)
        HIPCHK(c, launch_unshard(c->d_segs, c->d_segs_frame, 4, 1, W, H, si.tiles_x, 1, si.max_shard_tiles,
                                 c->stream));
    if (rgb_host) HIPCHK(c, launch_quantize(c->d_frame, (int)eb, c->d_rgb, npx * 3, spp, c->stream));
    if (sums_host)
        HIPCHK(c, hipMemcpyAsync(sums_host, c->d_frame, npx * 3 * eb, hipMemcpyDeviceToHost, c->stream));
    if (rgb_host) HIPCHK(c, hipMemcpyAsync(rgb_host, c->d_rgb, npx * 3 * 4, hipMemcpyDeviceToHost, c->stream));
    if (segments_host)
        HIPCHK(c, hipMemcpyAsync(segments_host, c->d_segs_frame, npx * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return RT_OK;
}

int rt_finish_frame_u8(rt_ctx* c, const void* gathered, int width, int height, int num_shards, int spp,
                       uint8_t* rgb8, void* stream) {
    if (!c) return RT_ERR_INVALID;
    if (!gathered || !rgb8 || width <= 0 || height <= 0 || num_shards <= 0 || spp <= 0)
        return fail(c, RT_ERR_INVALID, "finish %dx%d over %d shards at %d spp", width, height, num_shards, spp);
    rt_shard_info si;
    rt_shard_layout(width, height, 0, num_shards, &si);
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, launch_finish_u8(gathered, (int)elem_bytes(c), rgb8, width, height, si.tiles_x, num_shards,
                               si.max_shard_tiles, spp, st));
    return RT_OK;
}

void* rt_host_alloc(size_t bytes) {
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes ? bytes : 16, hipHostMallocDefault) != hipSuccess) return nullptr;
    return p;
}

void rt_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

int rt_render_frame_u8(rt_ctx* c, const rt_camera* cam, int spp, int max_depth, uint8_t* rgb8_host) {
    if (!c) return RT_ERR_INVALID;
    int rc = check_camera(c, cam);
    if (rc) return rc;
    if (!rgb8_host || spp <= 0) return fail(c, RT_ERR_INVALID, "rgb8_host %p, spp %d", (void*)rgb8_host, spp);
    HIPCHK(c, hipSetDevice(c->device));
    const int W = cam->image_width, H = cam->image_height;
    rt_shard_info si;
    rt_shard_layout(W, H, 0, 1, &si);
    const size_t bytes = (size_t)W * H * 3;
    if ((rc = grow(c, &c->d_shard, &c->shard_cap, (size_t)si.num_tiles * 64 * 3 * elem_bytes(c)))) return rc;
    if ((rc = grow(c, (void**)&c->d_rgb8, &c->rgb8_cap, bytes))) return rc;
    // copy straight into page-locked caller memory, else through the context's staging buffer
    hipPointerAttribute_t attr;
    bool pinned = hipPointerGetAttributes(&attr, rgb8_host) == hipSuccess && attr.type == hipMemoryTypeHost;
    (void)hipGetLastError();
    if (!pinned && c->pinned_cap < bytes) {
        if (c->h_pinned) HIPCHK(c, hipHostFree(c->h_pinned));
        c->h_pinned = nullptr;
        c->pinned_cap = 0;
        HIPCHK(c, hipHostMalloc(&c->h_pinned, bytes, hipHostMallocDefault));
        c->pinned_cap = bytes;
    }
    if ((rc = rt_render(c, cam, spp, max_depth, 0, 1, c->d_shard, nullptr, nullptr))) return rc;
    HIPCHK(c, launch_finish_u8(c->d_shard, (int)elem_bytes(c), c->d_rgb8, W, H, si.tiles_x, 1, si.max_shard_tiles, spp,
                               c->stream));
    HIPCHK(c, hipMemcpyAsync(pinned ? (void*)rgb8_host : c->h_pinned, c->d_rgb8, bytes, hipMemcpyDeviceToHost,
                             c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (!pinned) std::memcpy(rgb8_host, c->h_pinned, bytes);
    return RT_OK;
}

int rt_render_frame_multi(rt_ctx** cs, int n, const rt_camera* cam, int spp, int max_depth, void* sums_host,
                          int32_t* rgb_host) {
    if (!cs || n <= 0) return RT_ERR_INVALID;
    for (int r = 0; r < n; ++r) {
        if (!cs[r]) return RT_ERR_INVALID;
        if (cs[r]->precision != cs[0]->precision)
            return fail(cs[0], RT_ERR_INVALID, "contexts %d and 0 differ in precision", r);
        for (int q = 0; q < r; ++q)
            if (cs[q] == cs[r]) return fail(cs[0], RT_ERR_INVALID, "context %d is listed twice", r);
    }
    if (n == 1) return rt_render_frame(cs[0], cam, spp, max_depth, sums_host, rgb_host, nullptr);
    rt_ctx* c0 = cs[0];
    int rc = check_camera(c0, cam);
    if (rc) return rc;
    const int W = cam->image_width, H = cam->image_height;
    rt_shard_info si;
    rt_shard_layout(W, H, 0, n, &si);
    const size_t eb = elem_bytes(c0), per = (size_t)si.max_shard_tiles * 64 * 3 * eb, npx = (size_t)W * H;
    // each context renders its shard into its own device buffer, on its own stream
    for (int r = 0; r < n; ++r) {
        rt_ctx* c = cs[r];
        HIPCHK(c0, hipSetDevice(c->device));
        if ((rc = grow(c, &c->d_shard, &c->shard_cap, per))) return rc;
        if ((rc = rt_render(c, cam, spp, max_depth, r, n, c->d_shard, nullptr, nullptr)) != RT_OK) {
            if (c != c0) c0->err = std::string("context ") + std::to_string(r) + ": " + c->err;
            return rc;
        }
    }
    // gather to ctxs[0]'s device: it waits for each shard's render, then copies it
    HIPCHK(c0, hipSetDevice(c0->device));
    for (int r = 1; r < n; ++r) {
        int can = 0;
        if (cs[r]->device != c0->device && hipDeviceCanAccessPeer(&can, c0->device, cs[r]->device) == hipSuccess &&
            can) {
            const hipError_t e = hipDeviceEnablePeerAccess(cs[r]->device, 0);   // direct xGMI copies
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
                return fail(c0, RT_ERR_HIP, "peer access %d -> %d: %s", c0->device, cs[r]->device,
                            hipGetErrorString(e));
            (void)hipGetLastError();
        }
    }
    if ((rc = grow(c0, &c0->d_gather, &c0->gather_cap, per * (size_t)n))) return rc;
    if ((rc = grow(c0, &c0->d_frame, &c0->frame_cap, npx * 3 * eb))) return rc;
    if ((rc = grow(c0, (void**)&c0->d_rgb, &c0->rgb_cap, npx * 3 * 4))) return rc;
    if (c0->comm) {
        // RCCL: one grouped ncclGather, rank r on context r's stream after its render
        if ((rc = rt_comm_gather_group(cs, n, per / eb, c0->d_gather))) return rc;
    } else {
        for (int r = 0; r < n; ++r) {
            rt_ctx* c = cs[r];
            HIPCHK(c0, hipStreamWaitEvent(c0->stream, c->ev1, 0));   // ev1: end of that context's render
            void* dst = (char*)c0->d_gather + (size_t)r * per;
            if (c->device == c0->device)
                HIPCHK(c0, hipMemcpyAsync(dst, c->d_shard, per, hipMemcpyDeviceToDevice, c0->stream));
            else
                HIPCHK(c0, hipMemcpyPeerAsync(dst, c0->device, c->d_shard, c->device, per, c0->stream));
        }
    }
    HIPCHK(c0, launch_unshard(c0->d_gather, c0->d_frame, (int)eb, 3, W, H, si.tiles_x, n, si.max_shard_tiles,
                              c0->stream));
    if (rgb_host) HIPCHK(c0, launch_quantize(c0->d_frame, (int)eb, c0->d_rgb, npx * 3, spp, c0->stream));
    if (sums_host) HIPCHK(c0, hipMemcpyAsync(sums_host, c0->d_frame, npx * 3 * eb, hipMemcpyDeviceToHost, c0->stream));
    if (rgb_host) HIPCHK(c0, hipMemcpyAsync(rgb_host, c0->d_rgb, npx * 3 * 4, hipMemcpyDeviceToHost, c0->stream));
    HIPCHK(c0, hipStreamSynchronize(c0->stream));
    return RT_OK;
}

static int trace_rays(rt_ctx* c, const void* rays, int n, rt_hit* hits, void* stream, unsigned long long* diag) {
    if (!c) return RT_ERR_INVALID;
    if (!c->has_scene) return fail(c, RT_ERR_NO_SCENE, "rt_trace_rays before rt_upload_scene");
    if (n < 0 || (n > 0 && (!rays || !hits))) return fail(c, RT_ERR_INVALID, "rt_trace_rays: %d rays, rays %p, hits %p", n, rays, hits);
    HIPCHK(c, hipSetDevice(c->device));
    RenderParams P;
    rt_camera cam{};
    cam.image_width = cam.image_height = 1;
    fill_params(c, &cam, 1, 1, P);
    P.nodes = c->d_nodes;   // (the time-binned copies are a render-kernel option)
    P.diag = diag;
    const size_t lds = lds_scene_bytes_at(c, TRACE_BLOCK) +
                       (c->n_mnodes > 0 ? (size_t)TRACE_BLOCK * (size_t)P.mstack * 4
                                        : 0);
    if (lds > 160 * 1024) return fail(c, RT_ERR_LIMIT, "rt_trace_rays needs %zu B of LDS per workgroup", lds);
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    HIPCHK(c, hipEventRecord(c->ev0, st));
    const hipError_t e = c->precision == RT_PREC_F64 ? launch_trace_f64(P, lds, st, rays, n, hits, c->d_remap)
                                                     : launch_trace_f32(P, lds, st, rays, n, hits, c->d_remap, diag != nullptr);
    if (e != hipSuccess) return fail(c, RT_ERR_HIP, "trace launch: %s", hipGetErrorString(e));
    HIPCHK(c, hipEventRecord(c->ev1, st));
    c->timed = true;
    return RT_OK;
}

int rt_trace_rays(rt_ctx* c, const void* rays, int n, rt_hit* hits, void* stream) {
    return trace_rays(c, rays, n, hits, stream, nullptr);
}

int rt_trace_rays_diag(rt_ctx* c, const void* rays, int n, rt_hit* hits, uint64_t counters[4]) {
    if (!c || !counters) return RT_ERR_INVALID;
    if (c->precision != RT_PREC_F32 || c->n_mnodes > 0)
        return fail(c, RT_ERR_INVALID, "rt_trace_rays_diag instruments the fp32 sphere-scene kernel");
    unsigned long long* d = nullptr;
    HIPCHK(c, hipMalloc((void**)&d, DIAG_SLOTS * sizeof(unsigned long long)));
    hipError_t e = hipMemsetAsync(d, 0, DIAG_SLOTS * sizeof(unsigned long long), c->stream);
    int rc = e == hipSuccess ? trace_rays(c, rays, n, hits, c->stream, d) : RT_OK;
    unsigned long long h[DIAG_SLOTS] = {};
    if (e == hipSuccess && rc == RT_OK) e = hipMemcpyAsync(h, d, sizeof(h), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess && rc == RT_OK) e = hipStreamSynchronize(c->stream);
    (void)hipFree(d);
    if (rc) return rc;
    if (e != hipSuccess) return fail(c, RT_ERR_HIP, "trace diag: %s", hipGetErrorString(e));
    for (int k = 0; k < 4; ++k) counters[k] = h[2 + k];   // inner_it, inner_act, leaf_it, leaf_act
    return RT_OK;
}

static_assert(DIAG_SLOTS == RT_DIAG_SLOTS, "diag slots");
int rt_render_diag(rt_ctx* c, const rt_camera* cam, int spp, int max_depth, uint64_t counters[16]) {
    return rt_render_diag_ex(c, cam, spp, max_depth, counters, 16);
}

int rt_render_diag_ex(rt_ctx* c, const rt_camera* cam, int spp, int max_depth, uint64_t* counters, int n) {
    if (!c || !counters || n < 1 || n > DIAG_SLOTS)
        return c ? fail(c, RT_ERR_INVALID, "rt_render_diag_ex: counters and 1 <= n <= %d", DIAG_SLOTS) : RT_ERR_INVALID;
    if (c->precision != RT_PREC_F32) return fail(c, RT_ERR_INVALID, "rt_render_diag instruments the fp32 kernel");
    if (!c->has_scene) return fail(c, RT_ERR_NO_SCENE, "no scene");
    if (spp > FIX_LAUNCH_SAMPLES) return fail(c, RT_ERR_INVALID, "rt_render_diag: spp <= %d", FIX_LAUNCH_SAMPLES);
    int rc = check_camera(c, cam);
    if (rc) return rc;
    HIPCHK(c, hipSetDevice(c->device));
    rt_shard_info si;
    rt_shard_layout(cam->image_width, cam->image_height, 0, 1, &si);
    if ((rc = grow(c, &c->d_shard, &c->shard_cap, (size_t)si.num_tiles * 64 * 3 * 4))) return rc;
    unsigned long long* d = nullptr;
    HIPCHK(c, hipMalloc((void**)&d, DIAG_SLOTS * sizeof(unsigned long long)));
    hipError_t e = hipMemsetAsync(d, 0, DIAG_SLOTS * sizeof(unsigned long long), c->stream);
    // the persistent kernel of rt_render, instrumented (block 512, <= 64 VGPRs; the
    // coherent-primary kernel at the context's block, 512 or 1024; the ray pool at 512)
    // exactly the kernel rt_render runs for this tuning, instrumented (RT_DIAG_VARIANTS);
    // a tuning with no instrumented build is refused (RT_ERR_INVALID), never substituted
    c->diag_buf = d;
    if (e == hipSuccess) rc = rt_render(c, cam, spp, max_depth, 0, 1, c->d_shard, nullptr, nullptr);
    c->diag_buf = nullptr;
    if (e == hipSuccess && rc == RT_OK)
        e = hipMemcpyAsync(counters, d, (size_t)n * sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess && rc == RT_OK) e = hipStreamSynchronize(c->stream);
    (void)hipFree(d);
    if (rc) return rc;
    if (e != hipSuccess) return fail(c, RT_ERR_HIP, "diag render: %s", hipGetErrorString(e));
    return RT_OK;
}

int rt_trace_tape(rt_ctx* c, const double ray[7], int depth, const double* tape, int tape_len, double out[3],
                  int* used) {
    if (!c || !ray || !out || !used || tape_len < 0 || (tape_len > 0 && !tape)) return RT_ERR_INVALID;
    if (!c->has_scene) return fail(c, RT_ERR_NO_SCENE, "rt_trace_tape before rt_upload_scene");
    if (c->precision != RT_PREC_F64) return fail(c, RT_ERR_INVALID, "rt_trace_tape needs an RT_PREC_F64 context");
    if (depth > 64) return fail(c, RT_ERR_LIMIT, "depth %d > 64", depth);
    HIPCHK(c, hipSetDevice(c->device));
    int rc;
    if ((rc = grow(c, (void**)&c->d_tape, &c->tape_cap, (size_t)(tape_len > 0 ? tape_len : 1) * sizeof(double))))
        return rc;
    if (tape_len)
        HIPCHK(c, hipMemcpyAsync(c->d_tape, tape, (size_t)tape_len * sizeof(double), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->d_small, ray, 7 * sizeof(double), hipMemcpyHostToDevice, c->stream));
    rt_camera dummy{};
    dummy.image_width = dummy.image_height = 1;
    RenderParams P;
    fill_params(c, &dummy, 1, depth, P);
    HIPCHK(c, launch_tape_f64(P, depth, c->d_small, c->d_tape, tape_len, c->d_small + 8, c->d_used, c->stream));
    HIPCHK(c, hipMemcpyAsync(out, c->d_small + 8, 3 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(used, c->d_used, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return RT_OK;
}

}  // extern "C"

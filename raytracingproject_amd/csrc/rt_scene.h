// rt_scene.h -- scene records shared by the host builder (rt_bvh.cpp), the C ABI
// (rt_abi.cpp) and the kernels (rt_render_*.hip).  Plain structs, no HIP types.
#pragma once
#include <cstdint>

namespace rtx {

// ---- BVH node: the two children's boxes live in the parent (64 B, four 16-B LDS
// reads), so one node fetch tests both children and pushes only the far one.
// ref encoding (16 bit, so the per-lane LDS traversal stack is 2 B per entry):
//   inner node : index                         (0 .. 0x7fff)
//   leaf       : 0x8000 | (count-1) << 11 | first   (first < 2048, count 1..16)
//   empty      : REF_EMPTY (never stored by build_bvh: a single-leaf root holds the leaf twice)
constexpr uint32_t REF_LEAF = 0x8000u;
constexpr uint32_t REF_EMPTY = 0xffffu;
constexpr uint32_t REF_NONE = 0xffffffffu;   // traversal sentinel (never stored in a node)
constexpr int LEAF_MAX = 16;
constexpr int MAX_LEAF_FIRST = 2048;
constexpr int MAX_INNER = 0x8000;
constexpr int STACK_MAX = 32;   // deepest BVH the LDS stack is sized for

struct alignas(16) Node {
    float lo0[3]; uint32_t ref0;
    float hi0[3]; uint32_t ref1;
    float lo1[3]; uint32_t pad0;
    float hi1[3]; uint32_t pad1;
};
static_assert(sizeof(Node) == 64, "node is 64 B");


// ---- uniform grid over the tree's spheres (fp32 kernels, TRAV_GRID): an alternative to
// the sphere BVH for scenes of many similar spheres spread over a region (main.cpp:18-44's
// 22 x 22 field).  The header travels in the kernel arguments (RenderParams::grid: uniform
// values, scalar registers); one buffer is copied to LDS where the BVH nodes would go (no
// traversal stack; the sphere records follow it): one word per cell (x fastest) = its
// list's first entry | end entry << GRID_POS_BITS, with an empty x-y layer of cells before
// and after the grid (a step out of it reads an empty cell: no bounds test), then the lists:
// for each cell the byte offsets (from the buffer's start, 32 bits) of the sphere records
// whose swept box, padded beyond the rounding of the kernel's plane distances, meets the
// cell.  List positions are byte offsets from the buffer's start, which the kernels copy to
// LDS address 0, so a position is the entry's LDS address (r06; before, first | count << 20
// with word positions from the lists' start: one scalar base more, spilled, an add per step
// and a shift-and-add per test, C3 +1.6 % and +0.6 %, profiles/r06/r06w, r06an).  The front
// spheres [0, n_front) are never listed.
// After the lists (at slab_off, 16-B aligned): n_slab + 1 boxes, stored per axis as (lo, hi)
// float pairs -- x pairs for boxes 0..n_slab, then y, then z -- so that lanes reading
// different boxes hit different LDS banks (8-B stride).  Box k < n_slab bounds where the listed spheres are at the times of slab k, [k, k + 1)
// / n_slab (with a margin), padded as the cells' boxes; box n_slab is the grid box.  A ray
// is clipped to its time's slab box before the walk (times outside [0, 1]: the grid box):
// the cells are the same for every time, only the stretch of them walked gets shorter
// (main.cpp's spheres bounce up to 0.5 over the shutter, so at one time the field is
// thinner than its swept box).
struct alignas(16) GridHdr {
    float lo[3];       // grid box (the padded swept boxes' union)
    float inv_cs[3];   // 1 / cell size
    float cs[3];       // cell size
    int res[3];        // cells per axis
    uint32_t n_cells;  // res[0] * res[1] * res[2]
    float hi[3];
    uint32_t slab_off; // byte offset of the time-slab boxes in the buffer
    float slab_k;      // (float)n_slab
    int n_slab;        // time slabs (1 .. GRID_SLAB_MAX)
    // The walk's reach (r06, host only -- the kernels never read it): a launch whose rays
    // can start beyond +-far_o on some axis renders with the tree instead (rt_abi.cpp
    // grid_reach_ok).  Past it the fp32 rounding of the walk's plane distances, which grows
    // as ~(steps + 16) 2^-23 (|o| + the grid's largest coordinate), could exceed the padding
    // of the listed boxes, and far enough out (~2^24 cells) a step no longer moves its plane
    // distance at all.
    float far_o;
};
static_assert(sizeof(GridHdr) == 80, "GridHdr");
constexpr int GRID_SLAB_MAX = 64;
constexpr int GRID_POS_BITS = 16;   // a cell word's list positions (byte offsets; the buffer is <= 48 KB)
constexpr uint32_t GRID_POS_MASK = (1u << GRID_POS_BITS) - 1u;
constexpr int GRID_CELL_MAX = 4095;              // spheres listed in one cell at most
constexpr size_t GRID_MAX_BYTES = 48 * 1024;     // the whole buffer (LDS)

// material types (material.h:15, 31, 48); same values as RT_LAMBERTIAN.. in rt_hip.h
constexpr uint32_t MAT_LAMBERTIAN = 0, MAT_METAL = 1, MAT_DIELECTRIC = 2;

// meta word of a sphere record: material index | type << 24 | moving << 30
constexpr uint32_t META_MAT_MASK = 0x00ffffffu;
inline constexpr uint32_t make_meta(uint32_t mat, uint32_t type, uint32_t moving) {
    return (mat & META_MAT_MASK) | (type << 24) | (moving << 30);
}

// Sphere record in LDS, per precision: center, radius, center_vec, meta.
struct alignas(16) SphereF { float c[3]; float r; float cv[3]; uint32_t meta; };
struct alignas(16) SphereD { double c[3]; double r; double cv[3]; uint32_t meta; float inv_r; };  // inv_r: fp32 path
static_assert(sizeof(SphereF) == 32, "SphereF");
static_assert(sizeof(SphereD) == 64, "SphereD");
// fp32 kernels: the big spheres (the R = 1000 ground) relative to p0, the point of the
// sphere nearest the rest of the scene, with n the outward normal there: for f = o - c =
// q + r n (q = o - p0, small), |f|^2 - r^2 = q.q + 2 r (n.q) and f.d = q.d + r (n.d)
// have no catastrophic cancellation in fp32 (rt_device.h closest_hit)
struct alignas(16) BigF { float p0[3]; float r; float n[3]; float inv_r; float cv[3]; uint32_t meta; };
static_assert(sizeof(BigF) == 48, "BigF");

// Material record: albedo.rgb and the type's scalar (metal fuzz, dielectric ir).
struct alignas(16) MatF { float p[4]; };
struct alignas(16) MatD { double p[4]; };

// ---- mesh path (HBM-resident): 32-bit refs, same 64-B two-child node layout.
//   inner: index (< 2^31); leaf: MREF_LEAF | (count-1) << 24 | first (first < 2^24)
constexpr uint32_t MREF_LEAF = 0x80000000u;
constexpr uint32_t MREF_EMPTY = 0xffffffffu;
constexpr int MESH_LEAF_MAX = 8;
constexpr int MESH_MAX_TRIS = 1 << 24;
constexpr int MESH_STACK_MAX = 64;       // per-lane scratch stack entries
constexpr int MESH_TOP_MAX = 4096;       // breadth-first prefix of the node array (LDS-cacheable)
constexpr int MESH_HIT_BASE = 0x40000000;  // Hit::id of triangle k = MESH_HIT_BASE | k

// Mesh BVH node: 4 children, SoA boxes (one 128-B L2 line), refs as MREF_* (EMPTY slots
// carry an inverted box).  4-wide halves the dependent node-load chain of a binary tree.
struct alignas(16) Node4 {
    float lox[4], loy[4], loz[4], hix[4], hiy[4], hiz[4];
    uint32_t ref[4];
    uint32_t pad[4];
};
static_assert(sizeof(Node4) == 128, "Node4 layout");

// Triangle records, BVH leaf order.
//  fp64 (TriD, 80 B): v0, e1 = v1 - v0, e2 = v2 - v0 (in fp64), meta (material | type << 24):
//    Moller-Trumbore in the oracle's operation order (rt_oracle.c tri_hit), bit-exact.
//  fp32 (TriF, 48 B, r05): the three vertices, each rounded once from the caller's fp64
//    vertex, so a vertex shared by several triangles has the same fp32 coordinates in every
//    one of them -- what the watertight test (rt_device.h tri_wt) needs -- and the facet
//    normal n = (v1 - v0) x (v2 - v0), computed in fp64 and rounded once (the plane
//    distance, the orientation of the edge values and the shading normal); the meta words
//    live in a side array (RenderParams::tmeta), read only when a hit is shaded.  (A
//    packed 36-B record without n measured the same as r04's 48-B one; n saves the test
//    12 VALU, r05 A/B.)  The if-if mesh loop reads 112 B from a leaf's first triangle, so
//    the device array carries TRIF_SLACK bytes past the last record.
struct alignas(16) TriF { float v0[3]; float v1[3]; float v2[3]; float n[3]; };
struct alignas(16) TriD { double v0[3]; double e1[3]; double e2[3]; uint32_t meta; uint32_t pad; };
static_assert(sizeof(TriF) == 48, "TriF");
static_assert(sizeof(TriD) == 80, "TriD");
constexpr size_t TRIF_SLACK = 128;

// Spheres at least this large (the R=1000 ground of main.cpp:15) stay out of the BVH
// and are tested in fp64 in every precision: in fp32, c = |oc|^2 - r^2 at |oc| ~ r
// = 1000 cancels catastrophically (sphere.h:35), SURVEY.md §7 "fp32 precision".
constexpr double BIG_RADIUS = 64.0;

// Scene coordinates (centres, motion vectors, radii, vertices) must be finite and within
// +-COORD_MAX: the builders' SAH areas and the fp32 node boxes stay finite (checked by the
// C ABI and by both builders; RT_ERR_LIMIT otherwise).
constexpr double COORD_MAX = 1e30;
inline bool coord_ok(double x) { return x >= -COORD_MAX && x <= COORD_MAX; }   // false for NaN
constexpr int MAX_BIG = 8;

}  // namespace rtx

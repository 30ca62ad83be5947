// rt_bvh.h -- host BVH builder.  The reference's bvh_node (src/bvh.h:8-32) has an empty
// constructor (:12-14) and a hit() that does not compile (:17, undeclared `box`); it is
// completed here as what its hit() describes: a binary AABB tree (aabb.h:6-53) whose
// traversal visits children and shrinks t_max to the closest hit (bvh.h:16-24).  The
// tree is built with a full-sweep SAH and flattened into the two-children-per-node
// layout of rt_scene.h for LDS-resident traversal.
#pragma once
#include <string>
#include <vector>

#include "../../include/rt_hip.h"
#include "rt_scene.h"

namespace rtx {

struct BvhParams {
    double cost_traverse = 1.0;
    double cost_intersect = 1.0;
    int max_leaf = 4;
    int front = 0;                // the `front` largest spheres are tested before the tree, outside it
                                  // (-1: those with radius >= 4x the median, at most 8)
};

struct BuiltBvh {
    std::vector<Node> nodes;      // nodes[0] is the root (empty when no BVH prims)
    std::vector<int> order;       // BVH position -> input sphere index
    std::vector<int> big;         // input indices of the spheres kept out of the BVH
    int front = 0;                // order[0, front): spheres tested before the tree (not in it)
    int depth = 0;                // inner-node depth (LDS stack entries needed)
    int leaves = 0;
};

// Returns false (with err) if the scene exceeds the encodable limits of rt_scene.h.
bool build_bvh(const rt_sphere* spheres, int n, const BvhParams& p, BuiltBvh& out, std::string& err);

// Uniform grid over the fp32 sphere records [first, n) (rt_scene.h GridHdr): the header and
// the LDS buffer `out` (cell words, then sphere positions; a multiple of sizeof(Node) bytes:
// it takes the nodes' place in LDS).  density = cells per sphere; returns false (out empty)
// when the scene does not suit a grid: no spheres, a cell listing more than GRID_CELL_MAX,
// more than 4 list entries per sphere at every resolution tried (spheres much larger than
// the cells), more than half the cells empty (clustered spheres: the tree skips the empty
// space), more than 8 spheres per occupied cell, or a buffer over GRID_MAX_BYTES at the
// coarsest resolution.
// The lists hold record byte offsets from the buffer's start: the kernel's sphere records of
// rec_bytes each follow the buffer (padded to sizeof(Node)) in LDS.  slabs (1 ..
// GRID_SLAB_MAX): time slabs of the clip boxes after the lists (rt_scene.h GridHdr); a
// sphere is at c + t cv at time t (cv is zero for stationary spheres in both precisions).
bool build_sphere_grid(const SphereF* spheres, int first, int n, double density, int slabs, int rec_bytes,
                       GridHdr& hdr, std::vector<unsigned char>& out);

struct MeshBvh {
    std::vector<Node> nodes;      // binary tree (build stage), nodes[0] is the root
    std::vector<Node4> nodes4;    // the 4-wide tree the kernel traverses, nodes4[0] is the root
    std::vector<int> order;       // BVH position -> input triangle index
    int depth = 0, depth4 = 0, leaves = 0;
};

// Binned-SAH BVH over triangles (32-bit refs, rt_scene.h MREF_*).  cost_traverse is
// the node cost relative to one triangle test.  The binary tree is then collapsed into a
// 4-wide tree (each node adopts grandchildren, largest box first).  Node4 order: the first
// min(MESH_TOP_MAX, n) nodes breadth-first (the tree top, cacheable in LDS as a prefix),
// the rest depth-first (children near their parent).
bool build_mesh_bvh(const rt_triangle* tris, int n, int max_leaf, double cost_traverse, MeshBvh& out,
                    std::string& err);

// Float box of one sphere over time in [0,1] (sphere.h:12-13, 22-25), rounded outward
// and padded so that the fp32 slab test is conservative.
void sphere_box(const rt_sphere& s, float lo[3], float hi[3]);

}  // namespace rtx

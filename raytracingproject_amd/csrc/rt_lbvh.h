// rt_lbvh.h -- GPU BVH build for meshes (rt_lbvh.hip), called by rt_upload_scene_ex when
// rt_tuning.mesh_builder is RT_MESH_BUILD_GPU (treelet-restructured) or RT_MESH_BUILD_GPU_LBVH.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "../../include/rt_hip.h"
#include "rt_scene.h"

namespace rtx {

struct LbvhInput {
    const rt_triangle* tris;     // device, n records
    int n;
    const uint32_t* mat_type;    // device, material index -> MAT_* type
    double lo[3], inv[3];        // centroid bounds: Morton cell = (c - lo) * inv in [0, 1]
    int max_leaf;                // triangles per leaf (1..MESH_LEAF_MAX)
    bool f64;                    // TriD records (else TriF)
    int treelet_rounds = 0;      // rounds of treelet restructuring (rt_treelet.h; 0: the plain Morton tree)
};

// Scratch kept by the context between builds (grown on demand).
struct LbvhScratch {
    void *keys = nullptr, *child = nullptr, *box = nullptr, *index = nullptr, *sort_tmp = nullptr, *scan_tmp = nullptr;
    size_t keys_cap = 0, child_cap = 0, box_cap = 0, index_cap = 0, sort_tmp_cap = 0, scan_tmp_cap = 0;
    void release() {
        for (void* p : {keys, child, box, index, sort_tmp, scan_tmp}) (void)hipFree(p);
        *this = LbvhScratch();
    }
};

struct LbvhOutput {
    Node4* nodes;        // device, capacity nodes_cap (n - 1 suffices)
    int nodes_cap;
    void* tris;          // device, n TriF / TriD records in leaf order
    uint32_t* tmeta;     // device, n meta words (fp32: TriF carries none), else unused
    int node_count = 0, depth4 = 0, leaves = 0;
};

// Builds on `stream` and synchronises it (the host needs the node count).
hipError_t lbvh_build(const LbvhInput& in, LbvhScratch& ws, LbvhOutput& out, hipStream_t stream);
// After a build of n triangles: the device array of input triangle indices in leaf order
// (in the scratch; valid until the next build).
inline const uint32_t* lbvh_sorted_index(const LbvhScratch& ws, int) { return (const uint32_t*)ws.keys; }

}  // namespace rtx

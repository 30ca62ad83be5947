// rt_ctx.h -- the context behind the C ABI (include/rt_hip.h) and the helpers its
// implementation files share (rt_abi.cpp: scene, render, frames; rt_comm.cpp: RCCL).
// Internal: not installed, not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <array>
#include <string>
#include <vector>

#include "../../include/rt_hip.h"
#include "rt_device.h"
#include "rt_lbvh.h"

using namespace rtx;

struct rt_ctx {
    int device = 0;
    int precision = RT_PREC_F32;
    uint64_t seed = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool timed = false;
    std::string err;
    // measured best (tools/sweep.py, tools/mesh_sweep.py; profiles/r01)
    rt_tuning tuning{1024, 6, 1.0, 0.25, 8, RT_TRAV_DEFAULT, 2, -1, 2.0, 65536, 16384, RT_MESH_BUILD_HOST, -1, -1, 0, 32, 8.0, 20.0, 48, 0, 0, -1, 2.0, 32};

    // scene (device)
    bool has_scene = false;
    Node* d_nodes = nullptr;
    void* d_sph = nullptr;
    void* d_mat = nullptr;
    SphereD* d_big = nullptr;
    BigF* d_bigf = nullptr;     // the big spheres relative to their near points (fp32 kernels)
    int n_nodes = 0, n_sph = 0, n_mat = 0, n_big = 0, depth = 0, leaves = 0, n_input = 0;
    int n_front = 0;   // spheres [0, n_front) are tested before the BVH (rt_tuning.front_spheres)
    float box_extent = 0.f;   // bound of |coordinate| over the node boxes (RenderParams::box_extent)
    void* d_grid = nullptr;     // fp32: the uniform sphere grid (GridHdr ...), when the scene suits one
    int grid_nodes = 0;         // its size in sizeof(Node) units (it takes the nodes' LDS region)
    GridHdr grid_hdr{};         // its header (RenderParams::grid)
    int grid_entries = 0;       // sphere references over its cells
    double grid_density = 0.0;  // the sphere_grid_density it was built with (rt_scene_info, ABI 10)
    // r06: where a launch's rays can start (grid_reach_ok, rt_abi.cpp): the box of the
    // geometry a ray can leave from anywhere on it -- spheres outside the big class, triangles,
    // and big spheres that refract or move -- and the static opaque big spheres (centre,
    // radius), which a ray only reaches within its tangent distance
    double reach_lo[3] = {0, 0, 0}, reach_hi[3] = {0, 0, 0};
    std::vector<std::array<double, 4>> reach_big;
    bool grid_blocked = false;  // the current launch's rays could start beyond grid_hdr.far_o: the tree
    int* d_remap = nullptr;     // rt_trace_rays: kernel id slot -> input index (spheres | big | triangles)
    Node4* d_mnodes = nullptr;  // mesh BVH (4-wide) + triangles (HBM-resident)
    void* d_tris = nullptr;
    uint32_t* d_tmeta = nullptr;   // fp32: per-triangle meta words (leaf order), beside the 48-B TriF records
    int n_mnodes = 0, n_tris = 0, mdepth = 0, mleaves = 0;
    float mbox[6] = {};         // the mesh's box (lo xyz, hi xyz): union of the root's child boxes
    LbvhScratch lbvh;           // GPU mesh-BVH build scratch

    // scratch for the host-in/host-out paths (grown on demand, outside timed code)
    void* d_shard = nullptr;
    size_t shard_cap = 0;
    void* d_frame = nullptr;
    size_t frame_cap = 0;
    uint32_t* d_segs = nullptr;
    size_t segs_cap = 0;
    uint32_t* d_segs_frame = nullptr;
    size_t segs_frame_cap = 0;
    int32_t* d_rgb = nullptr;
    size_t rgb_cap = 0;
    double* d_tape = nullptr;
    size_t tape_cap = 0;
    double* d_small = nullptr;  // ray7 + out3
    int* d_used = nullptr;
    void* d_samples = nullptr;  // per-sample radiance of chunked launches
    uint32_t* d_queue64 = nullptr;   // fp64 persistent lanes (f64_kernel 3): work-queue control block
    size_t samples_cap = 0;
    void* d_gather = nullptr;   // rt_render_frame_multi: all contexts' shards
    size_t gather_cap = 0;

    // fp32 fixed-point pixel sums (RenderParams::accum), one slot per output buffer the
    // context renders into: rt_render_range(accumulate=1) continues a slot exactly.
    struct Accum {
        const void* out = nullptr;   // the out_sums buffer these sums belong to
        int W = 0, H = 0, shard = 0, nshards = 0;
        long long* acc = nullptr;    // npx * 3
        uint32_t* flags = nullptr;   // npx
        uint32_t* queue = nullptr;   // persistent-lane work counter of launches into this buffer
        unsigned long long* accp = nullptr;   // npx * 2: one launch's packed sums
        size_t acc_cap = 0, flags_cap = 0, accp_cap = 0;
        uint64_t used = 0;           // LRU stamp
    };
    static constexpr int ACCUM_SLOTS = 4;
    Accum accum[ACCUM_SLOTS];
    uint64_t accum_clock = 0;
    int n_cu = 0;                  // compute units of the device
    unsigned long long* diag_buf = nullptr;   // set only inside rt_render_diag: the instrumented kernel runs

    // 8-bit host-bound frames (rt_finish_frame_u8 / rt_render_frame_u8): device frame and
    // a pinned host staging buffer (DMA-able, so the copy runs at full PCIe rate)
    uint8_t* d_rgb8 = nullptr;
    size_t rgb8_cap = 0;
    void* h_pinned = nullptr;
    size_t pinned_cap = 0;

    // RCCL communicator (rt_comm_init_rank / rt_comm_init_all): rank comm_rank of comm_size
    void* comm = nullptr;   // ncclComm_t
    int comm_rank = 0, comm_size = 0;
    bool comm_nonblocking = false;   // made by rt_comm_init_rank[_timeout] (ncclConfig_t.blocking = 0)
};

namespace rtx_abi {

inline int fail(rt_ctx* c, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (c) c->err = buf;
    return code;
}

#define HIPCHK(ctx, expr)                                                                              \
    do {                                                                                               \
        hipError_t e_ = (expr);                                                                        \
        if (e_ != hipSuccess) return fail(ctx, RT_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_));   \
    } while (0)

inline int grow(rt_ctx* c, void** p, size_t* cap, size_t bytes) {
    if (*cap >= bytes && *p) return RT_OK;
    if (*p) HIPCHK(c, hipFree(*p));
    *p = nullptr;
    *cap = 0;
    HIPCHK(c, hipMalloc(p, bytes ? bytes : 16));
    *cap = bytes;
    return RT_OK;
}

}  // namespace rtx_abi

// rt_comm.cpp: drop the context's communicator (rt_destroy); the grouped gather of
// rt_render_frame_multi (every context rank r of n, shards in their d_shard)
void rt_comm_release(rt_ctx* c);
int rt_comm_gather_group(rt_ctx** cs, int n, size_t elems, void* gathered);

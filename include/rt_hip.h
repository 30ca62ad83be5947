/*
 * rt_hip.h -- C ABI of the MI355X path tracer (librt_hip.so).
 *
 * The reference has no FFI: its boundary is the C++ header API.  The
 * entry points below are what that API needs from a device backend; each cites the
 * reference interface it replaces.  include/rt/camera.h (C++ mirror of the reference
 * headers) is the drop-in caller; INTEGRATION.md shows the binding a maintainer adds.
 *
 * Conventions: plain pointers and sizes, no C++/torch types.  Every int-returning call
 * returns RT_OK (0) or a negative RT_ERR_* code; rt_last_error() has the message.
 * Device pointers are hipMalloc'd (or torch CUDA tensors); `stream` is a hipStream_t or
 * NULL for the context's own stream.  One context per process and GPU (the multi-GPU
 * path runs one process per GPU).
 */
#ifndef RT_HIP_H
#define RT_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 11

enum {
    RT_OK = 0,
    RT_ERR_INVALID = -1,   /* bad argument                                  */
    RT_ERR_HIP = -2,       /* a HIP runtime call failed                     */
    RT_ERR_NO_SCENE = -3,  /* rt_render before rt_upload_scene              */
    RT_ERR_LIMIT = -4,     /* scene/BVH/depth beyond what the kernel holds */
    RT_ERR_COMM = -5       /* an RCCL call failed (message: ncclGetErrorString) */
};

enum { RT_LAMBERTIAN = 0, RT_METAL = 1, RT_DIELECTRIC = 2 };  /* material.h:15,31,48 */
enum { RT_PREC_F32 = 0, RT_PREC_F64 = 1 };

/* sphere.h:9-28.  center_vec = center2 - center1 exactly as sphere.h:27 computes it;
 * zero (and moving = 0) for a stationary sphere.  64 bytes. */
typedef struct {
    double center[3];
    double radius;
    double center_vec[3];
    int32_t mat;      /* index into the material array */
    int32_t moving;
} rt_sphere;

/* lambertian(albedo) material.h:17, metal(albedo, fuzz) :33 (fuzz clamped to 1 here
 * as there), dielectric(ir) :50.  48 bytes. */
typedef struct {
    int32_t type;
    int32_t pad;
    double albedo[3];
    double fuzz;
    double ir;
} rt_material;

/* A triangle (mesh path; the reference has no triangle primitive):
 * vertices in counter-clockwise order as seen from the outward side, material index.
 * 80 bytes. */
typedef struct {
    double v0[3], v1[3], v2[3];
    int32_t mat;
    int32_t pad;
} rt_triangle;

/* OBJ geometry as loaded by rt_obj_load: num_vertices xyz doubles and num_triangles
 * index triples (0-based) after fan triangulation of num_faces faces. */
typedef struct {
    int32_t num_vertices, num_faces, num_triangles, pad;
    double* vertices;
    int32_t* indices;
} rt_obj_mesh;

/* The camera AFTER camera::initialize() (camera.h:52-85): the derived members of
 * camera.h:117-125 plus defocus_angle (camera.h:25, tested in get_ray :94). */
typedef struct {
    int32_t image_width, image_height;
    double center[3];
    double pixel00_loc[3];
    double pixel_delta_u[3];
    double pixel_delta_v[3];
    double defocus_disk_u[3];
    double defocus_disk_v[3];
    double defocus_angle;
} rt_camera;

/* camera.h:15-26: the public fields a caller sets before render(). */
typedef struct {
    double aspect_ratio;
    int32_t image_width, samples_per_pixel, max_depth, pad;
    double vfov;
    double lookfrom[3], lookat[3], vup[3];
    double defocus_angle, focus_dist;
} rt_camera_desc;

/* Framebuffer tiling for the multi-GPU split: 8x8-pixel tiles in
 * row-major tile order; tile t belongs to shard t % num_shards.  A shard buffer holds
 * its tiles back to back, 64 pixels x 3 channels each, pixel (x%8, y%8) at lane
 * (y%8)*8 + x%8. */
typedef struct {
    int32_t tile_w, tile_h;
    int32_t tiles_x, tiles_y, num_tiles;
    int32_t shard, num_shards, shard_tiles, max_shard_tiles;
} rt_shard_info;

typedef struct {
    int32_t num_spheres, num_materials;
    int32_t bvh_nodes, bvh_depth, bvh_leaves, big_spheres;
    int32_t lds_bytes;
    int32_t precision;
    int32_t num_triangles, mesh_nodes, mesh_depth, mesh_leaves;   /* mesh BVH: 4-wide nodes, their depth */
    int32_t render_block;   /* threads per workgroup the render kernel uses for this scene */
    int32_t render_traversal;   /* traversal flags of the fp32 kernel this scene runs (the tuning's, with 128
                                   added where the LDS sums would cost occupancy, 8192 added for fp32 mesh
                                   scenes unless 16384 was asked for, 131072 added to 65536 on a grid one
                                   cell tall in y unless 262144 was asked for) */
    int32_t render_waves_per_eu;    /* register-budget key of that fp32 kernel (waves_per_eu, or for meshes the
                                       resolved mesh_waves_per_eu: 0 or 6); 0 for fp64 (ABI 7) */
    int32_t render_mesh_lds_stack;  /* mesh traversal stack entries per lane it keeps in LDS (the resolved
                                       mesh_lds_stack); 0 without a mesh (ABI 7) */
    int32_t grid_res[3];    /* the uniform sphere grid's cells per axis (0 0 0: none built; ABI 8) */
    int32_t grid_entries;   /* sphere references listed over its cells */
    /* ABI 10: what the current grid was built with (the tuning's sphere_grid_density and
       sphere_grid_time_slabs at the last rt_upload_scene; 0 without a grid), and its walk's reach:
       the walk is exact and ends for ray origins within +-grid_far_o on every axis (its fp32 plane
       distances lose precision beyond); a launch whose camera or scene could start a ray beyond
       it renders with the sphere tree instead, the same frame (rt_grid_reach).  render_* above
       describe a launch within reach. */
    int32_t grid_time_slabs;
    float grid_far_o;
    double grid_density;
} rt_scene_info;

/* Kernel/BVH tuning (defaults are the measured best).  block: threads
 * per workgroup of the render kernel (fp64 always 256); max_leaf, the SAH costs and the
 * mesh_* build fields shape the BVHs built by the next rt_upload_scene[_ex].  Only the
 * (block, waves_per_eu, traversal) combinations instantiated in rt_render_f32.hip render
 * (rt_set_tuning checks the requested one, rt_render_range the one the scene runs -- the
 * library may add 128 -- with a clear RT_ERR_INVALID); meshes have their own smaller
 * set.  Every combination renders the same pixels bit for bit (the fp32 kernels fuse
 * multiply-adds only within one expression, -ffp-contract=on, so every inlined copy
 * rounds alike); the fp64 path ignores the kernel fields. */
typedef struct {
    int32_t block;
    int32_t max_leaf;
    double cost_traverse, cost_intersect;
    int32_t waves_per_eu;   /* fp32 register budget: 0 = compiler's choice, 4 / 6 / 8 = <= 128 / 80 / 64 VGPRs */
    int32_t traversal;      /* flags: 8 select root, 16 whole-record (b128) LDS reads of nodes and spheres,
                               64 coherent primaries (camera rays traced in per-tile batches), 128 with 64:
                               no LDS pixel sums (set automatically where they would cost occupancy), 512
                               pop culling (a popped stack top whose box starts beyond the closest hit so
                               far is dropped unvisited), 8192 (fp32 mesh scenes; added by the library
                               wherever instantiated) the if-if mesh loop -- each iteration a lane visits
                               one node or tests one leaf, node and triangle loads issued together -- and
                               16384 (mesh scenes) the while-while mesh loop of rounds 1-3 instead,
                               65536 (ABI 8) the uniform sphere grid instead of the sphere BVH -- dropped
                               where rt_upload_scene built no grid (sphere_grid_density 0, or no sphere
                               outside the front list and the ground class); mixed scenes get it in their
                               mesh kernels where instantiated, fp64 through f64_kernel 5 (C3 fp32 48.2 ->
                               38.3 ms, fp64 97.1 -> 81.7 ms; C5 geometry -9.5 %; r05).
                               131072 (ABI 11; added by the library with 65536 wherever the grid is one
                               cell tall in y -- main.cpp's field on its ground -- and the kernel exists:
                               the walk steps in x and z only; C3 -6 %, the same frame) unless 262144
                               (never in a kernel key) asks to keep the 3-D walk; fp64 likewise.
                               32768 (quantised 64-B mesh nodes) was measured slower in r05 and is refused.
                               256 (time-binned sphere trees) and 4096 (an LDS copy of the mesh tree top)
                               were measured slower, removed in ABI 6 and are refused.
                               Default RT_TRAV_DEFAULT with block 1024; the
                               one-path-per-lane kernel is traversal 8 with block 512.  Every combination
                               gives the same frame bit for bit */
    int32_t mesh_max_leaf;  /* triangle BVH: at most this many triangles per leaf (1..8; default 2) */
    int32_t mesh_lds_nodes; /* reserved (-1..4096 accepted, no effect): the LDS tree-top kernels it sized
                               (traversal 4096) were removed in ABI 6 */
    double mesh_cost_traverse;  /* triangle BVH SAH: node cost relative to one triangle test */
    int32_t chunk_waves;    /* reserved (>= 0 accepted, no effect): the one-wave-per-tile F64 kernels 1 / 2
                               whose samples it split were removed in ABI 6; every kernel now runs
                               persistent lanes over the work queue (item_* below) */
    int32_t sample_buffer_mb;  /* F64: cap of the per-sample radiance buffer (MiB) of kernels 3 / 4; longer
                               sample ranges run in passes, each of at most 65535 samples (the coherent
                               kernel's FIFO keeps a sample's index within its pass in 16 bits) */
    int32_t mesh_builder;   /* RT_MESH_BUILD_HOST: binned SAH on the host (best trees); RT_MESH_BUILD_GPU:
                               built on the device -- Morton-code LBVH, then two rounds of treelet
                               restructuring by SAH (r06, ABI 10; fast builds for large or changing
                               meshes); RT_MESH_BUILD_GPU_LBVH: the plain Morton-code LBVH (r03-r05) */
    int32_t mesh_waves_per_eu;  /* register budget of the mesh kernels: -1 = auto (the default: of the
                                   instantiated kernels, the one keeping more waves resident per CU, equal
                                   occupancy keeping the unspilled one), 0 = the compiler's budget (5 waves
                                   per SIMD; with mesh_block 512 only the while-while kernel exists there, so
                                   that pair renders only with traversal | 16384), 6 = <= 80 VGPRs (6 waves per SIMD; the path throughput spills
                                   once per bounce, none in the traversal loop; C4 -5 %, C5 geometry -12 %) */
    int32_t mesh_lds_stack;     /* mesh traversal stack entries per lane kept in LDS (0..64; deeper entries go
                                   to scratch memory); -1 = auto (the default): the most entries, up to 12,
                                   that cost no workgroup per CU -- none for the mixed-scene kernels over the
                                   sphere grid (r06: C5 geometry -2.7 %) */
    int32_t mesh_block;         /* threads per workgroup for scenes with a mesh: 256, 512, or 0 = auto (the
                                   one keeping more waves per CU given registers and LDS) */
    int32_t item_samples;       /* F32 work queue: samples per work item at most (1..32; items shrink to 1 */
    double item_balance;        /* sample towards the end: a chunk of c samples is handed out only while
                                   what is left keeps every resident lane busy for item_balance chunks;
                                   default 8 since r05 -- 4 before; C3 -0.6 %, its 8-GPU shard -1 %) */
    double mesh_item_balance;   /* item_balance for scenes with a mesh (their per-pixel cost varies more);
                                   fp32 doubles it on shards with fewer pixels than resident lanes */
    int32_t coh_refill;         /* coherent kernel: another shade round runs while at least this many lanes of
                                   a wave hold no ray (1..64; default 48) */
    int32_t f64_kernel;         /* fp64 render kernel: 0 = default (5 where the scene has a sphere grid and
                                   traversal carries RT_TRAV_GRID, else 4; 5 is kernel 4 walking the grid,
                                   ABI 8); 3 = conservative fp32 slab tests
                                   (each slab widened by a bound of its rounding: no box the exact ray
                                   enters is rejected) on persistent lanes over the work queue (item_*),
                                   each sample stored for the ordered reduction (sample_buffer_mb bounds
                                   the buffer); 4 = 3 with coherent primaries (camera rays traced in
                                   per-tile batches).  Both render the same frame bit for bit (kernels 1 /
                                   2, one wave per tile, were removed in ABI 6 and are refused) */
    int32_t grid_workgroups;    /* fp32 persistent kernels: workgroups per launch; 0 = what the device keeps
                                   resident (the default); more only queue behind them (tests) */
    int32_t front_spheres;      /* the N largest spheres (below the R >= 64 ground class) are tested by every
                                   ray before the BVH, outside it (0..16; 0 = all in the BVH; -1 = auto, the
                                   default: those with radius >= 4x the median, at most 8) */
    double sphere_grid_density; /* cells per sphere of the uniform sphere grid that traversal flag
                                   RT_TRAV_GRID traverses instead of the sphere BVH -- fp32 sphere and
                                   mixed scenes, and fp64 through f64_kernel 5 (built by rt_upload_scene
                                   over the spheres outside the front list, when the scene suits one: see
                                   build_sphere_grid); 0 = no grid (the BVH).  Read at rt_upload_scene: a
                                   later change takes effect at the next upload (rt_scene_info reports the
                                   values the current grid was built with) */
    int32_t sphere_grid_time_slabs; /* the grid's time slabs (1..64; default 32; ABI 9): a ray walks only the
                                   cells within the box of the spheres at its time's slab of [0, 1] (moving
                                   spheres fill less of their swept box at one time); 1 = the spheres'
                                   box over the whole shutter (C3 37.8 -> 36.2 ms, r05ao).  Read at
                                   rt_upload_scene, as sphere_grid_density */
} rt_tuning;
enum { RT_MESH_BUILD_HOST = 0, RT_MESH_BUILD_GPU = 1, RT_MESH_BUILD_GPU_LBVH = 2 };
enum { RT_TRAV_SELROOT = 8, RT_TRAV_B128 = 16, RT_TRAV_COH = 64, RT_TRAV_NOSUM = 128, RT_TRAV_TBIN = 256,
       RT_TRAV_CULL = 512, RT_TRAV_MTOP = 4096, RT_TRAV_MIFIF = 8192, RT_TRAV_MWHILE = 16384, RT_TRAV_MQ = 32768,
       RT_TRAV_GRID = 65536, RT_TRAV_GFLAT = 131072, RT_TRAV_G3D = 262144,
       RT_TRAV_DEFAULT = RT_TRAV_COH | RT_TRAV_SELROOT | RT_TRAV_B128 | RT_TRAV_CULL | RT_TRAV_GRID };

typedef struct rt_ctx rt_ctx;

/* ---- context ------------------------------------------------------------------ */
int rt_abi_version(void);
int rt_device_count(void);
/* precision: RT_PREC_F32 (fast path) or RT_PREC_F64 (reference-exact arithmetic).
 * seed keys the per-(pixel, sample) RNG streams (replaces rtweekend.h:25-29's global
 * mt19937, which no parallel renderer can share). */
rt_ctx* rt_create(int device, uint64_t seed, int precision);
void rt_destroy(rt_ctx* ctx);
const char* rt_last_error(const rt_ctx* ctx);
const char* rt_error_string(int code);
int rt_set_seed(rt_ctx* ctx, uint64_t seed);
void* rt_stream(rt_ctx* ctx);
int rt_get_tuning(rt_ctx* ctx, rt_tuning* t);
int rt_set_tuning(rt_ctx* ctx, const rt_tuning* t);

/* camera::initialize (camera.h:52-85) in fp64, operation for operation. */
int rt_camera_initialize(const rt_camera_desc* desc, rt_camera* cam);

/* ---- scene: replaces hittable_list::add (hittable_list.h:20-23) + bvh_node(list)
 * (bvh.h:10-14).  The host builds an SAH BVH over the spheres, keeps the very large
 * ones (the R=1000 ground, main.cpp:15) in a separate list tested in fp64, and uploads
 * the flattened arrays.  Arrays are copied; the caller keeps ownership. */
int rt_upload_scene(rt_ctx* ctx, const rt_sphere* spheres, int num_spheres, const rt_material* materials,
                    int num_materials);
/* ABI 10: 1 in *walks when a launch with this camera walks the sphere grid, 0 when it renders
 * with the sphere tree (no grid built, or a ray could start beyond the grid's reach,
 * rt_scene_info.grid_far_o: the camera itself, or hit points on the scene -- anywhere on its
 * spheres, triangles and the big spheres that refract or move, and the parts of static opaque
 * big spheres visible from those).  Either way the same frame. */
int rt_grid_reach(rt_ctx* ctx, const rt_camera* cam, int32_t* walks);
int rt_scene_info_get(rt_ctx* ctx, rt_scene_info* info);
/* Spheres plus triangles (configs 4/5: mesh, mixed).  Triangles get their own 4-wide BVH,
 * HBM-resident (nodes and triangles are read through L2/Infinity Cache with global loads;
 * the traversal stack is an LDS column per lane, deeper entries in scratch), built on the
 * host (binned SAH) or on the device (LBVH) per rt_tuning.mesh_builder.  Triangles are
 * two-sided with the sphere path's (0.001, inf) interval: fp64 Moller-Trumbore (the oracle's
 * operation order), fp32 a watertight edge-function test (r05); rt_render_diag
 * instruments the default mesh kernels too (slots 27-30).  Coordinates (centres, motion,
 * radii, vertices) must be finite and within +-1e30 (RT_ERR_LIMIT otherwise). */
int rt_upload_scene_ex(rt_ctx* ctx, const rt_sphere* spheres, int num_spheres, const rt_material* materials,
                       int num_materials, const rt_triangle* triangles, int num_triangles);

/* ---- OBJ: replaces ModelLoader::load (src/vulkan/model_loader.h:17-19, an empty stub)
 * over the vendored, never-called tinyobjloader (tiny_obj_loader.h:605).  Returns RT_OK
 * and malloc'd arrays (release with rt_obj_free); RT_ERR_INVALID on a parse error (an
 * unreadable path, a face index naming no vertex, a coordinate that overflows to +-inf);
 * RT_ERR_LIMIT for a face with more than RT_OBJ_MAX_FACE_VERTICES corners or when memory
 * runs out.  Coordinates follow tinyobjloader's number grammar (a missing or non-numeric
 * token is 0); lines end at \n, \r\n or \r. */
#define RT_OBJ_MAX_FACE_VERTICES 4096
int rt_obj_load(const char* path, rt_obj_mesh* out);
void rt_obj_free(rt_obj_mesh* mesh);

/* ---- render: replaces camera::render's pixel x sample loop + ray_color recursion
 * (camera.h:37-47, camera_cpu.h:8-26).  Renders the tiles of `shard` of
 * `num_shards` into out_sums (device, shard_tiles*64*3 values of the context
 * precision: float for F32, double for F64), each the SUM over spp samples of the
 * linear colour (the `pixel_color` of camera.h:40-44).  out_segments (device,
 * shard_tiles*64 uint32, may be NULL) receives per-pixel world.hit counts.  F64 sums are
 * the reference's: sequential fp64 additions in sample order.  F32 sums are exact sums of
 * the samples' fp32 radiance rounded to the grid 2^-28 (64-bit fixed point), rounded once
 * to float -- independent of how samples are split over waves, launches or GPUs, exact
 * while a pixel's sample radiances stay below 2^13 (non-finite sums give NaN / +-inf as
 * the reference's additions would).  Asynchronous
 * on `stream` (NULL: the context's own stream, created hipStreamNonBlocking, so it does
 * NOT wait for work on the legacy null stream: the caller orders the producers of
 * out_sums/out_segments before the call, or passes its own stream); rt_last_kernel_ms()
 * gives its kernel time once it has finished. */
int rt_shard_layout(int width, int height, int shard, int num_shards, rt_shard_info* info);
int rt_render(rt_ctx* ctx, const rt_camera* cam, int samples_per_pixel, int max_depth, int shard, int num_shards,
              void* out_sums, uint32_t* out_segments, void* stream);
int rt_last_kernel_ms(rt_ctx* ctx, float* ms);
/* Progressive / split rendering: samples [sample_begin, sample_begin + sample_count) of
 * every pixel of the shard.  accumulate = 1 continues the per-pixel sums (and world.hit
 * counts) already in out_sums / out_segments, so a frame rendered as several ranges is
 * bit-identical to one rt_render of all its samples.  F64 continues the values in
 * out_sums.  F32 continues the context's fixed-point sums of the last launches into this
 * same buffer (same shard layout; the context remembers the last 4 buffers) wherever
 * out_sums still holds what the last launch wrote there; for a buffer it holds no sums
 * for, or where the contents changed (e.g. freed and reallocated at the same address),
 * it starts from out_sums' float values.  spp > 8191 runs as consecutive launches
 * (rt_last_kernel_ms covers all of them).  (The role the
 * reference's interactive Vulkan frame loop would play, graphical_environment_vulkan.cpp
 * :208-225, as plain device accumulation.) */
int rt_render_range(rt_ctx* ctx, const rt_camera* cam, int sample_begin, int sample_count, int max_depth,
                    int shard, int num_shards, int accumulate, void* out_sums, uint32_t* out_segments, void* stream);

/* Scatter num_shards stacked shard buffers (shard s at s*max_shard_tiles*64*3) into a
 * row-major W*H*3 frame (device, context precision). */
int rt_unshard(rt_ctx* ctx, const void* gathered, int width, int height, int num_shards, void* frame,
               void* stream);
/* write_color (color.h:14-35) on the device: sums -> /spp -> sqrt -> clamp(0,0.999) ->
 * int(256 x).  rgb: W*H*3 int32 (device) -- int32 because the reference prints
 * static_cast<int> and a NaN sum prints INT_MIN. */
int rt_quantize(rt_ctx* ctx, const void* frame, int width, int height, int samples_per_pixel, int32_t* rgb,
                void* stream);

/* write_color straight to bytes, fused with the un-interleave: num_shards stacked shard
 * buffers (as rt_unshard) -> row-major W*H*3 uint8 (device).  A quarter of rt_quantize's
 * int32 frame, so the device->host copy of a frame is 6.2 MB at 1080p.  A NaN sum
 * (which the reference prints as static_cast<int>(NaN)) gives 0. */
int rt_finish_frame_u8(rt_ctx* ctx, const void* gathered, int width, int height, int num_shards,
                       int samples_per_pixel, uint8_t* rgb8, void* stream);
/* Page-locked host memory (hipHostMalloc): device->host copies into it run at the full
 * link rate and asynchronously.  rt_host_free releases it. */
void* rt_host_alloc(size_t bytes);
void rt_host_free(void* p);

/* Whole frame on this context's GPU, 8-bit host out (the camera::render output path):
 * render, rt_finish_frame_u8 and the copy into rgb8_host (W*H*3 bytes; copied directly
 * when it is rt_host_alloc memory, else through the context's pinned staging buffer).
 * Synchronous. */
int rt_render_frame_u8(rt_ctx* ctx, const rt_camera* cam, int samples_per_pixel, int max_depth, uint8_t* rgb8_host);

/* ---- RCCL: the gather of finished shards to rank 0 over xGMI.
 * One process per GPU: rank 0 makes an id with rt_comm_unique_id, every rank receives it
 * by any channel (a file, a socket, torch.distributed's store) and calls
 * rt_comm_init_rank (non-blocking ncclCommInitRankConfig, polled): a rank whose peers do
 * not all join within the timeout (RT_COMM_INIT_TIMEOUT_MS, or the _timeout variant's)
 * gets RT_ERR_COMM and the half-built communicator is aborted, so a failure on one rank
 * cannot leave the others blocked.  One process driving several GPUs:
 * rt_comm_init_all (ncclCommInitAll) gives context r rank r.  RCCL errors come back as
 * RT_ERR_COMM with ncclGetErrorString in rt_last_error (e.g. two ranks on one GPU). */
#define RT_COMM_ID_BYTES 128
#define RT_COMM_INIT_TIMEOUT_MS 120000
int rt_comm_unique_id(char id[RT_COMM_ID_BYTES]);
int rt_comm_init_rank(rt_ctx* ctx, int nranks, int rank, const char id[RT_COMM_ID_BYTES]);
int rt_comm_init_rank_timeout(rt_ctx* ctx, int nranks, int rank, const char id[RT_COMM_ID_BYTES], int timeout_ms);
int rt_comm_init_all(rt_ctx** ctxs, int num_ctxs);
int rt_comm_rank(rt_ctx* ctx, int* rank, int* nranks);   /* RT_ERR_INVALID without a communicator */
int rt_comm_destroy(rt_ctx* ctx);
/* ncclGather of this rank's shard buffer (max_shard_tiles*64*3 values of the context
 * precision for a W x H frame split over nranks) into `gathered` on rank 0 (nranks times
 * that, shard r at offset r; may be NULL on other ranks), enqueued on `stream` after the
 * work already there (the render).  Asynchronous. */
int rt_gather_shards(rt_ctx* ctx, const void* shard, void* gathered, int width, int height, void* stream);

/* Whole frame across several contexts in ONE process (e.g. one per GPU of the node, each
 * with the same scene uploaded): context r renders shard r of n on its own stream; the
 * shards are copied to ctxs[0]'s device (peer copies over xGMI when the devices differ),
 * un-interleaved and quantised there.  Same pixels as rt_render_frame on one context.
 * With communicators from rt_comm_init_all the shards travel by one grouped ncclGather;
 * otherwise by peer copies (hipMemcpyPeerAsync).  Synchronous; outputs as rt_render_frame.  (The per-process alternative for clusters of
 * ranks is rt_render + an RCCL gather, raytracingproject_amd/distributed.py.) */
int rt_render_frame_multi(rt_ctx** ctxs, int num_ctxs, const rt_camera* cam, int samples_per_pixel, int max_depth,
                          void* sums_host, int32_t* rgb_host);

/* Whole frame on this context's GPU, host in / host out (the drop-in camera::render
 * path).  sums_host: W*H*3 of the context precision (may be NULL); rgb_host: W*H*3 int32
 * (may be NULL); segments_host: W*H uint32 (may be NULL).  Synchronous. */
int rt_render_frame(rt_ctx* ctx, const rt_camera* cam, int samples_per_pixel, int max_depth, void* sums_host,
                    int32_t* rgb_host, uint32_t* segments_host);

/* One ray on an explicit tape of uniforms, fp64, reference order: the drop-in for a
 * direct ray_color(r, depth, world) call (camera_cpu.h:8, tests.cpp:42) that must keep
 * consuming the caller's sequential random stream.  ray = {orig[3], dir[3], time}.
 * *used = uniforms consumed (the caller advances its stream by that much); if *used
 * exceeds tape_len the result is invalid and the caller retries with a longer tape. */
int rt_trace_tape(rt_ctx* ctx, const double ray[7], int depth, const double* tape, int tape_len, double out[3],
                  int* used);

/* Batched world.hit: hittable::hit (hittable.h:28) of the uploaded world -- the closest
 * hit in (0.001, inf), hittable_list.h:25-39 / bvh.h:16-24 -- for n rays in one launch,
 * with each closest hit's hit_record (hittable.h:7-22).  rays: device memory, n records
 * of 7 values of the context precision {origin xyz, direction xyz, time}; hits: device
 * memory, n rt_hit.  id: the input index of the sphere hit (as given to
 * rt_upload_scene[_ex]), num_spheres + the triangle's input index, or -1 (miss: the other
 * fields are 0); mat: its material index.  fp64 contexts compute with the reference's
 * operations (sphere.h:30-57) and order.  Asynchronous on `stream` (NULL: the context's);
 * rt_last_kernel_ms times it. */
typedef struct {
    double t;
    double p[3], normal[3];
    int32_t id, front_face, mat, pad;
} rt_hit;
int rt_trace_rays(rt_ctx* ctx, const void* rays, int num_rays, rt_hit* hits, void* stream);
/* The same, instrumented (fp32 sphere scenes; synchronous): counters = {node-loop wave
 * iterations, their active lanes, sphere-loop wave iterations, their active lanes}. */
int rt_trace_rays_diag(rt_ctx* ctx, const void* rays, int num_rays, rt_hit* hits, uint64_t counters[4]);

/* ---- diagnostics (not on the render path) ---------------------------------------
 * Whole frame with the instrumented build of the persistent fp32 kernel (block 512, the
 * context's traversal flags 0, 1 or 8; spp <= 8191): counters[16] receives
 *  0 bounce-loop wave iterations, 1 active lanes summed over them,
 *  2 inner-node-loop wave iterations, 3 their active lanes, 4 leaf-sphere-loop wave
 *  iterations, 5 their active lanes, 6/7 shader cycles (s_memtime) summed over bounce
 *  iterations in closest-hit / shade+scatter, 8 cycles in the pixel-chunk hand-out and
 *  flush loop, 9 whole-kernel cycles, both summed over waves, 10 world.hit calls,
 *  11 pixel-chunk flushes, 12-14 the K-rays-per-lane model: wave step iterations (node
 *  visits + sphere tests of the slowest active lane) summed per closest_hit call (K=1),
 *  per pair (K=2) and per four consecutive calls (K=4). */
int rt_render_diag(rt_ctx* ctx, const rt_camera* cam, int samples_per_pixel, int max_depth, uint64_t counters[16]);
/* The same with n <= RT_DIAG_SLOTS counters.  The coherent-primary kernel (RT_TRAV_COH)
 * fills 0-15 as {0 bounce-loop wave iterations, 1 their active lanes, 2-5 as above,
 * 6 cycles in closest-hit (secondaries), 7 shade rounds, 8 camera-ray batches, 9 whole
 * kernel, 10 world.hit calls (secondaries), 11 finished paths, 12 batches, 13 batch
 * traversal wave iterations, 14 their active lanes, 15 primary hits popped} and 16-23
 * with each wave's timeline in s_memrealtime ticks (100 MHz): 16 latest wave end,
 * 17 ~earliest wave start (bitwise NOT), 18 sum over waves of (end - queue found dry),
 * 19 sum of (queue found dry - start), 20 ~earliest dry (NOT), 21 latest dry, 22 waves,
 * 23 bounce-loop wave iterations after the queue ran dry (the drain), and 24-27 with the
 * framebuffer traffic: 24 samples finished into their item's LDS sums, 25 samples
 * flushed straight to HBM (their item was no longer the wave's current one, or a value
 * outside [0, 1]), 26 item flushes (per pixel); mesh scenes add 27-30: 27 mesh-BVH node
 * wave iterations, 28 their active lanes, 29 triangle-test wave iterations, 30 their active
 * lanes. */
enum { RT_DIAG_SLOTS = 32 };
int rt_render_diag_ex(rt_ctx* ctx, const rt_camera* cam, int samples_per_pixel, int max_depth, uint64_t* counters,
                      int n);

#ifdef __cplusplus
}
#endif
#endif

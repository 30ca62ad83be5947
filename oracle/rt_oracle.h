/*
 * rt_oracle.h -- TEST INFRASTRUCTURE ONLY.  fp64 C restatement of the reference CPU
 * path tracer (reference src headers and main.cpp).  Used only by tests/, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg, always as the CHECKER,
 * never as the thing measured or shipped.  The product (raytracingproject_amd/) never
 * loads it.
 *
 * Parity pinned against the reference itself (oracle/_ref/ref_golden, built from the
 * unmodified sources by oracle/Makefile) and its committed output:
 *   - mt19937 mode reproduces /root/reference/image.ppm byte-exactly (sha256 0f946141...)
 *   - counter mode (RT-CRNG-1, rt_rng_spec.h) reproduces ref_golden's fp64 pixel sums
 *     bit-exactly (tests/test_oracle.py, tests/golden/).
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_LAMBERTIAN = 0, ORC_METAL = 1, ORC_DIELECTRIC = 2 };

typedef struct {
    double center[3];      /* center1 (sphere.h:61)                               */
    double center_vec[3];  /* center2 - center1 for moving spheres, else 0 (sphere.h:27) */
    double radius;
    int32_t moving;
    int32_t mat;           /* index into the material table                       */
} orc_sphere;

typedef struct {
    int32_t type;          /* ORC_LAMBERTIAN / ORC_METAL / ORC_DIELECTRIC          */
    int32_t pad;
    double albedo[3];
    double fuzz;           /* stored already clamped to <= 1 (material.h:33)       */
    double ir;
} orc_material;

/* camera.h:15-26 public fields, plus the derived members of camera.h:117-125. */
typedef struct {
    double aspect_ratio;
    int32_t image_width, samples_per_pixel, max_depth, image_height;
    double vfov, lookfrom[3], lookat[3], vup[3], defocus_angle, focus_dist;
    /* derived by orc_camera_initialize (camera.h:52-85) */
    double center[3], pixel00_loc[3], pixel_delta_u[3], pixel_delta_v[3];
    double u[3], v[3], w[3], defocus_disk_u[3], defocus_disk_v[3];
} orc_camera;

/* A triangle (mesh path).  The reference has no triangle primitive, so
 * this is the documented spec the GPU path follows (two-sided Moller-Trumbore, the
 * sphere path's (0.001, inf) interval, outward normal unit((v1-v0) x (v2-v0))): parity
 * for meshes is GPU vs this restatement ("parity unpinned" against the reference).
 * Same layout as rt_triangle (include/rt_hip.h). */
typedef struct {
    double v0[3], v1[3], v2[3];
    int32_t mat, pad;
} orc_triangle;

/* Triangles hit after the spheres by every call below (linear scan, test-only global
 * state); n = 0 clears.  The array is referenced, not copied. */
void orc_set_mesh(const orc_triangle* t, int n);

/* Acceleration hooks for measurement probes (tests/cpp/work_model.cpp: the algorithmic
 * work of a BVH traversal, counted on the reference's own path logic).  When set,
 * world.hit asks `sphere` for the closest sphere in (tmin, tmax) and then `tri` for the
 * closest triangle in (tmin, closest) instead of scanning the lists; each returns an index
 * or -1, and the oracle recomputes the hit record from that primitive with its own
 * arithmetic.  Only exact ties between primitives can resolve differently from the linear
 * scan.  NULL clears. */
typedef struct {
    int (*sphere)(void* ctx, const double o[3], const double d[3], double tm, double tmin, double tmax);
    int (*tri)(void* ctx, const double o[3], const double d[3], double tmin, double tmax);
    void* ctx;
} orc_accel;
void orc_set_accel(const orc_accel* a);
/* One primitive's root in (tmin, tmax) with the oracle's arithmetic (sphere.h:30-57; the
 * Moller-Trumbore restatement): 1 and *t, or 0. */
int orc_sphere_root(const orc_sphere* s, const double o[3], const double d[3], double tm, double tmin, double tmax,
                    double* t);
int orc_tri_root(const orc_triangle* tr, const double o[3], const double d[3], double tmin, double tmax, double* t);

/* RNG: mode 0 = the reference's global mt19937 stream (rtweekend.h:25-29),
 *      mode 1 = RT-CRNG-1 keyed per (pixel, sample). */
typedef struct {
    int32_t mode;
    uint32_t mt[624];
    int32_t mti;
    uint32_t key, ctr;
    uint64_t draws;
} orc_rng;

void orc_rng_init_mt(orc_rng* r);                 /* std::mt19937 default seed 5489 */
void orc_rng_init_counter(orc_rng* r);
void orc_rng_set_path(orc_rng* r, uint64_t seed, uint32_t pixel, uint32_t sample);
double orc_random_double(orc_rng* r);

/* Scenes.  Return the sphere count; materials are one per sphere. */
int orc_scene_random(orc_rng* r, orc_sphere* s, orc_material* m, int cap);   /* main.cpp:12-53 */
int orc_scene_four(orc_sphere* s, orc_material* m, int cap);                 /* main.cpp:14-15,46-53 */
int orc_scene_ground(orc_sphere* s, orc_material* m, int cap);               /* tests.cpp:26-29 */

void orc_camera_defaults(orc_camera* c);          /* main.cpp:57-68 */
void orc_camera_initialize(orc_camera* c);        /* camera.h:52-85 */

/* One camera ray (camera.h:87-113) and its radiance (camera_cpu.h:8-26).
 * ray = {orig[3], dir[3], time}.  *segments counts world.hit calls. */
void orc_get_ray(const orc_camera* c, orc_rng* r, int i, int j, double ray[7]);
void orc_ray_color(const orc_sphere* s, const orc_material* m, int n, const double ray[7], int depth,
                   orc_rng* r, double out[3], uint64_t* segments);

/* write_color (color.h:14-35): three ints as the PPM text would carry them. */
void orc_write_color(const double c[3], int spp, int32_t out[3]);

/* Full frame in the reference's sequential order on the mt stream r (camera.h:37-47).
 * sums: W*H*3 doubles (may be NULL); rgb: W*H*3 ints. */
void orc_render_mt(const orc_sphere* s, const orc_material* m, int n, const orc_camera* c, orc_rng* r,
                   double* sums, int32_t* rgb);

/* Counter-RNG render of npix pixels (pix = i0,j0,i1,j1,...).  sums: npix*3 doubles,
 * rgb: npix*3 ints, segs: npix (each may be NULL). */
void orc_render_counter(const orc_sphere* s, const orc_material* m, int n, const orc_camera* c,
                        uint64_t seed, const int32_t* pix, int npix, double* sums, int32_t* rgb,
                        uint64_t* segs);

/* Trace one ray on an explicit tape of uniforms (the GPU tape kernel's checker). */
int orc_trace_tape(const orc_sphere* s, const orc_material* m, int n, const double ray[7], int depth,
                   const double* tape, int tape_len, double out[3]);

/* As orc_render_mt, also adding the world.hit calls to *segments (may be NULL). */
void orc_render_mt_counted(const orc_sphere* s, const orc_material* m, int n, const orc_camera* c, orc_rng* r,
                           double* sums, int32_t* rgb, uint64_t* segments);

/* main.cpp end to end on the mt stream: returns H, fills rgb (W*H*3 ints, W = 400).
 * _counted also reports {scene draws, render draws, world.hit calls}. */
int orc_reference_main(int image_width, int spp, int32_t* rgb);
int orc_reference_main_counted(int image_width, int spp, int32_t* rgb, uint64_t counts[3]);

#ifdef __cplusplus
}
#endif
#endif

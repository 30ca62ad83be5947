/*
 * rt_oracle.c -- TEST INFRASTRUCTURE ONLY (see rt_oracle.h).  fp64 C restatement of the
 * reference path, operation for operation, so that IEEE-754 double results are
 * bit-identical to the g++-built reference (compile with -ffp-contract=off, no
 * -ffast-math).  Every function cites the reference file:line it follows.
 *
 * Evaluation order: g++ evaluates function/constructor arguments right-to-left, so in
 * vec3(random_double(..), random_double(..), random_double(..)) the z component takes
 * the FIRST draw.  The reference's committed image.ppm encodes that order (SURVEY.md
 * §0.3); this file spells every such order out explicitly.
 */
#include "rt_oracle.h"

#include <math.h>
#include <stddef.h>
#include <string.h>

#include "rt_rng_spec.h"

/* ---- vec3 (vec3.h:8-158) ---------------------------------------------------------- */
typedef struct { double x, y, z; } v3;

static inline v3 mk(double x, double y, double z) { v3 r = {x, y, z}; return r; }
static inline v3 ld(const double p[3]) { return mk(p[0], p[1], p[2]); }
static inline void st(double p[3], v3 v) { p[0] = v.x; p[1] = v.y; p[2] = v.z; }
static inline v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }      /* vec3.h:81-83 */
static inline v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }      /* vec3.h:85-87 */
static inline v3 mul(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }      /* vec3.h:89-91 */
static inline v3 scl(double t, v3 v) { return mk(t * v.x, t * v.y, t * v.z); }        /* vec3.h:93-99 */
static inline v3 dvs(v3 v, double t) { return scl(1 / t, v); }                        /* vec3.h:101-103 */
static inline v3 neg(v3 v) { return mk(-v.x, -v.y, -v.z); }                           /* vec3.h:21 */
static inline double dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }   /* vec3.h:105-109 */
static inline v3 cross(v3 u, v3 v) {                                                   /* vec3.h:111-115 */
    return mk(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}
static inline double len2(v3 v) { return v.x * v.x + v.y * v.y + v.z * v.z; }       /* vec3.h:46-48 */
static inline double len(v3 v) { return sqrt(len2(v)); }                               /* vec3.h:42-44 */
static inline v3 unit(v3 v) { return dvs(v, len(v)); }                                 /* vec3.h:117-119 */
static inline v3 reflect(v3 v, v3 n) { return sub(v, scl(2 * dot(v, n), n)); }       /* vec3.h:149-151 */
static inline v3 refract(v3 uv, v3 n, double e) {                                      /* vec3.h:153-157 */
    double cos_theta = fmin(dot(neg(uv), n), 1.0);
    v3 perp = scl(e, add(uv, scl(cos_theta, n)));
    v3 par = scl(-sqrt(fabs(1.0 - len2(perp))), n);
    return add(perp, par);
}

/* ---- RNG (rtweekend.h:25-34) ------------------------------------------------------ */
void orc_rng_init_mt(orc_rng* r) {
    memset(r, 0, sizeof(*r));
    r->mode = 0;
    r->mt[0] = 5489u;
    for (int k = 1; k < 624; ++k) r->mt[k] = 1812433253u * (r->mt[k - 1] ^ (r->mt[k - 1] >> 30)) + (uint32_t)k;
    r->mti = 624;
}

void orc_rng_init_counter(orc_rng* r) {
    memset(r, 0, sizeof(*r));
    r->mode = 1;
}

void orc_rng_set_path(orc_rng* r, uint64_t seed, uint32_t pixel, uint32_t sample) {
    r->key = rtspec_path_key(seed, pixel, sample);
    r->ctr = 0;
}

static uint32_t mt_next(orc_rng* r) {
    if (r->mti >= 624) {
        for (int k = 0; k < 624; ++k) {
            uint32_t y = (r->mt[k] & 0x80000000u) | (r->mt[(k + 1) % 624] & 0x7fffffffu);
            r->mt[k] = r->mt[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        r->mti = 0;
    }
    uint32_t y = r->mt[r->mti++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

/* uniform_real_distribution<double>(0,1) over mt19937: libstdc++ generate_canonical
 * takes two 32-bit draws, sum = g1 + g2*2^32 (rounded once), / 2^64, and maps a
 * result of 1.0 to nextafter(1, 0); then u*(b-a)+a with a=0, b=1. */
double orc_random_double(orc_rng* r) {
    r->draws++;
    if (r->mode == 0) {
        double g1 = (double)mt_next(r);
        double g2 = (double)mt_next(r);
        double sum = g1 + g2 * 4294967296.0;
        double u = sum / 18446744073709551616.0;
        if (u >= 1.0) u = nextafter(1.0, 0.0);
        return u * (1.0 - 0.0) + 0.0;
    }
    return rtspec_u(r->key, r->ctr++);
}

static inline double rnd(orc_rng* r, double lo, double hi) { return lo + (hi - lo) * orc_random_double(r); }

/* vec3::random(min,max) (vec3.h:67-69): arguments evaluated right to left. */
static inline v3 rnd_vec(orc_rng* r, double lo, double hi) {
    double z = rnd(r, lo, hi);
    double y = rnd(r, lo, hi);
    double x = rnd(r, lo, hi);
    return mk(x, y, z);
}
/* vec3::random() (vec3.h:63-65) */
static inline v3 rnd_vec01(orc_rng* r) {
    double z = orc_random_double(r);
    double y = orc_random_double(r);
    double x = orc_random_double(r);
    return mk(x, y, z);
}
static v3 random_in_unit_disk(orc_rng* r) {                                    /* vec3.h:121-127 */
    for (;;) {
        double y = rnd(r, -1, 1);
        double x = rnd(r, -1, 1);
        v3 p = mk(x, y, 0);
        if (len2(p) < 1) return p;
    }
}
static v3 random_in_unit_sphere(orc_rng* r) {                                  /* vec3.h:129-135 */
    for (;;) {
        v3 p = rnd_vec(r, -1, 1);
        if (len2(p) < 1) return p;
    }
}
static inline v3 random_unit_vector(orc_rng* r) { return unit(random_in_unit_sphere(r)); } /* vec3.h:137-139 */

/* ---- scenes ------------------------------------------------------------------------ */
static void put(orc_sphere* s, orc_material* m, int k, v3 c, v3 cv, int moving, double rad, int type, v3 alb,
                double fuzz, double ir) {
    st(s[k].center, c);
    st(s[k].center_vec, cv);
    s[k].radius = rad;
    s[k].moving = moving;
    s[k].mat = k;
    memset(&m[k], 0, sizeof(m[k]));
    m[k].type = type;
    st(m[k].albedo, alb);
    m[k].fuzz = fuzz < 1 ? fuzz : 1; /* material.h:33 */
    m[k].ir = ir;
}

int orc_scene_random(orc_rng* r, orc_sphere* s, orc_material* m, int cap) {
    int n = 0;
    v3 zero = mk(0, 0, 0);
    if (cap < 485) return -1;
    put(s, m, n++, mk(0, -1000, 0), zero, 0, 1000, ORC_LAMBERTIAN, mk(0.5, 0.5, 0.5), 0, 0); /* main.cpp:14-15 */
    for (int a = -11; a < 11; a++) {                                                        /* main.cpp:17-44 */
        for (int b = -11; b < 11; b++) {
            double choose_mat = orc_random_double(r);
            double cz = b + 0.9 * orc_random_double(r);   /* right-to-left: z first */
            double cx = a + 0.9 * orc_random_double(r);
            v3 center = mk(cx, 0.2, cz);
            if (len(sub(center, mk(4, 0.2, 0))) > 0.9) {
                if (choose_mat < 0.8) {
                    /* color::random() * color::random(): right operand first */
                    v3 rhs = rnd_vec01(r);
                    v3 lhs = rnd_vec01(r);
                    v3 albedo = mul(lhs, rhs);
                    v3 center2 = add(center, mk(0, rnd(r, 0, .5), 0));
                    put(s, m, n++, center, sub(center2, center), 1, 0.2, ORC_LAMBERTIAN, albedo, 0, 0);
                } else if (choose_mat < 0.95) {
                    v3 albedo = rnd_vec(r, 0.5, 1);
                    double fuzz = rnd(r, 0, 0.5);
                    put(s, m, n++, center, zero, 0, 0.2, ORC_METAL, albedo, fuzz, 0);
                } else {
                    put(s, m, n++, center, zero, 0, 0.2, ORC_DIELECTRIC, zero, 0, 1.5);
                }
            }
        }
    }
    put(s, m, n++, mk(0, 1, 0), zero, 0, 1.0, ORC_DIELECTRIC, zero, 0, 1.5);              /* main.cpp:46-47 */
    put(s, m, n++, mk(-4, 1, 0), zero, 0, 1.0, ORC_LAMBERTIAN, mk(0.4, 0.2, 0.1), 0, 0);  /* main.cpp:49-50 */
    put(s, m, n++, mk(4, 1, 0), zero, 0, 1.0, ORC_METAL, mk(0.7, 0.6, 0.5), 0.0, 0);      /* main.cpp:52-53 */
    return n;
}

int orc_scene_four(orc_sphere* s, orc_material* m, int cap) {
    v3 zero = mk(0, 0, 0);
    if (cap < 4) return -1;
    put(s, m, 0, mk(0, -1000, 0), zero, 0, 1000, ORC_LAMBERTIAN, mk(0.5, 0.5, 0.5), 0, 0);
    put(s, m, 1, mk(0, 1, 0), zero, 0, 1.0, ORC_DIELECTRIC, zero, 0, 1.5);
    put(s, m, 2, mk(-4, 1, 0), zero, 0, 1.0, ORC_LAMBERTIAN, mk(0.4, 0.2, 0.1), 0, 0);
    put(s, m, 3, mk(4, 1, 0), zero, 0, 1.0, ORC_METAL, mk(0.7, 0.6, 0.5), 0.0, 0);
    return 4;
}

int orc_scene_ground(orc_sphere* s, orc_material* m, int cap) {
    if (cap < 1) return -1;
    put(s, m, 0, mk(0, -1000, 0), mk(0, 0, 0), 0, 1000, ORC_LAMBERTIAN, mk(0.5, 0.5, 0.5), 0, 0);
    return 1;
}

/* ---- camera (camera.h:52-113) ------------------------------------------------------ */
void orc_camera_defaults(orc_camera* c) {
    memset(c, 0, sizeof(*c));
    c->aspect_ratio = 16.0 / 9.0;
    c->image_width = 400;
    c->samples_per_pixel = 30;
    c->max_depth = 50;
    c->vfov = 20;
    st(c->lookfrom, mk(13, 2, 3));
    st(c->lookat, mk(0, 0, 0));
    st(c->vup, mk(0, 1, 0));
    c->defocus_angle = 0.6;
    c->focus_dist = 10.0;
}

static const double PI = 3.1415926535897932385;                 /* rtweekend.h:17 */
static inline double deg2rad(double d) { return d * PI / 180.0; } /* rtweekend.h:21-23 */

void orc_camera_initialize(orc_camera* c) {
    int H = (int)(c->image_width / c->aspect_ratio);
    c->image_height = H < 1 ? 1 : H;
    v3 center = ld(c->lookfrom);
    double theta = deg2rad(c->vfov);
    double h = tan(theta / 2);
    double viewport_height = 2 * h * c->focus_dist;
    double viewport_width = viewport_height * ((double)c->image_width / c->image_height);
    v3 w = unit(sub(ld(c->lookfrom), ld(c->lookat)));
    v3 u = unit(cross(ld(c->vup), w));
    v3 v = cross(w, u);
    v3 viewport_u = scl(viewport_width, u);
    v3 viewport_v = scl(viewport_height, neg(v));
    v3 du = dvs(viewport_u, (double)c->image_width);
    v3 dv = dvs(viewport_v, (double)c->image_height);
    v3 upper_left = sub(sub(sub(center, scl(c->focus_dist, w)), dvs(viewport_u, 2)), dvs(viewport_v, 2));
    v3 p00 = add(upper_left, scl(0.5, add(du, dv)));
    double defocus_radius = c->focus_dist * tan(deg2rad(c->defocus_angle / 2));
    st(c->center, center);
    st(c->pixel00_loc, p00);
    st(c->pixel_delta_u, du);
    st(c->pixel_delta_v, dv);
    st(c->u, u);
    st(c->v, v);
    st(c->w, w);
    st(c->defocus_disk_u, scl(defocus_radius, u));
    st(c->defocus_disk_v, scl(defocus_radius, v));
}

void orc_get_ray(const orc_camera* c, orc_rng* r, int i, int j, double ray[7]) {
    v3 du = ld(c->pixel_delta_u), dv = ld(c->pixel_delta_v);
    v3 pixel_center = add(add(ld(c->pixel00_loc), scl((double)i, du)), scl((double)j, dv));
    double px = -0.5 + orc_random_double(r);                   /* camera.h:102-107 */
    double py = -0.5 + orc_random_double(r);
    v3 pixel_sample = add(pixel_center, add(scl(px, du), scl(py, dv)));
    v3 origin;
    if (c->defocus_angle <= 0) {
        origin = ld(c->center);
    } else {                                                   /* camera.h:109-113 */
        v3 p = random_in_unit_disk(r);
        origin = add(add(ld(c->center), scl(p.x, ld(c->defocus_disk_u))), scl(p.y, ld(c->defocus_disk_v)));
    }
    v3 dir = sub(pixel_sample, origin);
    double time = orc_random_double(r);                         /* camera.h:97 */
    st(ray, origin);
    st(ray + 3, dir);
    ray[6] = time;
}

/* ---- scene hit (hittable_list.h:25-39, sphere.h:30-57, hittable.h:15-21) ---------- */
typedef struct { v3 p, normal; int mat; double t; int front_face; } hrec;

static int sphere_hit(const orc_sphere* s, v3 o, v3 d, double tm, double tmin, double tmax, hrec* rec) {
    v3 center = s->moving ? add(ld(s->center), scl(tm, ld(s->center_vec))) : ld(s->center);
    v3 oc = sub(o, center);
    double a = len2(d);
    double half_b = dot(oc, d);
    double c = len2(oc) - s->radius * s->radius;
    double disc = half_b * half_b - a * c;
    if (disc < 0) return 0;
    double sqrtd = sqrt(disc);
    double root = (-half_b - sqrtd) / a;
    if (!(tmin < root && root < tmax)) {
        root = (-half_b + sqrtd) / a;
        if (!(tmin < root && root < tmax)) return 0;
    }
    rec->t = root;
    rec->p = add(o, scl(root, d));                             /* ray.h:19-21 */
    v3 outward = dvs(sub(rec->p, center), s->radius);
    rec->front_face = dot(d, outward) < 0;
    rec->normal = rec->front_face ? outward : neg(outward);
    rec->mat = s->mat;
    return 1;
}

static const orc_triangle* g_tris = 0;
static int g_ntris = 0;

void orc_set_mesh(const orc_triangle* t, int n) {
    g_tris = n > 0 ? t : 0;
    g_ntris = n > 0 ? n : 0;
}

/* Moller-Trumbore, two-sided; record as hittable.h:15-21 with the outward normal
 * unit(e1 x e2). */
static int tri_hit(const orc_triangle* t, v3 o, v3 d, double tmin, double tmax, hrec* rec) {
    v3 v0 = ld(t->v0);
    v3 e1 = sub(ld(t->v1), v0), e2 = sub(ld(t->v2), v0);
    v3 pv = cross(d, e2);
    double det = dot(e1, pv);
    if (det == 0) return 0;
    double inv_det = 1.0 / det;
    v3 tv = sub(o, v0);
    double u = dot(tv, pv) * inv_det;
    if (u < 0 || u > 1) return 0;
    v3 qv = cross(tv, e1);
    double v = dot(d, qv) * inv_det;
    if (v < 0 || u + v > 1) return 0;
    double tt = dot(e2, qv) * inv_det;
    if (!(tmin < tt && tt < tmax)) return 0;
    rec->t = tt;
    rec->p = add(o, scl(tt, d));
    v3 outward = unit(cross(e1, e2));
    rec->front_face = dot(d, outward) < 0;
    rec->normal = rec->front_face ? outward : neg(outward);
    rec->mat = t->mat;
    return 1;
}

static const orc_accel* g_accel = 0;

void orc_set_accel(const orc_accel* a) { g_accel = a; }

int orc_sphere_root(const orc_sphere* s, const double o[3], const double d[3], double tm, double tmin, double tmax,
                    double* t) {
    hrec r;
    if (!sphere_hit(s, ld(o), ld(d), tm, tmin, tmax, &r)) return 0;
    *t = r.t;
    return 1;
}

int orc_tri_root(const orc_triangle* tr, const double o[3], const double d[3], double tmin, double tmax, double* t) {
    hrec r;
    if (!tri_hit(tr, ld(o), ld(d), tmin, tmax, &r)) return 0;
    *t = r.t;
    return 1;
}

static int world_hit(const orc_sphere* s, int n, v3 o, v3 d, double tm, double tmin, double tmax, hrec* rec) {
    hrec tmp;
    int hit_anything = 0;
    double closest = tmax;
    if (g_accel) {   /* measurement probes: the closest primitive found by a BVH */
        double oo[3], dd[3];
        st(oo, o);
        st(dd, d);
        const int k = g_accel->sphere(g_accel->ctx, oo, dd, tm, tmin, tmax);
        if (k >= 0 && sphere_hit(&s[k], o, d, tm, tmin, closest, &tmp)) {
            hit_anything = 1;
            closest = tmp.t;
            *rec = tmp;
        }
        const int j = g_ntris > 0 ? g_accel->tri(g_accel->ctx, oo, dd, tmin, closest) : -1;
        if (j >= 0 && tri_hit(&g_tris[j], o, d, tmin, closest, &tmp)) {
            hit_anything = 1;
            *rec = tmp;
        }
        return hit_anything;
    }
    for (int k = 0; k < n; ++k) {
        if (sphere_hit(&s[k], o, d, tm, tmin, closest, &tmp)) {
            hit_anything = 1;
            closest = tmp.t;
            *rec = tmp;
        }
    }
    for (int k = 0; k < g_ntris; ++k) {
        if (tri_hit(&g_tris[k], o, d, tmin, closest, &tmp)) {
            hit_anything = 1;
            closest = tmp.t;
            *rec = tmp;
        }
    }
    return hit_anything;
}

/* ---- materials (material.h:15-82) --------------------------------------------------- */
static double reflectance(double cosine, double ref_idx) {     /* material.h:76-80 */
    double r0 = (1 - ref_idx) / (1 + ref_idx);
    r0 = r0 * r0;
    return r0 + (1 - r0) * pow((1 - cosine), 5);
}

typedef double (*draw_fn)(void* ctx);

static int scatter(const orc_material* m, v3 din, double tm, const hrec* rec, draw_fn draw, void* ctx,
                   v3* att, v3* sdir) {
    (void)tm;
    if (m->type == ORC_LAMBERTIAN) {                           /* material.h:19-25 */
        /* random_unit_vector via rejection, z drawn first */
        v3 p;
        for (;;) {
            double z = -1 + (1 - -1) * draw(ctx);
            double y = -1 + (1 - -1) * draw(ctx);
            double x = -1 + (1 - -1) * draw(ctx);
            p = mk(x, y, z);
            if (len2(p) < 1) break;
        }
        *sdir = add(rec->normal, unit(p));
        *att = ld(m->albedo);
        return 1;
    }
    if (m->type == ORC_METAL) {                                /* material.h:35-41 */
        v3 reflected = reflect(unit(din), rec->normal);
        v3 p;
        for (;;) {
            double z = -1 + (1 - -1) * draw(ctx);
            double y = -1 + (1 - -1) * draw(ctx);
            double x = -1 + (1 - -1) * draw(ctx);
            p = mk(x, y, z);
            if (len2(p) < 1) break;
        }
        *sdir = add(reflected, scl(m->fuzz, p));
        *att = ld(m->albedo);
        return dot(*sdir, rec->normal) > 0;
    }
    /* dielectric, material.h:52-71 */
    *att = mk(1.0, 1.0, 1.0);
    double ratio = rec->front_face ? (1.0 / m->ir) : m->ir;
    v3 ud = unit(din);
    double cos_theta = fmin(dot(neg(ud), rec->normal), 1.0);
    double sin_theta = sqrt(1.0 - cos_theta * cos_theta);
    int cannot_refract = ratio * sin_theta > 1.0;
    if (cannot_refract || reflectance(cos_theta, ratio) > draw(ctx))
        *sdir = reflect(ud, rec->normal);
    else
        *sdir = refract(ud, rec->normal, ratio);
    return 1;
}

/* ---- integrator (camera_cpu.h:8-26), recursive as the reference ------------------- */
typedef struct {
    const orc_sphere* s;
    const orc_material* m;
    int n;
    draw_fn draw;
    void* ctx;
    uint64_t segments;
} tracer;

static v3 ray_color(tracer* T, v3 o, v3 d, double tm, int depth) {
    if (depth <= 0) return mk(0, 0, 0);
    hrec rec;
    T->segments++;
    if (world_hit(T->s, T->n, o, d, tm, 0.001, INFINITY, &rec)) {
        v3 att, sdir;
        if (scatter(&T->m[rec.mat], d, tm, &rec, T->draw, T->ctx, &att, &sdir))
            return mul(att, ray_color(T, rec.p, sdir, tm, depth - 1));
        return mk(0, 0, 0);
    }
    v3 ud = unit(d);
    double a = 0.5 * (ud.y + 1.0);
    return add(scl(1.0 - a, mk(1.0, 1.0, 1.0)), scl(a, mk(0.5, 0.7, 1.0)));
}

static double draw_rng(void* ctx) { return orc_random_double((orc_rng*)ctx); }

void orc_ray_color(const orc_sphere* s, const orc_material* m, int n, const double ray[7], int depth, orc_rng* r,
                   double out[3], uint64_t* segments) {
    tracer T = {s, m, n, draw_rng, r, 0};
    v3 c = ray_color(&T, ld(ray), ld(ray + 3), ray[6], depth);
    st(out, c);
    if (segments) *segments += T.segments;
}

typedef struct { const double* tape; int len, pos; } tape_ctx;
static double draw_tape(void* ctx) {
    tape_ctx* t = (tape_ctx*)ctx;
    if (t->pos >= t->len) { t->pos++; return 0.5; }
    return t->tape[t->pos++];
}

int orc_trace_tape(const orc_sphere* s, const orc_material* m, int n, const double ray[7], int depth,
                   const double* tape, int tape_len, double out[3]) {
    tape_ctx tc = {tape, tape_len, 0};
    tracer T = {s, m, n, draw_tape, &tc, 0};
    v3 c = ray_color(&T, ld(ray), ld(ray + 3), ray[6], depth);
    st(out, c);
    return tc.pos;
}

/* ---- output (color.h:9-35) ---------------------------------------------------------- */
static int32_t quant(double x) {
    /* interval(0, 0.999).clamp (interval.h:14-18); a NaN passes through both tests and
     * static_cast<int>(256*NaN) is INT_MIN on x86-64 (cvttsd2si). */
    if (x < 0.000) x = 0.000;
    else if (x > 0.999) x = 0.999;
    double y = 256 * x;
    if (y != y) return (int32_t)0x80000000u;
    return (int32_t)y;
}

void orc_write_color(const double c[3], int spp, int32_t out[3]) {
    double scale = 1.0 / spp;
    double r = c[0] * scale, g = c[1] * scale, b = c[2] * scale;
    r = sqrt(r);
    g = sqrt(g);
    b = sqrt(b);
    out[0] = quant(r);
    out[1] = quant(g);
    out[2] = quant(b);
}

/* ---- frames ------------------------------------------------------------------------- */
void orc_render_mt(const orc_sphere* s, const orc_material* m, int n, const orc_camera* c, orc_rng* r,
                   double* sums, int32_t* rgb) {
    orc_render_mt_counted(s, m, n, c, r, sums, rgb, NULL);
}

void orc_render_mt_counted(const orc_sphere* s, const orc_material* m, int n, const orc_camera* c, orc_rng* r,
                           double* sums, int32_t* rgb, uint64_t* segments) {
    const int W = c->image_width, H = c->image_height, spp = c->samples_per_pixel;
    for (int j = 0; j < H; ++j) {
        for (int i = 0; i < W; ++i) {
            double pc[3] = {0, 0, 0};
            for (int k = 0; k < spp; ++k) {
                double ray[7], col[3];
                orc_get_ray(c, r, i, j, ray);
                orc_ray_color(s, m, n, ray, c->max_depth, r, col, segments);
                pc[0] += col[0];
                pc[1] += col[1];
                pc[2] += col[2];
            }
            size_t o = ((size_t)j * W + i) * 3;
            if (sums) { sums[o] = pc[0]; sums[o + 1] = pc[1]; sums[o + 2] = pc[2]; }
            if (rgb) orc_write_color(pc, spp, rgb + o);
        }
    }
}

void orc_render_counter(const orc_sphere* s, const orc_material* m, int n, const orc_camera* c, uint64_t seed,
                        const int32_t* pix, int npix, double* sums, int32_t* rgb, uint64_t* segs) {
    const int W = c->image_width, spp = c->samples_per_pixel;
    orc_rng r;
    orc_rng_init_counter(&r);
    for (int q = 0; q < npix; ++q) {
        const int i = pix[2 * q], j = pix[2 * q + 1];
        double pc[3] = {0, 0, 0};
        uint64_t sg = 0;
        for (int k = 0; k < spp; ++k) {
            double ray[7], col[3];
            orc_rng_set_path(&r, seed, (uint32_t)(j * W + i), (uint32_t)k);
            orc_get_ray(c, &r, i, j, ray);
            orc_ray_color(s, m, n, ray, c->max_depth, &r, col, &sg);
            pc[0] += col[0];
            pc[1] += col[1];
            pc[2] += col[2];
        }
        if (sums) { sums[3 * q] = pc[0]; sums[3 * q + 1] = pc[1]; sums[3 * q + 2] = pc[2]; }
        if (rgb) orc_write_color(pc, spp, rgb + 3 * q);
        if (segs) segs[q] = sg;
    }
}

int orc_reference_main(int image_width, int spp, int32_t* rgb) {
    return orc_reference_main_counted(image_width, spp, rgb, NULL);
}

int orc_reference_main_counted(int image_width, int spp, int32_t* rgb, uint64_t counts[3]) {
    static orc_sphere s[485];
    static orc_material m[485];
    orc_rng r;
    orc_rng_init_mt(&r);
    int n = orc_scene_random(&r, s, m, 485);
    const uint64_t scene_draws = r.draws;
    orc_camera c;
    orc_camera_defaults(&c);
    c.image_width = image_width;
    c.samples_per_pixel = spp;
    orc_camera_initialize(&c);
    uint64_t segs = 0;
    orc_render_mt_counted(s, m, n, &c, &r, NULL, rgb, &segs);
    if (counts) {
        counts[0] = scene_draws;
        counts[1] = r.draws - scene_draws;
        counts[2] = segs;
    }
    return c.image_height;
}

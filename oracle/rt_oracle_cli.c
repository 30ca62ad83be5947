#define _POSIX_C_SOURCE 199309L
/* rt_oracle_cli.c -- TEST INFRASTRUCTURE.  Command-line face of the C restatement, with
 * the same subcommands and output formats as oracle/_ref/ref_golden, so the two can be
 * diffed (tests/test_oracle.py, tests/golden/make_golden.py). */
#include <stdio.h>
#include <time.h>
#include <stdlib.h>
#include <string.h>

#include "rt_oracle.h"

static const char* arg(int argc, char** argv, const char* key, const char* dflt) {
    for (int k = 2; k + 1 < argc; ++k)
        if (!strcmp(argv[k], key)) return argv[k + 1];
    return dflt;
}

static orc_sphere S[4096];
static orc_material M[4096];

static int scene(const char* name, orc_camera* cam) {
    orc_camera_defaults(cam);
    if (!strcmp(name, "random")) {
        orc_rng r;
        orc_rng_init_mt(&r);
        return orc_scene_random(&r, S, M, 4096);
    }
    if (!strcmp(name, "four")) return orc_scene_four(S, M, 4096);
    if (!strcmp(name, "ground")) return orc_scene_ground(S, M, 4096);
    fprintf(stderr, "unknown scene %s\n", name);
    exit(2);
}

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: rt_oracle_cli main|scene|render ...\n");
        return 2;
    }
    if (!strcmp(argv[1], "main")) {
        int W = atoi(arg(argc, argv, "--width", "400"));
        int spp = atoi(arg(argc, argv, "--spp", "30"));
        int32_t* rgb = malloc(sizeof(int32_t) * 3 * (size_t)W * (size_t)W);
        int H = orc_reference_main(W, spp, rgb);
        printf("P3\n%d %d\n255\n", W, H);
        for (long p = 0; p < (long)W * H; ++p) printf("%d %d %d\n", rgb[3 * p], rgb[3 * p + 1], rgb[3 * p + 2]);
        free(rgb);
        return 0;
    }
    if (!strcmp(argv[1], "scene")) {
        orc_camera cam;
        int n = scene("random", &cam);
        printf("# moving c0x c0y c0z cvx cvy cvz radius mat_type ax ay az fuzz ir\n");
        for (int k = 0; k < n; ++k) {
            const orc_sphere* s = &S[k];
            const orc_material* m = &M[s->mat];
            printf("%d %.17g %.17g %.17g %.17g %.17g %.17g %.17g %d %.17g %.17g %.17g %.17g %.17g\n", s->moving,
                   s->center[0], s->center[1], s->center[2], s->center_vec[0], s->center_vec[1], s->center_vec[2],
                   s->radius, m->type, m->albedo[0], m->albedo[1], m->albedo[2], m->fuzz, m->ir);
        }
        return 0;
    }
    if (!strcmp(argv[1], "render")) {
        orc_camera cam;
        int n = scene(arg(argc, argv, "--scene", "random"), &cam);
        cam.image_width = atoi(arg(argc, argv, "--width", "400"));
        cam.samples_per_pixel = atoi(arg(argc, argv, "--spp", "10"));
        cam.max_depth = atoi(arg(argc, argv, "--depth", "50"));
        unsigned long long seed = strtoull(arg(argc, argv, "--seed", "0"), NULL, 0);
        const char* pix = arg(argc, argv, "--pixels", "all");
        const char* v;
        if ((v = arg(argc, argv, "--aspect", NULL))) cam.aspect_ratio = strtod(v, NULL);
        if ((v = arg(argc, argv, "--vfov", NULL))) cam.vfov = strtod(v, NULL);
        if ((v = arg(argc, argv, "--defocus-angle", NULL))) cam.defocus_angle = strtod(v, NULL);
        if ((v = arg(argc, argv, "--focus-dist", NULL))) cam.focus_dist = strtod(v, NULL);
        orc_camera_initialize(&cam);
        const int W = cam.image_width, H = cam.image_height;
        int cap = W * H, np = 0;
        int32_t* P = malloc(sizeof(int32_t) * 2 * (size_t)cap);
        if (!strcmp(pix, "all")) {
            for (int j = 0; j < H; ++j)
                for (int i = 0; i < W; ++i) { P[2 * np] = i; P[2 * np + 1] = j; ++np; }
        } else if (!strncmp(pix, "stride:", 7)) {
            int k = atoi(pix + 7);
            for (int p = 0; p < W * H; p += k) { P[2 * np] = p % W; P[2 * np + 1] = p / W; ++np; }
        } else if (!strncmp(pix, "list:", 5)) {
            FILE* f = fopen(pix + 5, "r");
            int i, j;
            while (f && np < cap && fscanf(f, "%d %d", &i, &j) == 2) { P[2 * np] = i; P[2 * np + 1] = j; ++np; }
            if (f) fclose(f);
        }
        double* sums = malloc(sizeof(double) * 3 * (size_t)(np ? np : 1));
        int32_t* rgb = malloc(sizeof(int32_t) * 3 * (size_t)(np ? np : 1));
        uint64_t* segs = malloc(sizeof(uint64_t) * (size_t)(np ? np : 1));
        orc_render_counter(S, M, n, &cam, seed, P, np, sums, rgb, segs);
        printf("# i j sum_r sum_g sum_b ir ig ib segments\n");
        for (int q = 0; q < np; ++q)
            printf("%d %d %.17g %.17g %.17g %d %d %d %llu\n", P[2 * q], P[2 * q + 1], sums[3 * q], sums[3 * q + 1],
                   sums[3 * q + 2], rgb[3 * q], rgb[3 * q + 1], rgb[3 * q + 2], (unsigned long long)segs[q]);
        free(P); free(sums); free(rgb); free(segs);
        return 0;
    }
    if (!strcmp(argv[1], "bench")) {
        /* Same interface and output as `ref_golden bench`: the linear 485-sphere list on
         * the mt19937 stream over rows j = rem, rem+mod, ... (scene build excluded). */
        orc_camera cam;
        int n = scene("random", &cam);
        cam.image_width = atoi(arg(argc, argv, "--width", "1920"));
        cam.samples_per_pixel = atoi(arg(argc, argv, "--spp", "1"));
        cam.max_depth = atoi(arg(argc, argv, "--depth", "50"));
        int mod = atoi(arg(argc, argv, "--rows-mod", "1")), rem = atoi(arg(argc, argv, "--rows-rem", "0"));
        orc_camera_initialize(&cam);
        orc_rng r;
        orc_rng_init_mt(&r);
        for (int k = 0; k < 4471; ++k) orc_random_double(&r); /* the scene's draws */
        const int W = cam.image_width, H = cam.image_height, spp = cam.samples_per_pixel;
        unsigned long long rays = 0, segs = 0;
        double checksum = 0;
        struct timespec t0, t1;
        clock_gettime(CLOCK_MONOTONIC, &t0);
        for (int j = rem; j < H; j += mod)
            for (int i = 0; i < W; ++i) {
                double pc[3] = {0, 0, 0};
                for (int k = 0; k < spp; ++k) {
                    double ray[7], col[3];
                    uint64_t sg = 0;
                    orc_get_ray(&cam, &r, i, j, ray);
                    orc_ray_color(S, M, n, ray, cam.max_depth, &r, col, &sg);
                    segs += sg;
                    pc[0] += col[0]; pc[1] += col[1]; pc[2] += col[2];
                }
                checksum += pc[0] + pc[1] + pc[2];
                rays += spp;
            }
        clock_gettime(CLOCK_MONOTONIC, &t1);
        double sec = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
        printf("{\"rays\": %llu, \"segments\": %llu, \"seconds\": %.6f, \"W\": %d, \"H\": %d, \"spp\": %d, "
               "\"rows_mod\": %d, \"rows_rem\": %d, \"checksum\": %.6f}\n",
               rays, segs, sec, W, H, spp, mod, rem, checksum);
        return 0;
    }
    fprintf(stderr, "unknown command\n");
    return 2;
}

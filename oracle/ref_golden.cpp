// ref_golden.cpp -- TEST INFRASTRUCTURE ONLY (never linked into the product).
//
// Driver around the UNMODIFIED reference sources under /root/reference/src.  It is
// compiled by oracle/Makefile (g++, the reference's own compiler family; see
// SURVEY.md §8(c) for why g++ and not clang) into oracle/_ref/ref_golden and used to
//   * pin the C restatement (oracle/rt_oracle.c) against the reference itself,
//   * generate the golden fixtures under tests/golden/ (tests/golden/make_golden.py),
//   * serve as the timed CPU baseline (cpu_baseline.kind = "reference") in bench.py.
//
// Nothing from the reference is copied here: the reference headers and main.cpp are
// #included from their location (-I $(REF)/src).  Two hooks are applied:
//   1. RNG injection.  rtweekend.h:25-29 draws from a function-static std::mt19937.
//      `mt19937` is redirected to std::HookGen while rtweekend.h is parsed, so that
//      random_double() calls HookGen, which either
//        mode 0: returns g1 | g2<<32 from a real std::mt19937 (default seed) -- bit-
//                identical to the unmodified binary (libstdc++ generate_canonical
//                needs 2 x 32-bit draws for a double; one 64-bit draw gives the same
//                correctly-rounded double(g1 + g2*2^32) / 2^64), or
//        mode 1: returns the RT-CRNG-1 counter stream (oracle/rt_rng_spec.h) keyed by
//                the (pixel, sample) being rendered.
//   2. Scene capture.  main.cpp (src/main.cpp:11-71) is included with `main` renamed
//      and `render(world)` (main.cpp:70) rewritten into a capture call, so the random-
//      spheres world is built by the reference's own code on the reference's own
//      stream and handed back here instead of being rendered.
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <limits>
#include <memory>
#include <random>
#include <sstream>
#include <string>
#include <utility>
#include <vector>

extern "C" {
#include "rt_rng_spec.h"
}

namespace std {
struct HookGen {
    using result_type = unsigned long long;
    static constexpr result_type min() { return 0; }
    static constexpr result_type max() { return ~0ull; }
    result_type operator()();
};
}  // namespace std

#define mt19937 HookGen
#include "rtweekend.h"
#undef mt19937

// Private members (sphere.h:60-66, material.h:28,44-45,74, camera.h:117-125) are read
// for the scene dump and camera dump only.  camera_cpu.h has no include guard, so it
// is reached only once, through main.cpp.
#define private public
#define protected public
#include "camera.h"
#include "color.h"
#include "hittable_list.h"
#include "material.h"
#include "sphere.h"

static int g_mode = 0;            // 0 = mt19937 (reference stream), 1 = RT-CRNG-1
static std::mt19937 g_mt;         // default seed 5489, as rtweekend.h:27
static uint32_t g_key = 0, g_ctr = 0;
static unsigned long long g_draws = 0;

std::HookGen::result_type std::HookGen::operator()() {
    ++g_draws;
    if (g_mode == 0) {
        unsigned long long a = g_mt();
        unsigned long long b = g_mt();
        return a | (b << 32);
    }
    uint32_t x24 = rtspec_draw24(g_key, g_ctr++);
    return (unsigned long long)x24 << 40;
}

// ---- scene capture from the reference main.cpp ----------------------------------
template <class Cam>
static void g_capture(Cam& cam, const hittable_list& world);

// `int main() {` becomes `int g_main_unused = 0; static void reference_main() {`: main.cpp
// relies on main's implicit `return 0`, which a renamed int function would not have.
#define main() g_main_unused = 0; static void reference_main()
#define render(w) image_width; g_capture(cam, w)
#include "main.cpp"
#undef render
#undef main
#undef private
#undef protected

static hittable_list g_world;
static CPUImpl::Camera g_cam;
static bool g_captured = false;

template <class Cam>
static void g_capture(Cam& cam, const hittable_list& world) {
    g_cam.aspect_ratio = cam.aspect_ratio;
    g_cam.image_width = cam.image_width;
    g_cam.samples_per_pixel = cam.samples_per_pixel;
    g_cam.max_depth = cam.max_depth;
    g_cam.vfov = cam.vfov;
    g_cam.lookfrom = cam.lookfrom;
    g_cam.lookat = cam.lookat;
    g_cam.vup = cam.vup;
    g_cam.defocus_angle = cam.defocus_angle;
    g_cam.focus_dist = cam.focus_dist;
    g_world = world;
    g_captured = true;
}

// ---- helpers ----------------------------------------------------------------------
struct counting_world : public hittable {
    const hittable& w;
    mutable unsigned long long n = 0;
    explicit counting_world(const hittable& world) : w(world) {}
    bool hit(const ray& r, interval t, hit_record& rec) const override {
        ++n;
        return w.hit(r, t, rec);
    }
    aabb bounding_box() const override { return w.bounding_box(); }
};

// Camera fields of main.cpp:57-68 / tests.cpp:12-23 for the scenes built here.
static void default_camera(CPUImpl::Camera& cam) {
    cam.aspect_ratio = 16.0 / 9.0;
    cam.image_width = 400;
    cam.samples_per_pixel = 30;
    cam.max_depth = 50;
    cam.vfov = 20;
    cam.lookfrom = point3(13, 2, 3);
    cam.lookat = point3(0, 0, 0);
    cam.vup = vec3(0, 1, 0);
    cam.defocus_angle = 0.6;
    cam.focus_dist = 10.0;
}

static void build_scene(const std::string& name, hittable_list& world, CPUImpl::Camera& cam) {
    default_camera(cam);
    if (name == "random") {
        g_mode = 0;
        reference_main();
        if (!g_captured) { fprintf(stderr, "scene capture failed\n"); exit(2); }
        world = g_world;
        cam.aspect_ratio = g_cam.aspect_ratio;
        cam.image_width = g_cam.image_width;
        cam.samples_per_pixel = g_cam.samples_per_pixel;
        cam.max_depth = g_cam.max_depth;
        cam.vfov = g_cam.vfov;
        cam.lookfrom = g_cam.lookfrom;
        cam.lookat = g_cam.lookat;
        cam.vup = g_cam.vup;
        cam.defocus_angle = g_cam.defocus_angle;
        cam.focus_dist = g_cam.focus_dist;
    } else if (name == "four") {
        // ground (main.cpp:14-15) + the three big spheres (main.cpp:46-53)
        world.add(make_shared<sphere>(point3(0, -1000, 0), 1000, make_shared<lambertian>(color(0.5, 0.5, 0.5))));
        world.add(make_shared<sphere>(point3(0, 1, 0), 1.0, make_shared<dielectric>(1.5)));
        world.add(make_shared<sphere>(point3(-4, 1, 0), 1.0, make_shared<lambertian>(color(0.4, 0.2, 0.1))));
        world.add(make_shared<sphere>(point3(4, 1, 0), 1.0, make_shared<metal>(color(0.7, 0.6, 0.5), 0.0)));
    } else if (name == "ground") {
        // tests.cpp:26-29
        world.add(make_shared<sphere>(point3(0, -1000, 0), 1000, make_shared<lambertian>(color(0.5, 0.5, 0.5))));
    } else {
        fprintf(stderr, "unknown scene %s\n", name.c_str());
        exit(2);
    }
}

static void write8(color c, int spp, int out[3]) {
    std::ostringstream os;
    write_color(os, c, spp);
    std::istringstream is(os.str());
    is >> out[0] >> out[1] >> out[2];
}

static const char* arg(int argc, char** argv, const char* key, const char* dflt) {
    for (int k = 2; k + 1 < argc; ++k)
        if (!strcmp(argv[k], key)) return argv[k + 1];
    return dflt;
}

// ---- subcommands ------------------------------------------------------------------
static int cmd_scene() {
    hittable_list world;
    CPUImpl::Camera cam;
    build_scene("random", world, cam);
    printf("# draws_after_scene %llu\n", g_draws);
    // center_vec is dumped as the reference stores it (sphere.h:27), so that
    // center1 + time*center_vec (sphere.h:68-72) is reproduced bit-for-bit.
    printf("# moving c0x c0y c0z cvx cvy cvz radius mat_type ax ay az fuzz ir\n");
    for (auto& obj : world.objects) {
        auto* s = dynamic_cast<sphere*>(obj.get());
        point3 c0 = s->center1;
        vec3 cv = s->is_moving ? s->center_vec : vec3(0, 0, 0);
        int type = -1;
        color alb(0, 0, 0);
        double fuzz = 0, ir = 0;
        if (auto* l = dynamic_cast<lambertian*>(s->mat.get())) { type = 0; alb = l->albedo; }
        else if (auto* m = dynamic_cast<metal*>(s->mat.get())) { type = 1; alb = m->albedo; fuzz = m->fuzz; }
        else if (auto* d = dynamic_cast<dielectric*>(s->mat.get())) { type = 2; ir = d->ir; }
        printf("%d %.17g %.17g %.17g %.17g %.17g %.17g %.17g %d %.17g %.17g %.17g %.17g %.17g\n",
               (int)s->is_moving, c0.x(), c0.y(), c0.z(), cv.x(), cv.y(), cv.z(), s->radius, type,
               alb.x(), alb.y(), alb.z(), fuzz, ir);
    }
    return 0;
}

static int cmd_draws(int n) {
    g_mode = 0;
    for (int k = 0; k < n; ++k) printf("%.17g\n", random_double());
    return 0;
}

static int cmd_pixelmatch() {
    // tests/tests.cpp:35-45 on a fresh stream
    g_mode = 0;
    hittable_list world;
    CPUImpl::Camera cam;
    build_scene("ground", world, cam);
    cam.initialize();
    auto sz = cam.image_size();
    ray r = cam.get_ray(sz.first / 2, sz.second / 2);
    unsigned long long d0 = g_draws;
    color c = cam.ray_color(r, cam.max_depth, world);
    printf("%.17g %.17g %.17g %llu %llu\n", c.x(), c.y(), c.z(), d0, g_draws - d0);
    return 0;
}

static int cmd_camera(const std::string& scene, int width) {
    hittable_list world;
    CPUImpl::Camera cam;
    build_scene(scene, world, cam);
    cam.image_width = width;
    cam.initialize();
    auto p = [](const char* n, vec3 v) { printf("%s %.17g %.17g %.17g\n", n, v.x(), v.y(), v.z()); };
    printf("image_height %d\n", cam.image_height);
    p("center", cam.center);
    p("pixel00_loc", cam.pixel00_loc);
    p("pixel_delta_u", cam.pixel_delta_u);
    p("pixel_delta_v", cam.pixel_delta_v);
    p("defocus_disk_u", cam.defocus_disk_u);
    p("defocus_disk_v", cam.defocus_disk_v);
    return 0;
}

// Render a pixel subset.  counter mode: each (pixel, sample) path draws from its own
// RT-CRNG-1 stream; mt mode: one sequential stream in camera.h:37-47 order (only
// meaningful with --pixels all).
static int cmd_render(int argc, char** argv) {
    std::string scene = arg(argc, argv, "--scene", "random");
    int width = atoi(arg(argc, argv, "--width", "400"));
    int spp = atoi(arg(argc, argv, "--spp", "10"));
    int depth = atoi(arg(argc, argv, "--depth", "50"));
    unsigned long long seed = strtoull(arg(argc, argv, "--seed", "0"), nullptr, 0);
    std::string rng = arg(argc, argv, "--rng", "counter");
    std::string pix = arg(argc, argv, "--pixels", "all");

    hittable_list world;
    CPUImpl::Camera cam;
    build_scene(scene, world, cam);
    cam.image_width = width;
    cam.samples_per_pixel = spp;
    cam.max_depth = depth;
    // optional camera overrides (camera.h:15-26 fields)
    if (const char* v = arg(argc, argv, "--aspect", nullptr)) cam.aspect_ratio = strtod(v, nullptr);
    if (const char* v = arg(argc, argv, "--vfov", nullptr)) cam.vfov = strtod(v, nullptr);
    if (const char* v = arg(argc, argv, "--defocus-angle", nullptr)) cam.defocus_angle = strtod(v, nullptr);
    if (const char* v = arg(argc, argv, "--focus-dist", nullptr)) cam.focus_dist = strtod(v, nullptr);
    cam.initialize();
    const int W = cam.image_width, H = cam.image_height;

    std::vector<std::pair<int, int>> pixels;
    if (pix == "all") {
        for (int j = 0; j < H; ++j)
            for (int i = 0; i < W; ++i) pixels.push_back({i, j});
    } else if (pix.rfind("stride:", 0) == 0) {
        int k = atoi(pix.c_str() + 7);
        for (int p = 0; p < W * H; p += k) pixels.push_back({p % W, p / W});
    } else if (pix.rfind("list:", 0) == 0) {
        FILE* f = fopen(pix.c_str() + 5, "r");
        if (!f) { perror("pixel list"); return 2; }
        int i, j;
        while (fscanf(f, "%d %d", &i, &j) == 2) pixels.push_back({i, j});
        fclose(f);
    } else {
        fprintf(stderr, "bad --pixels\n");
        return 2;
    }

    g_mode = (rng == "mt") ? 0 : 1;
    counting_world cw(world);
    printf("# W %d H %d spp %d depth %d seed %llu rng %s scene %s\n", W, H, spp, depth, seed, rng.c_str(),
           scene.c_str());
    printf("# i j sum_r sum_g sum_b ir ig ib segments draws\n");
    for (auto& px : pixels) {
        const int i = px.first, j = px.second;
        color pixel_color(0, 0, 0);
        unsigned long long s0 = cw.n, d0 = g_draws;
        for (int s = 0; s < spp; ++s) {
            if (g_mode == 1) {
                g_key = rtspec_path_key(seed, (uint32_t)(j * W + i), (uint32_t)s);
                g_ctr = 0;
            }
            ray r = cam.get_ray(i, j);
            pixel_color += cam.ray_color(r, cam.max_depth, cw);
        }
        int q[3];
        write8(pixel_color, spp, q);
        printf("%d %d %.17g %.17g %.17g %d %d %d %llu %llu\n", i, j, pixel_color.x(), pixel_color.y(),
               pixel_color.z(), q[0], q[1], q[2], cw.n - s0, g_draws - d0);
    }
    return 0;
}

// Timed CPU baseline: the reference path (linear hittable_list, recursion, mt19937 stream)
// over rows j = rem, rem+mod, ... of the random-spheres scene.  Scene build excluded.
static int cmd_bench(int argc, char** argv) {
    int width = atoi(arg(argc, argv, "--width", "1920"));
    int spp = atoi(arg(argc, argv, "--spp", "1"));
    int mod = atoi(arg(argc, argv, "--rows-mod", "1"));
    int rem = atoi(arg(argc, argv, "--rows-rem", "0"));
    int depth = atoi(arg(argc, argv, "--depth", "50"));
    hittable_list world;
    CPUImpl::Camera cam;
    build_scene("random", world, cam);
    cam.image_width = width;
    cam.samples_per_pixel = spp;
    cam.max_depth = depth;
    cam.initialize();
    const int W = cam.image_width, H = cam.image_height;
    counting_world cw(world);
    double checksum = 0;
    unsigned long long rays = 0;
    auto t0 = std::chrono::steady_clock::now();
    for (int j = rem; j < H; j += mod) {
        for (int i = 0; i < W; ++i) {
            color pc(0, 0, 0);
            for (int s = 0; s < spp; ++s) {
                ray r = cam.get_ray(i, j);
                pc += cam.ray_color(r, cam.max_depth, cw);
            }
            checksum += pc.x() + pc.y() + pc.z();
            rays += spp;
        }
    }
    auto t1 = std::chrono::steady_clock::now();
    double sec = std::chrono::duration<double>(t1 - t0).count();
    printf("{\"rays\": %llu, \"segments\": %llu, \"seconds\": %.6f, \"W\": %d, \"H\": %d, \"spp\": %d, "
           "\"rows_mod\": %d, \"rows_rem\": %d, \"checksum\": %.6f}\n",
           rays, cw.n, sec, W, H, spp, mod, rem, checksum);
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: ref_golden main|scene|draws N|pixelmatch|camera|render|bench ...\n");
        return 2;
    }
    std::string cmd = argv[1];
    if (cmd == "main") {
        // src/main.cpp end to end: scene on the mt stream, then camera::render (camera.h:32-50)
        g_mode = 0;
        reference_main();
        const unsigned long long scene_draws = g_draws;
        counting_world cw(g_world);
        g_cam.render(cw);   // camera::render is non-virtual and takes any hittable (camera.h:32)
        // stream statistics on stderr (stdout stays the reference's PPM byte for byte)
        fprintf(stderr, "# scene_draws %llu render_draws %llu segments %llu\n", scene_draws,
                g_draws - scene_draws, (unsigned long long)cw.n);
        return 0;
    }
    if (cmd == "scene") return cmd_scene();
    if (cmd == "draws") return cmd_draws(argc > 2 ? atoi(argv[2]) : 6);
    if (cmd == "pixelmatch") return cmd_pixelmatch();
    if (cmd == "camera") return cmd_camera(arg(argc, argv, "--scene", "random"), atoi(arg(argc, argv, "--width", "400")));
    if (cmd == "render") return cmd_render(argc, argv);
    if (cmd == "bench") return cmd_bench(argc, argv);
    fprintf(stderr, "unknown command %s\n", cmd.c_str());
    return 2;
}

// host_queries.cpp -- the reference's scene interface used directly, as code written
// against src/hittable.h / src/material.h would use it:
//   * a user subclass of hittable overriding hit() (a sphere that counts its tests) and
//     one with no device form (a disk: hit() and bounding_box() only);
//   * world.hit(ray, interval, rec) and rec.mat->scatter(...) called by hand, in the
//     reference's own recursion (camera_cpu.h:8-26), on the host in fp64 -- against
//     HIPImpl::Camera::ray_color, the same ray traced by the device's fp64 kernel on the
//     same global random stream: colours and stream positions must agree bit for bit;
//   * rendering a world that holds the disk is refused (std::invalid_argument).
// Exit status 0 = pass.
#include <cstdio>
#include <stdexcept>

#include "bvh.h"
#include "camera_hip.h"
#include "hittable_list.h"
#include "material.h"
#include "sphere.h"

class counted_sphere : public sphere {
  public:
    using sphere::sphere;
    mutable long tests = 0;
    bool hit(const ray& r, interval ray_t, hit_record& rec) const override {
        ++tests;
        return sphere::hit(r, ray_t, rec);
    }
};

// A flat disk: a reference-style hittable with no flatten() (no device form).
class disk : public hittable {
  public:
    disk(point3 c, double rad, shared_ptr<material> m) : c_(c), r_(rad), m_(m) {}
    bool hit(const ray& r, interval ray_t, hit_record& rec) const override {
        const double dy = r.direction().y();
        if (dy == 0) return false;
        const double t = (c_.y() - r.origin().y()) / dy;
        if (!ray_t.surrounds(t)) return false;
        const point3 p = r.at(t);
        if ((p - c_).length_squared() > r_ * r_) return false;
        rec.t = t;
        rec.p = p;
        rec.set_face_normal(r, vec3(0, 1, 0));
        rec.mat = m_;
        return true;
    }
    aabb bounding_box() const override { return aabb(c_ - vec3(r_, 0, r_), c_ + vec3(r_, 0, r_)); }

  private:
    point3 c_;
    double r_;
    shared_ptr<material> m_;
};

// camera_cpu.h:8-26 through the virtual interface
static color host_ray_color(const ray& r, int depth, const hittable& world) {
    if (depth <= 0) return color(0, 0, 0);
    hit_record rec;
    if (world.hit(r, interval(0.001, infinity), rec)) {
        ray scattered;
        color attenuation;
        if (rec.mat->scatter(r, rec, attenuation, scattered))
            return attenuation * host_ray_color(scattered, depth - 1, world);
        return color(0, 0, 0);
    }
    const vec3 u = unit_vector(r.direction());
    const double a = 0.5 * (u.y() + 1.0);
    return (1.0 - a) * color(1.0, 1.0, 1.0) + a * color(0.5, 0.7, 1.0);
}

int main() {
    hittable_list spheres;
    spheres.add(make_shared<sphere>(point3(0, -1000, 0), 1000, make_shared<lambertian>(color(0.5, 0.5, 0.5))));
    auto counted = make_shared<counted_sphere>(point3(0, 1, 0), 1.0, make_shared<dielectric>(1.5));
    spheres.add(counted);
    spheres.add(make_shared<sphere>(point3(-4, 1, 0), 1.0, make_shared<lambertian>(color(0.4, 0.2, 0.1))));
    spheres.add(make_shared<sphere>(point3(4, 1, 0), 1.0, make_shared<metal>(color(0.7, 0.6, 0.5), 0.0)));
    for (int a = -5; a < 5; ++a)
        for (int b = -5; b < 5; ++b) {
            const double pick = random_double();
            const point3 c(a + 0.9 * random_double(), 0.2, b + 0.9 * random_double());
            if (pick < 0.6) {
                const point3 c2 = c + vec3(0, random_double(0, 0.5), 0);
                spheres.add(make_shared<sphere>(c, c2, 0.2, make_shared<lambertian>(color::random() * color::random())));
            } else if (pick < 0.85) {
                spheres.add(make_shared<sphere>(c, 0.2, make_shared<metal>(color::random(0.5, 1), random_double(0, 0.5))));
            } else {
                spheres.add(make_shared<sphere>(c, 0.2, make_shared<dielectric>(1.5)));
            }
        }
    hittable_list world;
    world.add(make_shared<bvh_node>(spheres));   // bvh_node::hit on the host: same closest hits

    HIPImpl::Camera cam;
    cam.precision = RT_PREC_F64;
    cam.aspect_ratio = 16.0 / 9.0;
    cam.image_width = 64;
    cam.vfov = 20;
    cam.lookfrom = point3(13, 2, 3);
    cam.lookat = point3(0, 0, 0);
    cam.vup = vec3(0, 1, 0);
    cam.defocus_angle = 0.6;
    cam.focus_dist = 10.0;
    cam.initialize();

    int bad = 0, rays = 0;
    long hits = 0;
    for (int j = 0; j < 36; j += 3)
        for (int i = 0; i < 64; i += 3) {
            const ray r = cam.get_ray(i, j);
            const std::mt19937 before = rt_host::generator();
            hit_record rec;
            hits += world.hit(r, interval(0.001, infinity), rec) ? 1 : 0;
            const color h = host_ray_color(r, 50, world);
            const std::mt19937 after_host = rt_host::generator();
            rt_host::generator() = before;
            const color d = cam.ray_color(r, 50, world);
            const bool same = h.x() == d.x() && h.y() == d.y() && h.z() == d.z() && rt_host::generator() == after_host;
            if (!same && bad++ < 5)
                std::printf("ray (%d,%d): host %.17g %.17g %.17g device %.17g %.17g %.17g\n", i, j, h.x(), h.y(), h.z(),
                            d.x(), d.y(), d.z());
            ++rays;
        }

    hittable_list with_disk = world;
    with_disk.add(make_shared<disk>(point3(0, 2.5, 0), 1.0, make_shared<lambertian>(color(0.9, 0.1, 0.1))));
    hit_record rec;
    const bool disk_hit = with_disk.hit(ray(point3(0, 5, 0), vec3(0, -1, 0)), interval(0.001, infinity), rec) &&
                          rec.t == 2.5 && rec.front_face;
    bool refused = false;
    try {
        cam.render(with_disk);
    } catch (const std::invalid_argument&) {
        refused = true;
    }
    const bool ok = bad == 0 && counted->tests > 0 && hits > 0 && disk_hit && refused;
    std::printf("rays %d mismatched %d world.hit %ld counted_sphere tests %ld disk_hit %d render_refused %d %s\n", rays,
                bad, hits, counted->tests, disk_hit, refused, ok ? "PASS" : "FAIL");
    return ok ? 0 : 1;
}

// sphere.h -- drop-in for src/sphere.h: stationary sphere(center, radius, mat) and
// moving sphere(center1, center2, radius, mat) whose centre is center1 + t*(center2 -
// center1) at ray time t (sphere.h:68-72).  Rendering tests spheres on the device; hit()
// is the host fp64 test for one-ray queries (sphere.h:30-57 arithmetic, half-b quadratic).
#pragma once
#include "hittable.h"

class sphere : public hittable {
  public:
    sphere(point3 center, double radius, shared_ptr<material> mat)
        : center1(center), radius(radius), mat(mat), is_moving(false) {
        const vec3 rv(radius, radius, radius);
        bbox = aabb(center1 - rv, center1 + rv);
    }
    sphere(point3 c1, point3 c2, double radius, shared_ptr<material> mat)
        : center1(c1), radius(radius), mat(mat), is_moving(true), center_vec(c2 - c1) {
        const vec3 rv(radius, radius, radius);
        bbox = aabb(aabb(c1 - rv, c1 + rv), aabb(c2 - rv, c2 + rv));
    }

    bool hit(const ray& r, interval ray_t, hit_record& rec) const override {
        const point3 c = is_moving ? center1 + r.time() * center_vec : center1;
        const vec3 oc = r.origin() - c;
        const double a = r.direction().length_squared();
        const double hb = dot(oc, r.direction());
        const double cc = oc.length_squared() - radius * radius;
        const double disc = hb * hb - a * cc;
        if (disc < 0) return false;
        const double sq = std::sqrt(disc);
        double t = (-hb - sq) / a;   // nearer root first, then the farther one
        if (!ray_t.surrounds(t)) {
            t = (-hb + sq) / a;
            if (!ray_t.surrounds(t)) return false;
        }
        rec.t = t;
        rec.p = r.at(t);
        rec.set_face_normal(r, (rec.p - c) / radius);
        rec.mat = mat;
        return true;
    }
    aabb bounding_box() const override { return bbox; }
    void flatten(scene_builder& out) const override {
        out.add_sphere(center1, is_moving ? center_vec : vec3(0, 0, 0), is_moving, radius, mat);
    }

  private:
    point3 center1;
    double radius;
    shared_ptr<material> mat;
    bool is_moving;
    vec3 center_vec;
    aabb bbox;
};

// hittable.h -- drop-in for src/hittable.h.
//
// The reference's interface is kept: hit(ray, interval, hit_record&) (src/hittable.h:28)
// and bounding_box() (:29), with host fp64 implementations for one-ray queries (they
// round exactly as the reference does).  Rendering never calls them: camera::render()
// runs the closest-hit query inside the MI355X kernel, so every hittable also knows how
// to flatten itself into the arrays the device consumes (rt_hip.h rt_sphere / rt_material
// / rt_triangle).  A subclass that only overrides hit() and bounding_box() (as a
// reference user would write it) works for host queries; its flatten() is the default,
// which rejects it at camera::render() with std::invalid_argument (no device form).
#pragma once
#include <map>
#include <memory>
#include <stdexcept>
#include <vector>

#include "../rt_hip.h"
#include "aabb.h"
#include "rtweekend.h"

class material;

class hit_record {
  public:
    point3 p;
    vec3 normal;
    shared_ptr<material> mat;
    double t = 0;
    bool front_face = false;

    // hittable.h:15-21: outward_normal is unit length; store it facing the ray.
    void set_face_normal(const ray& r, const vec3& outward_normal) {
        front_face = dot(r.direction(), outward_normal) < 0;
        normal = front_face ? outward_normal : -outward_normal;
    }
};

// Collects flattened spheres, triangles and de-duplicated materials (shared_ptr
// identity, as the reference shares material objects between spheres).
class scene_builder {
  public:
    std::vector<rt_sphere> spheres;
    std::vector<rt_triangle> triangles;
    std::vector<rt_material> materials;

    int32_t material_index(const material* m);
    void add_sphere(const point3& center1, const vec3& center_vec, bool moving, double radius,
                    const shared_ptr<material>& mat);
    void add_triangle(const point3& v0, const point3& v1, const point3& v2, int32_t mat);

  private:
    std::map<const material*, int32_t> index_;
};

class hittable {
  public:
    virtual ~hittable() = default;
    // closest hit with t strictly inside ray_t (interval::surrounds); fills rec
    virtual bool hit(const ray& r, interval ray_t, hit_record& rec) const = 0;
    virtual aabb bounding_box() const = 0;
    virtual void flatten(scene_builder&) const {
        throw std::invalid_argument("hittable without a device form (sphere, triangle_mesh, hittable_list, bvh_node)");
    }
};

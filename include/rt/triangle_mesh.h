// triangle_mesh.h -- an indexed triangle mesh with one material, and OBJ loading.
// The reference's src/ has no triangle primitive: its model hook is an empty stub
// (src/vulkan/model_loader.h:17-19) over a vendored, never-called tinyobjloader
// (dependencies/tinyobjloader, LoadObj at tiny_obj_loader.h:605).  This is that hook for
// the MI355X path: load_obj() reads positions and faces through rt_obj_load (same
// triangulation as tinyobjloader's LoadObj), and the mesh flattens into rt_triangle
// records that get their own BVH on the device (rt_upload_scene_ex).  Triangles are
// two-sided; the outward normal is unit((v1 - v0) x (v2 - v0)).
#pragma once
#include <array>
#include <stdexcept>
#include <string>
#include <vector>

#include "hittable.h"
#include "material.h"

class triangle_mesh : public hittable {
  public:
    triangle_mesh(std::vector<point3> vertices, std::vector<std::array<int, 3>> faces, shared_ptr<material> mat)
        : vertices_(std::move(vertices)), faces_(std::move(faces)), mat_(std::move(mat)) {
        if (!mat_) throw std::invalid_argument("triangle_mesh without a material");
        for (const auto& f : faces_)
            for (int k : f)
                if (k < 0 || k >= (int)vertices_.size()) throw std::invalid_argument("face index out of range");
        if (!vertices_.empty()) {
            point3 lo = vertices_[0], hi = vertices_[0];
            for (const auto& v : vertices_)
                for (int a = 0; a < 3; ++a) {
                    lo[a] = std::fmin(lo[a], v[a]);
                    hi[a] = std::fmax(hi[a], v[a]);
                }
            bbox_ = aabb(lo, hi);
        }
    }

    // Wavefront OBJ (positions + faces; polygons triangulated as tinyobjloader does).
    static shared_ptr<triangle_mesh> load_obj(const std::string& path, shared_ptr<material> mat) {
        rt_obj_mesh m{};
        const int rc = rt_obj_load(path.c_str(), &m);
        if (rc != RT_OK) throw std::runtime_error("rt_obj_load(" + path + "): " + rt_error_string(rc));
        std::vector<point3> v((size_t)m.num_vertices);
        for (size_t k = 0; k < v.size(); ++k) v[k] = point3(m.vertices[3 * k], m.vertices[3 * k + 1], m.vertices[3 * k + 2]);
        std::vector<std::array<int, 3>> f((size_t)m.num_triangles);
        for (size_t k = 0; k < f.size(); ++k) f[k] = {m.indices[3 * k], m.indices[3 * k + 1], m.indices[3 * k + 2]};
        rt_obj_free(&m);
        return make_shared<triangle_mesh>(std::move(v), std::move(f), std::move(mat));
    }

    size_t num_triangles() const { return faces_.size(); }

    // Host fp64 closest hit over the triangles (one-ray queries; rendering traverses the
    // device BVH): two-sided Moller-Trumbore in the operation order of the device test
    // (csrc/rt_device.h tri_root), outward normal unit((v1 - v0) x (v2 - v0)).
    bool hit(const ray& r, interval ray_t, hit_record& rec) const override {
        bool any = false;
        const vec3 d = r.direction();
        for (const auto& f : faces_) {
            const point3& v0 = vertices_[f[0]];
            const vec3 e1 = vertices_[f[1]] - v0, e2 = vertices_[f[2]] - v0;
            const vec3 pv = cross(d, e2);
            const double det = dot(e1, pv);
            if (det == 0) continue;
            const double inv = 1 / det;
            const vec3 tv = r.origin() - v0;
            const double u = dot(tv, pv) * inv;
            if (u < 0 || u > 1) continue;
            const vec3 qv = cross(tv, e1);
            const double v = dot(d, qv) * inv;
            if (v < 0 || u + v > 1) continue;
            const double t = dot(e2, qv) * inv;
            if (!interval(ray_t.min, any ? rec.t : ray_t.max).surrounds(t)) continue;
            any = true;
            rec.t = t;
            rec.p = r.at(t);
            rec.set_face_normal(r, unit_vector(cross(e1, e2)));
            rec.mat = mat_;
        }
        return any;
    }
    aabb bounding_box() const override { return bbox_; }
    void flatten(scene_builder& out) const override {
        const int32_t m = out.material_index(mat_.get());
        for (const auto& f : faces_) out.add_triangle(vertices_[f[0]], vertices_[f[1]], vertices_[f[2]], m);
    }

  private:
    std::vector<point3> vertices_;
    std::vector<std::array<int, 3>> faces_;
    shared_ptr<material> mat_;
    aabb bbox_;
};

// material.h -- drop-in for src/material.h: lambertian(albedo), metal(albedo, fuzz)
// (fuzz clamped to 1 as material.h:33), dielectric(index_of_refraction).  scatter()
// (material.h:11-12) is evaluated by the device kernel; the host describes the material.
#pragma once
#include "color.h"
#include "hittable.h"

class material {
  public:
    virtual ~material() = default;
    virtual rt_material describe() const = 0;
};

class lambertian : public material {
  public:
    lambertian(const color& a) : albedo(a) {}
    rt_material describe() const override {
        rt_material m{};
        m.type = RT_LAMBERTIAN;
        for (int k = 0; k < 3; ++k) m.albedo[k] = albedo[k];
        return m;
    }

  private:
    color albedo;
};

class metal : public material {
  public:
    metal(const color& a, double f) : albedo(a), fuzz(f < 1 ? f : 1) {}
    rt_material describe() const override {
        rt_material m{};
        m.type = RT_METAL;
        for (int k = 0; k < 3; ++k) m.albedo[k] = albedo[k];
        m.fuzz = fuzz;
        return m;
    }

  private:
    color albedo;
    double fuzz;
};

class dielectric : public material {
  public:
    dielectric(double index_of_refraction) : ir(index_of_refraction) {}
    rt_material describe() const override {
        rt_material m{};
        m.type = RT_DIELECTRIC;
        m.ir = ir;
        return m;
    }

  private:
    double ir;
};

inline int32_t scene_builder::material_index(const material* m) {
    auto it = index_.find(m);
    if (it != index_.end()) return it->second;
    const int32_t k = (int32_t)materials.size();
    materials.push_back(m->describe());
    index_.emplace(m, k);
    return k;
}

inline void scene_builder::add_triangle(const point3& v0, const point3& v1, const point3& v2, int32_t mat) {
    rt_triangle t{};
    for (int k = 0; k < 3; ++k) {
        t.v0[k] = v0[k];
        t.v1[k] = v1[k];
        t.v2[k] = v2[k];
    }
    t.mat = mat;
    triangles.push_back(t);
}

inline void scene_builder::add_sphere(const point3& c1, const vec3& cv, bool moving, double radius,
                                      const shared_ptr<material>& mat) {
    if (!mat) throw std::invalid_argument("sphere without a material");
    rt_sphere s{};
    for (int k = 0; k < 3; ++k) {
        s.center[k] = c1[k];
        s.center_vec[k] = cv[k];
    }
    s.radius = radius;
    s.moving = moving ? 1 : 0;
    s.mat = material_index(mat.get());
    spheres.push_back(s);
}

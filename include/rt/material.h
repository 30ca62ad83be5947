// material.h -- drop-in for src/material.h: lambertian(albedo), metal(albedo, fuzz)
// (fuzz clamped to 1 as material.h:33), dielectric(index_of_refraction).
// scatter(r_in, rec, attenuation, scattered) (material.h:11-12) is the reference's
// interface, implemented on the host in fp64 and drawing from the global random_double()
// stream in the reference's order (for one-ray queries); rendering evaluates the same
// materials in the device kernel from describe().  A material subclass without
// describe() has no device form and is rejected at camera::render().
#pragma once
#include <cmath>

#include "color.h"
#include "hittable.h"

class material {
  public:
    virtual ~material() = default;
    virtual bool scatter(const ray& r_in, const hit_record& rec, color& attenuation, ray& scattered) const = 0;
    virtual rt_material describe() const {
        throw std::invalid_argument("material without a device form (lambertian, metal, dielectric)");
    }
};

class lambertian : public material {
  public:
    lambertian(const color& a) : albedo(a) {}
    // material.h:19-25: normal + a random unit vector (no near-zero guard)
    bool scatter(const ray& r_in, const hit_record& rec, color& attenuation, ray& scattered) const override {
        scattered = ray(rec.p, rec.normal + random_unit_vector(), r_in.time());
        attenuation = albedo;
        return true;
    }
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
    // material.h:35-41: mirror direction plus fuzz; absorbed when it points into the surface
    bool scatter(const ray& r_in, const hit_record& rec, color& attenuation, ray& scattered) const override {
        const vec3 mirror = reflect(unit_vector(r_in.direction()), rec.normal);
        scattered = ray(rec.p, mirror + fuzz * random_in_unit_sphere(), r_in.time());
        attenuation = albedo;
        return dot(scattered.direction(), rec.normal) > 0;
    }
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
    // material.h:52-71: refract, or reflect on total internal reflection or with Schlick's
    // probability (no draw when it cannot refract: the reference's short-circuit ||)
    bool scatter(const ray& r_in, const hit_record& rec, color& attenuation, ray& scattered) const override {
        attenuation = color(1.0, 1.0, 1.0);
        const double eta = rec.front_face ? (1.0 / ir) : ir;
        const vec3 d = unit_vector(r_in.direction());
        const double cos_t = std::fmin(dot(-d, rec.normal), 1.0);
        const double sin_t = std::sqrt(1.0 - cos_t * cos_t);
        bool mirror = eta * sin_t > 1.0;
        if (!mirror) mirror = schlick(cos_t, eta) > random_double();
        scattered = ray(rec.p, mirror ? reflect(d, rec.normal) : refract(d, rec.normal, eta), r_in.time());
        return true;
    }
    rt_material describe() const override {
        rt_material m{};
        m.type = RT_DIELECTRIC;
        m.ir = ir;
        return m;
    }

  private:
    double ir;

    // material.h:76-80
    static double schlick(double cosine, double eta) {
        double r0 = (1 - eta) / (1 + eta);
        r0 = r0 * r0;
        return r0 + (1 - r0) * std::pow(1 - cosine, 5);
    }
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

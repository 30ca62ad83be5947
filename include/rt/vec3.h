// vec3.h -- drop-in for src/vec3.h: three doubles with the reference's operators and
// helpers.  Expressions that draw several random numbers are written as constructor
// arguments, as in the reference, so a g++ build draws them in the same (right-to-left)
// order and scene construction reproduces the reference bit for bit.
#pragma once
#include <cmath>
#include <iostream>

class vec3 {
  public:
    double e[3];

    vec3() : e{0, 0, 0} {}
    vec3(double x, double y, double z) : e{x, y, z} {}

    double x() const { return e[0]; }
    double y() const { return e[1]; }
    double z() const { return e[2]; }
    double operator[](int i) const { return e[i]; }
    double& operator[](int i) { return e[i]; }
    vec3 operator-() const { return vec3(-e[0], -e[1], -e[2]); }

    vec3& operator+=(const vec3& o) {
        for (int k = 0; k < 3; ++k) e[k] += o.e[k];
        return *this;
    }
    vec3& operator*=(double t) {
        for (int k = 0; k < 3; ++k) e[k] *= t;
        return *this;
    }
    vec3& operator/=(double t) { return *this *= 1 / t; }

    double length_squared() const { return e[0] * e[0] + e[1] * e[1] + e[2] * e[2]; }
    double length() const { return std::sqrt(length_squared()); }

    bool near_zero() const {
        const double s = 1e-8;
        return std::fabs(e[0]) < s && std::fabs(e[1]) < s && std::fabs(e[2]) < s;
    }
    // per-component |a - b| < 1e-3 (the reference's test tolerance)
    bool similar_to(const vec3& o) const {
        const double s = 1e-3;
        return std::fabs(e[0] - o.e[0]) < s && std::fabs(e[1] - o.e[1]) < s && std::fabs(e[2] - o.e[2]) < s;
    }

    static vec3 random();
    static vec3 random(double min, double max);
};

using point3 = vec3;

inline std::ostream& operator<<(std::ostream& os, const vec3& v) { return os << v[0] << ' ' << v[1] << ' ' << v[2]; }
inline vec3 operator+(const vec3& a, const vec3& b) { return vec3(a.e[0] + b.e[0], a.e[1] + b.e[1], a.e[2] + b.e[2]); }
inline vec3 operator-(const vec3& a, const vec3& b) { return vec3(a.e[0] - b.e[0], a.e[1] - b.e[1], a.e[2] - b.e[2]); }
inline vec3 operator*(const vec3& a, const vec3& b) { return vec3(a.e[0] * b.e[0], a.e[1] * b.e[1], a.e[2] * b.e[2]); }
inline vec3 operator*(double t, const vec3& v) { return vec3(t * v.e[0], t * v.e[1], t * v.e[2]); }
inline vec3 operator*(const vec3& v, double t) { return t * v; }
inline vec3 operator/(const vec3& v, double t) { return (1 / t) * v; }
inline double dot(const vec3& a, const vec3& b) { return a.e[0] * b.e[0] + a.e[1] * b.e[1] + a.e[2] * b.e[2]; }
inline vec3 cross(const vec3& a, const vec3& b) {
    return vec3(a.e[1] * b.e[2] - a.e[2] * b.e[1], a.e[2] * b.e[0] - a.e[0] * b.e[2], a.e[0] * b.e[1] - a.e[1] * b.e[0]);
}
inline vec3 unit_vector(vec3 v) { return v / v.length(); }

double random_double();
double random_double(double, double);
inline vec3 vec3::random() { return vec3(random_double(), random_double(), random_double()); }
inline vec3 vec3::random(double lo, double hi) {
    return vec3(random_double(lo, hi), random_double(lo, hi), random_double(lo, hi));
}

inline vec3 random_in_unit_disk() {
    for (;;) {
        vec3 p(random_double(-1, 1), random_double(-1, 1), 0);
        if (p.length_squared() < 1) return p;
    }
}
inline vec3 random_in_unit_sphere() {
    for (;;) {
        vec3 p = vec3::random(-1, 1);
        if (p.length_squared() < 1) return p;
    }
}
inline vec3 random_unit_vector() { return unit_vector(random_in_unit_sphere()); }
inline vec3 random_on_hemisphere(const vec3& n) {
    vec3 u = random_unit_vector();
    return dot(u, n) > 0.0 ? u : -u;
}
inline vec3 reflect(const vec3& v, const vec3& n) { return v - 2 * dot(v, n) * n; }
inline vec3 refract(const vec3& uv, const vec3& n, double etai_over_etat) {
    double c = std::fmin(dot(-uv, n), 1.0);
    vec3 perp = etai_over_etat * (uv + c * n);
    vec3 par = -std::sqrt(std::fabs(1.0 - perp.length_squared())) * n;
    return perp + par;
}

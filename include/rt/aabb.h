// aabb.h -- drop-in for src/aabb.h: one interval per axis.  The device traverses its own
// flattened float boxes; this host class serves bounding_box() and the BVH builder's API.
#pragma once
#include "interval.h"
#include "vec3.h"

class aabb {
  public:
    interval x, y, z;

    aabb() {}
    aabb(const interval& ix, const interval& iy, const interval& iz) : x(ix), y(iy), z(iz) {}
    aabb(const point3& a, const point3& b)
        : x(std::fmin(a[0], b[0]), std::fmax(a[0], b[0])),
          y(std::fmin(a[1], b[1]), std::fmax(a[1], b[1])),
          z(std::fmin(a[2], b[2]), std::fmax(a[2], b[2])) {}
    aabb(const aabb& a, const aabb& b) : x(a.x, b.x), y(a.y, b.y), z(a.z, b.z) {}

    const interval& axis(int n) const { return n == 1 ? y : (n == 2 ? z : x); }
};

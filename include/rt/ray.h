// ray.h -- drop-in for src/ray.h: origin, (unnormalised) direction and time.
#pragma once
#include "vec3.h"

class ray {
  public:
    ray() : tm(0) {}
    ray(const point3& origin, const vec3& direction, double time = 0.0) : orig(origin), dir(direction), tm(time) {}

    point3 origin() const { return orig; }
    vec3 direction() const { return dir; }
    double time() const { return tm; }
    point3 at(double t) const { return orig + t * dir; }

  private:
    point3 orig;
    vec3 dir;
    double tm;
};

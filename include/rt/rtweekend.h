// rtweekend.h -- drop-in for the reference's src/rtweekend.h (constants, random_double,
// common headers) on top of the MI355X renderer.
//
// random_double() keeps the reference's ONE global std::mt19937 stream (default seed)
// read through uniform_real_distribution<double>(0, 1) (src/rtweekend.h:25-34): host code
// that builds scenes with it (src/main.cpp:17-44) gets the reference's numbers exactly.
// Rendering does not use this stream: the device keys one stream per (pixel, sample).
#pragma once
#include <cmath>
#include <limits>
#include <memory>
#include <random>

using std::make_shared;
using std::shared_ptr;
using std::sqrt;

const double infinity = std::numeric_limits<double>::infinity();
const double pi = 3.1415926535897932385;

inline double degrees_to_radians(double degrees) { return degrees * pi / 180.0; }

namespace rt_host {
// The global reference stream; rt_host::generator() lets camera::ray_color cut a tape of
// uniforms from a copy of it (camera_hip.h).
inline std::mt19937& generator() {
    static std::mt19937 g;
    return g;
}
inline std::uniform_real_distribution<double>& unit_distribution() {
    static std::uniform_real_distribution<double> d(0.0, 1.0);
    return d;
}
}  // namespace rt_host

inline double random_double() { return rt_host::unit_distribution()(rt_host::generator()); }

// [min, max)
inline double random_double(double min, double max) { return min + (max - min) * random_double(); }

#include "interval.h"
#include "ray.h"
#include "vec3.h"

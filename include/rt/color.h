// color.h -- drop-in for src/color.h: the PPM P3 pixel line of write_color.
#pragma once
#include <iostream>

#include "interval.h"
#include "vec3.h"

using color = vec3;

inline double linear_to_gamma(double linear_component) { return std::sqrt(linear_component); }

// color.h:14-35: average over the samples, gamma 2, clamp to [0, 0.999], int(256 x).
inline int quantize_component(double sum, double scale) {
    static const interval intensity(0.000, 0.999);
    return static_cast<int>(256 * intensity.clamp(linear_to_gamma(sum * scale)));
}

inline void write_color(std::ostream& out, color pixel_color, int samples_per_pixel) {
    const double scale = 1.0 / samples_per_pixel;
    out << quantize_component(pixel_color.x(), scale) << ' ' << quantize_component(pixel_color.y(), scale) << ' '
        << quantize_component(pixel_color.z(), scale) << '\n';
}

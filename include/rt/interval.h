// interval.h -- drop-in for src/interval.h: a closed range [min, max] with the
// reference's strict `surrounds` and clamp.
#pragma once
#include <cmath>

class interval {
  public:
    double min, max;

    interval() : min(+std::numeric_limits<double>::infinity()), max(-std::numeric_limits<double>::infinity()) {}
    interval(double lo, double hi) : min(lo), max(hi) {}
    interval(const interval& a, const interval& b) : min(std::fmin(a.min, b.min)), max(std::fmax(a.max, b.max)) {}

    double size() const { return max - min; }
    bool contains(double x) const { return min <= x && x <= max; }
    bool surrounds(double x) const { return min < x && x < max; }
    double clamp(double x) const { return x < min ? min : (x > max ? max : x); }
    interval expand(double delta) const { return interval(min - delta / 2, max + delta / 2); }
};

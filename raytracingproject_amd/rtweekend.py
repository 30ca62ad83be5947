"""Host-side random stream of the reference (src/rtweekend.h:25-34).

random_double() draws from ONE global std::mt19937 (default seed 5489) through
std::uniform_real_distribution<double>(0, 1).  libstdc++'s generate_canonical takes two
32-bit words g1, g2 and returns (g1 + g2 * 2^32) / 2^64 (one rounding), mapping 1.0 to
nextafter(1, 0).  This module restates that stream on the host so scene construction
(src/main.cpp:17-44) and direct get_ray/ray_color calls (tests/tests.cpp:41-42) consume
exactly the reference's numbers.  It is host setup, not the render path: rendering uses
the per-(pixel, sample) counter streams on the GPU.
"""
from __future__ import annotations

import math

_N, _M = 624, 397


class MT19937:
    """std::mt19937 (32-bit Mersenne Twister)."""

    def __init__(self, seed: int = 5489):
        self.mt = [0] * _N
        self.mt[0] = seed & 0xFFFFFFFF
        for k in range(1, _N):
            self.mt[k] = (1812433253 * (self.mt[k - 1] ^ (self.mt[k - 1] >> 30)) + k) & 0xFFFFFFFF
        self.idx = _N

    def copy(self) -> "MT19937":
        c = MT19937.__new__(MT19937)
        c.mt = list(self.mt)
        c.idx = self.idx
        return c

    def _twist(self) -> None:
        mt = self.mt
        for k in range(_N):
            y = (mt[k] & 0x80000000) | (mt[(k + 1) % _N] & 0x7FFFFFFF)
            mt[k] = mt[(k + _M) % _N] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
        self.idx = 0

    def next32(self) -> int:
        if self.idx >= _N:
            self._twist()
        y = self.mt[self.idx]
        self.idx += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y & 0xFFFFFFFF

    def canonical(self) -> float:
        g1 = float(self.next32())
        g2 = float(self.next32())
        u = (g1 + g2 * 4294967296.0) / 18446744073709551616.0
        if u >= 1.0:
            u = math.nextafter(1.0, 0.0)
        return u * (1.0 - 0.0) + 0.0


_generator = MT19937()


def reset_stream(seed: int = 5489) -> None:
    """Restart the global stream (a fresh process of the reference)."""
    global _generator
    _generator = MT19937(seed)


def stream() -> MT19937:
    return _generator


def random_double(lo: float | None = None, hi: float | None = None) -> float:
    """rtweekend.h:25-34."""
    u = _generator.canonical()
    if lo is None:
        return u
    return lo + (hi - lo) * u


infinity = math.inf
pi = 3.1415926535897932385


def degrees_to_radians(degrees: float) -> float:
    return degrees * pi / 180.0

// rt_node4q.h -- Node4 -> Node4Q (rt_scene.h): the quantised 64-B mesh node, from the same
// code on the host (host-built trees, rt_abi.cpp) and on the GPU (LBVH trees, rt_lbvh.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "rt_scene.h"

namespace rtx {

// One node: per axis the corner p (the smallest child lo, an exact float) and the
// smallest e in [-126, 127] with (largest hi - p) <= 255 * 2^e; each child's lo plane
// rounded down and hi plane rounded up to that grid (fp64: the differences of two floats
// and the divisions by 2^e are exact, so floor / ceil are the exact grid cells).
__host__ __device__ inline void quantize_node4(const Node4& n, Node4Q& q) {
    const float* lo[3] = {n.lox, n.loy, n.loz};
    const float* hi[3] = {n.hix, n.hiy, n.hiz};
    q.ex = 0;
    for (int a = 0; a < 3; ++a) {
        q.qlo[a] = q.qhi[a] = 0;
        double mn = HUGE_VAL, mx = -HUGE_VAL;
        for (int c = 0; c < 4; ++c) {
            if (n.ref[c] == MREF_EMPTY) continue;
            mn = lo[a][c] < mn ? (double)lo[a][c] : mn;
            mx = hi[a][c] > mx ? (double)hi[a][c] : mx;
        }
        if (!(mn <= mx)) {   // no child (never in a built tree): a valid, empty encoding
            q.p[a] = 0.f;
            q.ex |= 1u << (8 * a);
            continue;
        }
        q.p[a] = (float)mn;
        const double ext = mx - mn;
        int e = ext > 0 ? ilogb(ext / 255.0) : -126;   // then the exact smallest e
        e = e < -126 ? -126 : (e > 127 ? 127 : e);
        while (e < 127 && ext > 255.0 * ldexp(1.0, e)) ++e;
        while (e > -126 && ext <= 255.0 * ldexp(1.0, e - 1)) --e;
        const double s = ldexp(1.0, e);
        q.ex |= (uint32_t)(e + 127) << (8 * a);
        for (int c = 0; c < 4; ++c) {
            if (n.ref[c] == MREF_EMPTY) continue;
            double ql = floor(((double)lo[a][c] - mn) / s), qh = ceil(((double)hi[a][c] - mn) / s);
            ql = ql < 0 ? 0 : (ql > 255 ? 255 : ql);
            qh = qh < 0 ? 0 : (qh > 255 ? 255 : qh);
            q.qlo[a] |= (uint32_t)ql << (8 * c);
            q.qhi[a] |= (uint32_t)qh << (8 * c);
        }
    }
    q.pad[0] = q.pad[1] = 0;
    for (int c = 0; c < 4; ++c) q.ref[c] = n.ref[c];
}

}  // namespace rtx

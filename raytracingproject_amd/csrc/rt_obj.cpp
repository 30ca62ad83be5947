// rt_obj.cpp -- Wavefront OBJ geometry loader (host).  The reference's model loader is an
// empty stub (src/vulkan/model_loader.h:17-19) next to a vendored tinyobjloader that is
// never called (dependencies/tinyobjloader, LoadObj at tiny_obj_loader.h:605); this is
// the loader the mesh path needs: `v x y z` positions and `f` faces (v, v/vt, v//vn,
// v/vt/vn; negative = relative).  Polygons are triangulated exactly as tinyobjloader's
// default ("simple") LoadObj does, so a model yields the same triangles through either
// loader: quads split along the shorter diagonal, larger polygons by its ear clipping
// (both in float, its real_t).  Faces with fewer than 3 vertices are skipped, as there.
// Other statements (vt, vn, o, g, s, usemtl, mtllib, ...) are skipped.  Parsing is
// cross-checked against tinyobjloader in tests/test_mesh.py (oracle/_ref/obj_dump and
// committed dumps under tests/golden/).
//
// Untrusted input (tests/test_sanitize.py runs this file under ASan/UBSan over the
// malformed-OBJ corpus in tests/golden/obj_malformed/ and a mutation fuzzer):
//  * lines end at \n, \r\n or a lone \r (tinyobjloader's safeGetline); a NUL byte ends
//    the statement (the rest of its line is skipped, as tinyobjloader's C strings do);
//  * a coordinate is one token (up to a space, tab or line end) read with
//    tinyobjloader's number grammar (tryParseDouble, tiny_obj_loader.h:891-1021:
//    [+-](digits[.digits]|.digits)[(e|E)[+-]digits], longest prefix; a token that does
//    not start a number -- "nan", "inf", "abc" -- or a missing one gives 0, as
//    parseV's defaults do, tiny_obj_loader.h:1062-1071);
//  * a coordinate that overflows to +-inf is an error (RT_ERR_INVALID): the renderer
//    cannot bound it;
//  * face indices must name an existing vertex (0, past the end, or before the first
//    for a relative index: RT_ERR_INVALID; tinyobjloader refuses 0 but passes the
//    others through unchecked); trailing characters of an index token are skipped, as
//    atoi does there; a `#` ends a face line (tinyobjloader fails on it);
//  * a face with more than RT_OBJ_MAX_FACE_VERTICES corners is RT_ERR_LIMIT: the ear
//    clipping is quadratic in the corner count for convex polygons and cubic in the
//    worst case;
//  * allocation failure is RT_ERR_LIMIT (no exception leaves the C ABI).
#include <cerrno>
#include <climits>
#include <clocale>
#include <locale.h>
#include <stdlib.h>
#include <new>
#include <stdexcept>
#include <cmath>
#include <limits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rt_hip.h"

namespace {

inline bool is_digit(char c) { return c >= '0' && c <= '9'; }
inline bool is_eol(char c) { return c == '\n' || c == '\r' || c == '\0'; }
inline bool is_sep(char c) { return c == ' ' || c == '\t' || is_eol(c); }

// One face index token (v, v/vt, v//vn, v/vt/vn; atoi-like: trailing characters of the
// token are skipped); false unless it names one of the nverts vertices.
bool parse_index(const char*& p, long nverts, long& out) {
    char* end = nullptr;
    errno = 0;
    const long v = std::strtol(p, &end, 10);
    if (end == p || errno == ERANGE) return false;
    p = end;
    while (!is_sep(*p)) ++p;
    if (v > 0)
        out = v - 1;
    else if (v < 0 && v >= -nverts)
        out = nverts + v;
    else
        return false;
    return out >= 0 && out < nverts;
}

// One coordinate: the next token of the line read with tinyobjloader's grammar
// (tryParseDouble, tiny_obj_loader.h:891-1021), `dflt` when the token is missing or does
// not start a number (parseReal's default, :1023-1031).  The accepted prefix is converted
// by strtod_l in the "C" locale (correctly rounded like strtod, but a host that set
// LC_NUMERIC to a comma-decimal locale cannot turn "1.5" into 1; tinyobjloader's own
// grammar has no locale either), from a stack copy of the prefix for ordinary tokens.
double parse_coord(const char*& p, double dflt) {
    while (*p == ' ' || *p == '\t') ++p;
    const char* tok = p;
    while (!is_sep(*p)) ++p;
    const char* q = tok;
    bool neg = false;
    if (q < p && (*q == '+' || *q == '-')) neg = *q++ == '-';
    const bool lead_dot = q < p && *q == '.';
    size_t digits = 0;
    if (!lead_dot) {
        while (q < p && is_digit(*q)) ++q, ++digits;
        if (digits == 0) return dflt;
    }
    if (q < p && *q == '.') {
        ++q;
        while (q < p && is_digit(*q)) ++q, ++digits;
    }
    if (q < p && (*q == 'e' || *q == 'E')) {
        ++q;
        if (q < p && (*q == '+' || *q == '-')) ++q;
        int exp_digits = 0;
        long e = 0;
        while (q < p && is_digit(*q)) {
            if (e > 2147483647L / 10) return dflt;   // its exponent overflow check
            e = e * 10 + (*q++ - '0');
            ++exp_digits;
        }
        if (exp_digits == 0) return dflt;           // "1e", "1e+" fail there
    }
    if (digits == 0) return neg ? -0.0 : 0.0;       // "." / "-." assemble to a zero
    static const locale_t c_locale = newlocale(LC_ALL_MASK, "C", (locale_t)0);
    const size_t len = (size_t)(q - tok);
    char buf[96];
    if (len < sizeof buf) {
        std::memcpy(buf, tok, len);
        buf[len] = '\0';
        return strtod_l(buf, nullptr, c_locale);
    }
    const std::string num(tok, q);   // very long digit strings
    return strtod_l(num.c_str(), nullptr, c_locale);
}

// pnpoly (W. R. Franklin), as tiny_obj_loader.h:1411-1423 uses it
bool pnpoly3(const float* vx, const float* vy, float tx, float ty) {
    bool c = false;
    for (int i = 0, j = 2; i < 3; j = i++) {
        if (((vy[i] > ty) != (vy[j] > ty)) && (tx < (vx[j] - vx[i]) * (ty - vy[i]) / (vy[j] - vy[i]) + vx[i])) c = !c;
    }
    return c;
}

// One face -> triangles (index triples), tinyobjloader's triangulation
// (tiny_obj_loader.h:1488-1584 quads, :1706-1925 ear clipping) restated.
void triangulate(const std::vector<long>& poly, const std::vector<double>& verts, std::vector<int32_t>& tris) {
    auto V = [&](long vi, int a) -> float { return (float)verts[(size_t)vi * 3 + a]; };
    auto emit = [&](long a, long b, long c) {
        tris.push_back((int32_t)a);
        tris.push_back((int32_t)b);
        tris.push_back((int32_t)c);
    };
    const size_t n = poly.size();
    if (n == 3) {
        emit(poly[0], poly[1], poly[2]);
        return;
    }
    if (n == 4) {
        const long i0 = poly[0], i1 = poly[1], i2 = poly[2], i3 = poly[3];
        const float e02x = V(i2, 0) - V(i0, 0), e02y = V(i2, 1) - V(i0, 1), e02z = V(i2, 2) - V(i0, 2);
        const float e13x = V(i3, 0) - V(i1, 0), e13y = V(i3, 1) - V(i1, 1), e13z = V(i3, 2) - V(i1, 2);
        const float sqr02 = e02x * e02x + e02y * e02y + e02z * e02z;
        const float sqr13 = e13x * e13x + e13y * e13y + e13z * e13z;
        if (sqr02 < sqr13) {
            emit(i0, i1, i2);
            emit(i0, i2, i3);
        } else {
            emit(i0, i1, i3);
            emit(i1, i2, i3);
        }
        return;
    }
    // projection plane from the first corner with a non-degenerate cross product
    int axes[2] = {1, 2};
    for (size_t k = 0; k < n; ++k) {
        const long a = poly[k % n], b = poly[(k + 1) % n], c = poly[(k + 2) % n];
        const float e0x = V(b, 0) - V(a, 0), e0y = V(b, 1) - V(a, 1), e0z = V(b, 2) - V(a, 2);
        const float e1x = V(c, 0) - V(b, 0), e1y = V(c, 1) - V(b, 1), e1z = V(c, 2) - V(b, 2);
        const float cx = std::fabs(e0y * e1z - e0z * e1y);
        const float cy = std::fabs(e0z * e1x - e0x * e1z);
        const float cz = std::fabs(e0x * e1y - e0y * e1x);
        const float eps = std::numeric_limits<float>::epsilon();
        if (cx > eps || cy > eps || cz > eps) {
            if (!(cx > cy && cx > cz)) {
                axes[0] = 0;
                if (cz > cx && cz > cy) axes[1] = 1;
            }
            break;
        }
    }
    std::vector<long> rem = poly;
    size_t guess = 0, iters = n, prev = n;
    while (rem.size() > 3 && iters > 0) {
        const size_t np = rem.size();
        if (guess >= np) guess -= np;
        if (prev != np) {
            prev = np;
            iters = np;
        } else {
            --iters;
        }
        long ind[3];
        float vx[3], vy[3];
        for (int k = 0; k < 3; ++k) {
            ind[k] = rem[(guess + k) % np];
            vx[k] = V(ind[k], axes[0]);
            vy[k] = V(ind[k], axes[1]);
        }
        const float e0x = vx[1] - vx[0], e0y = vy[1] - vy[0], e1x = vx[2] - vx[1], e1y = vy[2] - vy[1];
        const float cross = e0x * e1y - e0y * e1x;
        const float area = (vx[0] * vy[1] - vy[0] * vx[1]) * 0.5f;
        if (cross * area < 0.0f) {
            guess += 1;
            continue;
        }
        bool overlap = false;
        for (size_t o = 3; o < np; ++o) {
            const long q = rem[(guess + o) % np];
            if (pnpoly3(vx, vy, V(q, axes[0]), V(q, axes[1]))) {
                overlap = true;
                break;
            }
        }
        if (overlap) {
            guess += 1;
            continue;
        }
        emit(ind[0], ind[1], ind[2]);
        rem.erase(rem.begin() + (long)((guess + 1) % np));
    }
    if (rem.size() == 3) emit(rem[0], rem[1], rem[2]);
}

}  // namespace

namespace {

int load(const char* path, rt_obj_mesh* out) {
    FILE* f = std::fopen(path, "rb");
    if (!f) return RT_ERR_INVALID;
    std::vector<char> text;
    {
        long n = -1;
        if (std::fseek(f, 0, SEEK_END) == 0) n = std::ftell(f);
        if (n < 0 || n == LONG_MAX || std::fseek(f, 0, SEEK_SET) != 0) {   // not a regular file
            std::fclose(f);
            return RT_ERR_INVALID;
        }
        text.resize((size_t)n + 1);
        const size_t got = std::fread(text.data(), 1, (size_t)n, f);
        std::fclose(f);
        text[got] = '\0';
    }
    std::vector<double> verts;
    std::vector<int32_t> tris;
    long faces = 0;
    const char* p = text.data();
    const char* const end = text.data() + text.size() - 1;
    std::vector<long> poly;
    while (p < end) {
        while (*p == ' ' || *p == '\t') ++p;
        if (p[0] == 'v' && (p[1] == ' ' || p[1] == '\t')) {
            p += 2;
            for (int k = 0; k < 3; ++k) {
                const double x = parse_coord(p, 0.0);
                if (!std::isfinite(x)) return RT_ERR_INVALID;
                verts.push_back(x);
            }
        } else if (p[0] == 'f' && (p[1] == ' ' || p[1] == '\t')) {
            p += 2;
            poly.clear();
            const long nv = (long)(verts.size() / 3);
            for (;;) {
                while (*p == ' ' || *p == '\t') ++p;
                if (is_eol(*p) || *p == '#') break;
                long idx;
                if (!parse_index(p, nv, idx)) return RT_ERR_INVALID;
                if (poly.size() >= (size_t)RT_OBJ_MAX_FACE_VERTICES) return RT_ERR_LIMIT;
                poly.push_back(idx);
            }
            if (poly.size() >= 3) {   // tinyobjloader skips degenerate faces
                ++faces;
                triangulate(poly, verts, tris);
                if (tris.size() / 3 > (size_t)INT32_MAX) return RT_ERR_LIMIT;
            }
        }
        // rest of line (comments, unsupported statements; text after a NUL byte, which
        // ends tinyobjloader's C-string view of the line)
        while (p < end && *p != '\n' && *p != '\r') ++p;
        if (p < end) ++p;          // \n, \r (a \r\n pair leaves an empty line)
    }
    if (verts.size() / 3 > (size_t)INT32_MAX || faces > INT32_MAX) return RT_ERR_LIMIT;
    out->num_vertices = (int32_t)(verts.size() / 3);
    out->num_faces = (int32_t)faces;
    out->num_triangles = (int32_t)(tris.size() / 3);
    out->vertices = (double*)std::malloc(verts.size() * sizeof(double) + 8);
    out->indices = (int32_t*)std::malloc(tris.size() * sizeof(int32_t) + 4);
    if (!out->vertices || !out->indices) {
        std::free(out->vertices);
        std::free(out->indices);
        std::memset(out, 0, sizeof(*out));
        return RT_ERR_LIMIT;
    }
    if (!verts.empty()) std::memcpy(out->vertices, verts.data(), verts.size() * sizeof(double));
    if (!tris.empty()) std::memcpy(out->indices, tris.data(), tris.size() * sizeof(int32_t));
    return RT_OK;
}

}  // namespace

extern "C" int rt_obj_load(const char* path, rt_obj_mesh* out) {
    if (!path || !out) return RT_ERR_INVALID;
    std::memset(out, 0, sizeof(*out));
    try {
        return load(path, out);
    } catch (const std::bad_alloc&) {
        return RT_ERR_LIMIT;
    } catch (const std::length_error&) {
        return RT_ERR_LIMIT;
    }
}

extern "C" void rt_obj_free(rt_obj_mesh* m) {
    if (!m) return;
    std::free(m->vertices);
    std::free(m->indices);
    std::memset(m, 0, sizeof(*m));
}

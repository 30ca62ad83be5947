// Host code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5
// "Sanitizers"; the reference's own ASan flags are commented out, CMakeLists.txt:18-23).
// Built by `python -m raytracingproject_amd.build --sanitize` together with the product's
// host sources (csrc/rt_obj.cpp, csrc/rt_bvh.cpp) and the oracle (oracle/rt_oracle.c),
// all with -fsanitize=address,undefined -fno-sanitize-recover=all; tests/test_sanitize.py
// runs it.  Any sanitizer report aborts with a non-zero exit code.
//
//   san_driver obj FILE...              rt_obj_load each file; print "<status> <nv> <nf> <nt>";
//                                       loaded meshes go through build_mesh_bvh, and the
//                                       4-wide tree is checked (every triangle once, refs in range)
//   san_driver fuzz SEED ITERS FILE...  mutation fuzzer over the given OBJ files (byte flips,
//                                       token splices, truncation, line duplication, number
//                                       edge cases); every mutant is loaded and, if it loads,
//                                       its tree built and checked
//   san_driver spheres FILE             rt_sphere records (tests/test_sanitize.py writes the
//                                       random scene): build_bvh over several parameter sets and
//                                       adversarial variants (coincident centres, huge/NaN
//                                       coordinates), then oracle renders (counter + mt modes)
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <unistd.h>
#include <string>
#include <vector>

#include "../../oracle/rt_oracle.h"
#include "../../raytracingproject_amd/csrc/rt_bvh.h"

using namespace rtx;

namespace {

int fail_count = 0;
int grids_built = 0;

void check(bool ok, const char* what) {
    if (!ok) {
        std::printf("CHECK FAILED: %s\n", what);
        ++fail_count;
    }
}

// every triangle index appears exactly once among the leaves; inner refs in range
void check_mesh_tree(const MeshBvh& b, int ntri) {
    std::vector<int> seen(ntri, 0);
    for (int k : b.order) {
        check(k >= 0 && k < ntri, "order index in range");
        if (k >= 0 && k < ntri) seen[k]++;
    }
    for (int k = 0; k < ntri; ++k) check(seen[k] == 1, "triangle in exactly one leaf");
    const uint32_t n4 = (uint32_t)b.nodes4.size();
    for (const Node4& nd : b.nodes4)
        for (uint32_t r : nd.ref) {
            if (r == MREF_EMPTY) continue;
            if (r & MREF_LEAF) {
                const uint32_t first = r & 0xffffffu, count = ((r >> 24) & 0x7fu) + 1;
                check(first + count <= b.order.size(), "leaf range in order");
            } else {
                check(r < n4, "inner ref in range");
            }
        }
}

int load_and_build(const char* path, bool print) {
    rt_obj_mesh m;
    const int rc = rt_obj_load(path, &m);
    if (print) std::printf("%d %d %d %d\n", rc, m.num_vertices, m.num_faces, m.num_triangles);
    if (rc != RT_OK) return rc;
    std::vector<rt_triangle> T(m.num_triangles);
    for (int k = 0; k < m.num_triangles; ++k) {
        for (int c = 0; c < 3; ++c) {
            const int vi = m.indices[3 * k + c];
            check(vi >= 0 && vi < m.num_vertices, "triangle index in range");
            double* dst = c == 0 ? T[k].v0 : c == 1 ? T[k].v1 : T[k].v2;
            for (int a = 0; a < 3; ++a) dst[a] = m.vertices[3 * vi + a];
        }
        T[k].mat = 0;
        T[k].pad = 0;
    }
    rt_obj_free(&m);
    for (int leaf : {1, 2, 8}) {
        MeshBvh b;
        std::string err;
        if (build_mesh_bvh(T.data(), (int)T.size(), leaf, 1.5, b, err)) check_mesh_tree(b, (int)T.size());
        else if (print) std::printf("  build(leaf %d): %s\n", leaf, err.c_str());
    }
    return rc;
}

std::string read_file(const char* path) {
    std::string s;
    if (FILE* f = std::fopen(path, "rb")) {
        char buf[65536];
        size_t n;
        while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) s.append(buf, n);
        std::fclose(f);
    }
    return s;
}

const char* const TOKENS[] = {"v ", "f ", "vt ", "vn ", "#", "\n", "\r", "\r\n", " ", "\t", "/", "//", "-", "+",
                              ".", "e", "E", "0", "-1", "-999999", "2147483648", "99999999999999999999",
                              "1e308", "1e999", "-1e-999", "nan", "inf", "0x1p3", "1.5abc", "1/2/3", "1//",
                              "f 1 2 3 4 5 6 7 8 9", "v 1 2", "f 1", "\0"};

std::string mutate(std::mt19937& g, std::string s) {
    const int ops = 1 + (int)(g() % 4);
    for (int k = 0; k < ops; ++k) {
        const size_t n = s.size();
        switch (g() % 6) {
            case 0:   // flip a byte
                if (n) s[g() % n] = (char)(g() & 0xff);
                break;
            case 1: {   // splice a token
                const char* t = TOKENS[g() % (sizeof TOKENS / sizeof *TOKENS)];
                const size_t len = *t ? std::strlen(t) : 1;
                s.insert(n ? g() % (n + 1) : 0, t, len);
                break;
            }
            case 2:   // truncate
                if (n) s.resize(g() % n);
                break;
            case 3: {   // duplicate a line
                if (!n) break;
                const size_t a = s.rfind('\n', g() % n);
                const size_t b0 = a == std::string::npos ? 0 : a + 1;
                const size_t b1 = s.find('\n', b0);
                const std::string line = s.substr(b0, b1 == std::string::npos ? std::string::npos : b1 - b0 + 1);
                s.insert(b0, line);
                break;
            }
            case 4:   // delete a span
                if (n) {
                    const size_t a = g() % n;
                    s.erase(a, 1 + g() % 16);
                }
                break;
            default:   // replace a digit run by an edge-case number
                if (n) {
                    size_t a = g() % n;
                    while (a < n && !(s[a] >= '0' && s[a] <= '9')) ++a;
                    size_t b = a;
                    while (b < n && s[b] >= '0' && s[b] <= '9') ++b;
                    if (a < n) s.replace(a, b - a, TOKENS[17 + g() % 12]);
                }
        }
    }
    return s;
}

int cmd_fuzz(unsigned seed, int iters, int nfiles, char** files) {
    std::vector<std::string> base;
    for (int k = 0; k < nfiles; ++k) base.push_back(read_file(files[k]));
    std::mt19937 g(seed);
    char path[] = "/tmp/rt_san_fuzz_XXXXXX";
    const int fd = mkstemp(path);
    if (fd < 0) return 2;
    close(fd);
    int loaded = 0;
    for (int it = 0; it < iters; ++it) {
        const std::string m = mutate(g, base[g() % base.size()]);
        FILE* f = std::fopen(path, "wb");
        std::fwrite(m.data(), 1, m.size(), f);
        std::fclose(f);
        if (load_and_build(path, false) == RT_OK) ++loaded;
    }
    std::remove(path);
    std::printf("fuzz iterations %d loaded %d\n", iters, loaded);
    return 0;
}

// ---- the uniform sphere grid (build_sphere_grid) over a built tree's sphere order: its
// layout, and a walk restating the kernel's (rt_device.h closest_hit, TRAV_GRID: fp32 plane
// distances, the same stop test) that must reach the brute-force closest hit of every ray.
double sphere_t(const SphereF& q, const double o[3], const double d[3], double tm) {
    double c[3], oc[3], a = 0, h = 0, cc = 0;
    for (int x = 0; x < 3; ++x) {
        c[x] = (double)q.c[x] + tm * (double)q.cv[x];
        oc[x] = c[x] - o[x];
        a += d[x] * d[x];
        h += d[x] * oc[x];
        cc += oc[x] * oc[x];
    }
    cc -= (double)q.r * (double)q.r;
    const double disc = h * h - a * cc;
    if (disc < 0) return INFINITY;
    const double sq = std::sqrt(disc);
    double t = (h - sq) / a;
    if (!(t > 0.001)) t = (h + sq) / a;
    return t > 0.001 ? t : INFINITY;
}

long long walked = 0, walked_flat = 0, beyond = 0, beyond_bad = 0;

int check_grid(const std::vector<SphereF>& sf, int front, double density, int slabs, std::mt19937& g, int rays) {
    GridHdr hd;
    std::vector<unsigned char> buf;
    if (!build_sphere_grid(sf.data(), front, (int)sf.size(), density, slabs, (int)sizeof(SphereF), hd, buf)) return 0;
    const uint32_t pad = (uint32_t)hd.res[0] * hd.res[1];   // empty layers either side
    const uint32_t* cells = (const uint32_t*)buf.data() + pad;
    // list entries: record byte offsets from the buffer's start (records follow the buffer);
    // list positions are byte offsets from the buffer's start: the lists start at word lb
    const uint32_t lb = hd.n_cells + 2 * pad;
    const uint32_t* offs = (const uint32_t*)buf.data() + lb;
    std::vector<uint32_t> idv;
    check(hd.n_slab == slabs && hd.slab_k == (float)slabs && hd.slab_off % 16 == 0 &&
              hd.slab_off >= (hd.n_cells + 2 * pad) * 4 && hd.slab_off + (size_t)(slabs + 1) * 24 <= buf.size(),
          "time-slab boxes after the lists");
    const size_t nent = (hd.slab_off - (size_t)(hd.n_cells + 2 * pad) * 4) / 4;
    for (size_t k = 0; k < nent; ++k) {
        const uint32_t o = offs[k];
        idv.push_back(o >= buf.size() && (o - buf.size()) % sizeof(SphereF) == 0 ? (uint32_t)((o - buf.size()) / sizeof(SphereF))
                                                                                 : 0xffffffffu);
    }
    const uint32_t* ids = idv.data();
    // (a cell word's first / end positions as entry indices; a pad cell's word is 0: none)
    auto first_of = [&](uint32_t w) {
        if (w == 0) return 0u;
        check((w & GRID_POS_MASK) % 4 == 0 && (w & GRID_POS_MASK) / 4 >= lb, "list position in the lists");
        return (w & GRID_POS_MASK) / 4 - lb;
    };
    auto end_of = [&](uint32_t w) { return w == 0 ? 0u : (w >> GRID_POS_BITS) / 4 - lb; };
    for (uint32_t c = 0; c < pad; ++c) check(cells[(int)c - (int)pad] == 0 && cells[hd.n_cells + c] == 0, "pad cells empty");
    check(hd.n_cells == (uint32_t)hd.res[0] * hd.res[1] * hd.res[2], "cell count");
    check(buf.size() % sizeof(Node) == 0 && buf.size() <= GRID_MAX_BYTES + sizeof(Node), "buffer size");
    uint32_t run = 0;
    for (uint32_t c = 0; c < hd.n_cells; ++c) {
        check(first_of(cells[c]) == run && end_of(cells[c]) >= first_of(cells[c]), "cell lists contiguous");
        const uint32_t n = end_of(cells[c]) - first_of(cells[c]);
        for (uint32_t k = run; k < run + n; ++k)
            check(k < idv.size() && ids[k] >= (uint32_t)front && ids[k] < sf.size(), "listed record offset in range");
        run += n;
    }
    check((size_t)(hd.n_cells + 2 * pad) * 4 + (size_t)run * 4 <= hd.slab_off, "lists before the slab boxes");
    // the time-slab boxes: within the grid box (the last one is it), and each holding every
    // listed sphere at times across its slab, including the slab's edges
    const float* sb = (const float*)(buf.data() + hd.slab_off);
    // (lo, hi) pairs per axis: box k's axis x at sb[(x * (slabs + 1) + k) * 2]
    auto slo = [&](int k, int x) { return sb[((size_t)x * (slabs + 1) + k) * 2]; };
    auto shi = [&](int k, int x) { return sb[((size_t)x * (slabs + 1) + k) * 2 + 1]; };
    for (int x = 0; x < 3; ++x)
        check(slo(slabs, x) == hd.lo[x] && shi(slabs, x) == hd.hi[x], "last slab box = grid box");
    for (int k = 0; k < slabs; ++k)
        for (int q = 0; q <= 8; ++q) {
            const double tm = ((double)k + q / 8.0) / slabs;
            for (size_t i = front; i < sf.size(); ++i)
                for (int x = 0; x < 3; ++x) {
                    const double c = (double)sf[i].c[x] + tm * (double)sf[i].cv[x], r = std::fabs((double)sf[i].r);
                    check(slo(k, x) >= hd.lo[x] && shi(k, x) <= hd.hi[x], "slab box inside the grid box");
                    check(c - r >= slo(k, x) && c + r <= shi(k, x), "slab box holds its spheres");
                }
        }
    // the walk's reach (r06): the kernel walks only launches whose rays all start within
    // +-far_o (rt_abi.cpp grid_reach_ok), which must cover rays from near the grid
    const int max_steps = hd.res[0] + hd.res[1] + hd.res[2] + 2;
    double gext = 0;
    for (int x = 0; x < 3; ++x) gext = std::max(gext, std::max(std::fabs((double)hd.lo[x]), std::fabs((double)hd.hi[x])));
    check(hd.far_o > 2 * gext, "far_o covers rays from near the grid");
    // the walk, as the kernel does it (rt_device.h closest_hit, TRAV_GRID: one loop, a cell
    // step whenever the lane's list is done), for random rays through the grid's box and from
    // origins 10 .. 10^9 cells away from it -- those within far_o must walk exactly, in at most
    // max_steps steps, within the pad layers; those beyond (never walked by the product) are
    // walked here too under a guard, to count how often the bound is needed
    std::uniform_real_distribution<double> u(0.0, 1.0);
    int misses = 0;
    const float INF = INFINITY;
    for (int r = 0; r < rays; ++r) {
        double o[3], d[3];
        const bool far = r % 4 == 3;
        double dist_cells = 0;
        for (int x = 0; x < 3; ++x) {
            const double span = (double)hd.hi[x] - hd.lo[x];
            o[x] = hd.lo[x] - 0.2 * span + 1.4 * span * u(g);
            d[x] = u(g) * 2 - 1;
        }
        if (far) {
            // aimed at a point of the box from 10 .. 10^9 cell sizes away; some along a plane of
            // two axes (a zero direction component: the slab products overflow past ~2^27 units)
            dist_cells = std::pow(10.0, 1.0 + 8.0 * u(g));
            if (r % 40 == 3) d[(r / 40) % 3] = 0.0;
            double len = 0;
            for (int x = 0; x < 3; ++x) len += d[x] * d[x];
            len = std::sqrt(len);
            for (int x = 0; x < 3; ++x) {
                const double tgt = hd.lo[x] + ((double)hd.hi[x] - hd.lo[x]) * u(g);
                o[x] = tgt - d[x] / len * dist_cells * hd.cs[0];
            }
        }
        // (every tenth ray at a slab edge: the kernel's rounding of t * slabs)
        double tm = u(g);
        if (r % 10 == 0) tm = std::nextafter((double)(int)(tm * slabs) / slabs, r % 20 == 0 ? 2.0 : -1.0);
        if (r % 50 == 0) tm = r % 100 == 0 ? 0.0 : 1.0;
        double best = INFINITY;
        int best_id = -1;
        for (size_t k = front; k < sf.size(); ++k) {
            const double t = sphere_t(sf[k], o, d, tm);
            if (t < best) best = t, best_id = (int)k;
        }
        // the kernel's walk (fp32), candidates tested exactly as above
        const float of[3] = {(float)o[0], (float)o[1], (float)o[2]}, df[3] = {(float)d[0], (float)d[1], (float)d[2]};
        float inv[3], oi[3], t0[3], t1[3];
        const float tmf = (float)tm;
        const int sk = tmf >= 0.f && tmf <= 1.f ? std::min((int)(tmf * hd.slab_k), hd.n_slab - 1) : hd.n_slab;
        const float om = std::fmax(std::fmax(std::fabs(of[0]), std::fabs(of[1])), std::fabs(of[2]));
        const bool far_o = !(om <= hd.far_o);
        check(!far_o || far, "rays near the grid are within far_o");
        for (int x = 0; x < 3; ++x) {
            inv[x] = 1.0f / (df[x] + std::copysign(0x1p-100f, df[x]));
            oi[x] = of[x] * inv[x];
            t0[x] = std::fmaf(slo(sk, x), inv[x], -oi[x]);
            t1[x] = std::fmaf(shi(sk, x), inv[x], -oi[x]);
        }
        const float tn = std::fmax(std::fmax(std::fmin(t0[0], t1[0]), std::fmin(t0[1], t1[1])),
                                   std::fmax(std::fmin(t0[2], t1[2]), 0.001f));
        const float tf = std::fmin(std::fmin(std::fmax(t0[0], t1[0]), std::fmax(t0[1], t1[1])),
                                   std::fmin(std::fmax(t0[2], t1[2]), INF));
        // the 3-D walk, and on a grid one cell tall in y also the flat one (TRAV_GFLAT: steps
        // in x and z only, from the entry cell's x and z)
        for (int flat = 0; flat < (hd.res[1] == 1 ? 2 : 1); ++flat) {
        double tmax = INFINITY;
        int hit = -1;
        bool bad = false;   // (beyond far_o: the walk failed -- left the cells, ran on, or missed)
        if (tn <= tf) {
            int i[3];
            float nx[3], dt[3];
            for (int x = 0; x < 3; ++x) {
                const int c = (int)std::fmin(std::fmax((std::fmaf(tn, df[x], of[x]) - hd.lo[x]) * hd.inv_cs[x], 0.f),
                                             (float)(hd.res[x] - 1));
                const float plane = std::fmaf((float)(df[x] > 0 ? c + 1 : c), hd.cs[x], hd.lo[x]);
                nx[x] = df[x] != 0 ? std::fmaf(plane, inv[x], -oi[x]) : INF;
                dt[x] = hd.cs[x] * std::fabs(inv[x]);
                i[x] = c;
            }
            if (flat) nx[1] = INF;   // (never the nearest plane: no y step)
            int ci = (i[2] * hd.res[1] + i[1]) * hd.res[0] + i[0];
            const int st[3] = {df[0] > 0 ? 1 : -1, df[1] > 0 ? hd.res[0] : -hd.res[0],
                               df[2] > 0 ? hd.res[0] * hd.res[1] : -hd.res[0] * hd.res[1]};
            uint32_t w = cells[ci];
            uint32_t cur = first_of(w), end = end_of(w);
            int steps = 0;
            for (;;) {
                if (steps > (far_o ? 1 << 16 : max_steps)) {
                    if (far_o) bad = true;
                    else check(false, "a walk within far_o takes at most max_steps steps");
                    break;
                }
                if (cur >= end) {
                    const float te = std::fmin(std::fmin(nx[0], nx[1]), nx[2]);
                    if (!(te < (float)tmax && te < tf)) break;
                    // (flat: x where nx <= nz, as the kernel's compare-and-select)
                    const int a = flat ? (nx[0] <= nx[2] ? 0 : 2) : nx[0] == te ? 0 : (nx[1] == te ? 1 : 2);
                    ci += st[a];
                    nx[a] += dt[a];
                    ++steps;
                    // (no range check in the kernel: within far_o the walk's index stays within
                    // the pad layers, which this mirror asserts)
                    const bool inside = ci >= -(int)pad && ci < (int)(hd.n_cells + pad);
                    if (!inside) {
                        if (far_o) bad = true;
                        else check(false, "a step out of the grid stays within the pad layers");
                        break;
                    }
                    w = cells[ci];
                    cur = first_of(w);
                    end = end_of(w);
                }
                if (cur < end) {
                    const uint32_t id = ids[cur];
                    const double t = sphere_t(sf[id], o, d, tm);
                    if (t < tmax) tmax = t, hit = (int)id;
                    ++cur;
                }
            }
            ++(far_o ? beyond : flat ? walked_flat : walked);
        }
        if (far_o) {
            if (!flat) beyond_bad += bad || (hit != best_id && !(best == tmax));
            continue;
        }
        if (hit != best_id && !(best == tmax)) {
            ++misses;
            if (std::getenv("RT_SAN_VERBOSE"))
                std::printf("miss flat %d far %d cells %.3g |o| %.4g far_o %.4g best %d %.9g got %d %.9g tn %g tf %g\n",
                            flat, (int)far, dist_cells,
                            std::fmax(std::fmax(std::fabs(o[0]), std::fabs(o[1])), std::fabs(o[2])), (double)hd.far_o,
                            best_id, best, hit, tmax, (double)tn, (double)tf);
        }
        }
    }
    check(misses == 0, "grid walk reaches every brute-force closest hit");
    return 1;
}

bool build_ok(const std::vector<rt_sphere>& S, int leaf, double ct, double ci, int front) {
    BuiltBvh b;
    std::string err;
    BvhParams p;
    p.max_leaf = leaf;
    p.cost_traverse = ct;
    p.cost_intersect = ci;
    p.front = front;
    if (!build_bvh(S.data(), (int)S.size(), p, b, err)) return false;
    std::vector<int> seen(S.size(), 0);
    for (int k : b.order) seen[k]++;
    for (int k : b.big) seen[k]++;
    for (size_t k = 0; k < S.size(); ++k) check(seen[k] == 1, "sphere placed exactly once");
    // the grid over the tree's spheres in their LDS order (as rt_upload_scene builds it)
    std::vector<SphereF> sf;
    for (int k : b.order) {
        SphereF r{};
        for (int x = 0; x < 3; ++x) {
            r.c[x] = (float)S[k].center[x];
            r.cv[x] = S[k].moving ? (float)S[k].center_vec[x] : 0.f;
        }
        r.r = (float)S[k].radius;
        sf.push_back(r);
    }
    std::mt19937 g(1234u + (unsigned)leaf);
    for (double density : {0.5, 2.0, 8.0})
        for (int slabs : {1, 16}) grids_built += check_grid(sf, b.front, density, slabs, g, 2000);
    return true;
}

int cmd_spheres(const char* path) {
    const std::string raw = read_file(path);
    std::vector<rt_sphere> S(raw.size() / sizeof(rt_sphere));
    std::memcpy(S.data(), raw.data(), S.size() * sizeof(rt_sphere));
    int built = 0;
    for (int leaf : {1, 2, 6, 16})
        for (int front : {-1, 0, 3}) built += build_ok(S, leaf, 1.0, 0.25, front);
    // adversarial variants: coincident centres, one huge / NaN / inf coordinate
    std::vector<rt_sphere> A = S;
    for (auto& s : A) {
        s.center[0] = s.center[1] = s.center[2] = 1.0;
        s.moving = 0;
    }
    built += build_ok(A, 2, 1.0, 0.25, 0);
    const double bad[] = {1e300, -1e31, NAN, INFINITY};
    int refused = 0;
    for (double x : bad) {
        A = S;
        A[7].center[1] = x;
        refused += !build_ok(A, 6, 1.0, 0.25, -1);
        A = S;
        A[9].center_vec[2] = x;
        refused += !build_ok(A, 6, 1.0, 0.25, -1);
    }
    check(refused == 8, "out-of-range sphere coordinates refused");
    {
        // two far-apart clusters: most cells of a grid over both would be empty -- refused
        std::vector<SphereF> cl;
        for (size_t k = 0; k < S.size(); ++k) {
            if (S[k].radius >= 0.5) continue;
            SphereF r{};
            for (int x = 0; x < 3; ++x) r.c[x] = (float)S[k].center[x];
            if (k % 2) r.c[0] += 500.f;
            r.r = (float)S[k].radius;
            cl.push_back(r);
        }
        GridHdr hd;
        std::vector<unsigned char> buf;
        check(!build_sphere_grid(cl.data(), 0, (int)cl.size(), 2.0, 16, (int)sizeof(SphereF), hd, buf) && buf.empty(),
              "clustered spheres get no grid");
    }
    // the oracle on the same spheres (restated as orc_sphere): counter mode on a few
    // pixels, then the reference's main.cpp in mt mode at a small width
    std::vector<orc_sphere> os(S.size());
    std::vector<orc_material> om(S.size());
    orc_rng r;
    orc_rng_init_mt(&r);
    const int n = orc_scene_random(&r, os.data(), om.data(), (int)os.size());
    orc_camera cam;
    orc_camera_defaults(&cam);
    cam.image_width = 64;
    cam.samples_per_pixel = 2;
    orc_camera_initialize(&cam);
    const int32_t pix[] = {0, 0, 31, 17, 63, 35, 10, 20};
    double sums[12];
    int32_t rgb[12];
    uint64_t segs[4];
    orc_render_counter(os.data(), om.data(), n, &cam, 0x5EED, pix, 4, sums, rgb, segs);
    std::vector<int32_t> img(100 * 56 * 3);
    const int H = orc_reference_main(100, 1, img.data());
    std::printf("spheres %zu builds %d refused %d oracle n %d H %d px %d %d %d grids %d walked %lld walked_flat %lld "
                "beyond %lld beyond_bad %lld\n", S.size(), built, refused, n, H, rgb[0], rgb[1], rgb[2], grids_built, walked,
                walked_flat, beyond, beyond_bad);
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: san_driver obj FILE... | fuzz SEED ITERS FILE... | spheres FILE\n");
        return 2;
    }
    const std::string cmd = argv[1];
    int rc = 0;
    if (cmd == "obj") {
        for (int k = 2; k < argc; ++k) {
            std::printf("%s ", argv[k]);
            load_and_build(argv[k], true);
        }
    } else if (cmd == "fuzz" && argc >= 5) {
        rc = cmd_fuzz((unsigned)std::strtoul(argv[2], nullptr, 0), std::atoi(argv[3]), argc - 4, argv + 4);
    } else if (cmd == "spheres" && argc == 3) {
        rc = cmd_spheres(argv[2]);
    } else {
        return 2;
    }
    std::printf("checks failed %d\n", fail_count);
    return rc ? rc : (fail_count ? 1 : 0);
}

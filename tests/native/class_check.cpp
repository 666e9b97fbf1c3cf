// class_check: rta::classify_class (the class alone, rt_animate's per-frame check)
// equals rta::classify's class on random triangles, on triangles placed at both
// of classify's square-root thresholds (stored-plane steepness kMinCos, normal
// length 1e-6 / 1e6) to a relative 1e-12, and on degenerate and non-finite
// records; then times both over 640 triangles. Exits non-zero on any mismatch.
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <random>
#include <vector>

#include "../../opengl-ray-tracer_amd/csrc/accel_bound.h"

using namespace rta;

static FlatShape tri(const double a[3], const double b[3], const double c[3], const double n[3], double d) {
    FlatShape s;
    std::memset(&s, 0, sizeof s);
    s.type = RT_TRIANGLE;
    s.triP1 = {float(a[0]), float(a[1]), float(a[2])};
    s.triP2 = {float(b[0]), float(b[1]), float(b[2])};
    s.triP3 = {float(c[0]), float(c[1]), float(c[2])};
    s.planeNormal = {float(n[0]), float(n[1]), float(n[2])};
    s.planeD = float(d);
    return s;
}

int main() {
    std::mt19937_64 g(20251017);
    std::uniform_real_distribution<double> u(-1, 1);
    long bad = 0, total = 0, bounded = 0;
    auto check = [&](const FlatShape& s) {
        Box3 b;
        const int want = classify(s, b, 5500.0), got = classify_class(s, 5500.0);
        ++total;
        bounded += want == BOUNDED;
        if (want != got) {
            if (bad < 5) std::printf("MISMATCH classify %d classify_class %d\n", want, got);
            ++bad;
        }
    };
    const double o[3] = {0, 0, 0};
    for (int it = 0; it < 400000; ++it) {
        double a[3], b[3], c[3], n[3];
        for (int k = 0; k < 3; ++k) {
            a[k] = u(g) * 10;
            b[k] = a[k] + u(g);
            c[k] = a[k] + u(g);
            n[k] = u(g);
        }
        const int mode = it % 4;
        if (mode == 1) {  // the stored normal at the kMinCos steepness threshold (to 1e-12 relative)
            const double e1[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]}, e2[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
            double cr[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
            const double cl = std::sqrt(cr[0] * cr[0] + cr[1] * cr[1] + cr[2] * cr[2]);
            double t[3] = {n[1] * cr[2] - n[2] * cr[1], n[2] * cr[0] - n[0] * cr[2], n[0] * cr[1] - n[1] * cr[0]};
            const double tl = std::sqrt(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]);
            const double cs = 0.05 * (1 + 1e-7 * u(g));  // cos to the vertices' plane
            const double sn = std::sqrt(1 - cs * cs);
            for (int k = 0; k < 3; ++k) n[k] = cs * cr[k] / cl + sn * t[k] / tl;
        } else if (mode == 2) {  // normal length at 1e-6 or 1e6
            const double l = (it & 8 ? 1e-6 : 1e6) * (1 + 1e-9 * u(g)), nl = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
            for (int k = 0; k < 3; ++k) n[k] *= l / nl;
        } else if (mode == 3) {  // thin and degenerate triangles
            for (int k = 0; k < 3; ++k) c[k] = a[k] + (b[k] - a[k]) * 0.5 + 1e-3 * u(g) * (it & 16 ? 1 : 0);
        }
        check(tri(a, b, c, n, u(g)));
    }
    const double inf = std::numeric_limits<double>::infinity(), nan = std::numeric_limits<double>::quiet_NaN();
    const double p[3] = {1, 2, 3}, q[3] = {2, 2, 3}, r[3] = {1, 3, 3}, nz[3] = {0, 0, 1}, z[3] = {0, 0, 0};
    const double pi[3] = {inf, 0, 0}, pn[3] = {nan, 0, 0};
    check(tri(p, q, r, nz, -3));
    check(tri(p, p, r, nz, -3));
    check(tri(pi, q, r, nz, 0));
    check(tri(pn, q, r, nz, 0));
    check(tri(p, q, r, z, 0));
    check(tri(p, q, r, nz, inf));
    (void)o;
    // cost over 640 triangles (the car's wheels)
    std::vector<FlatShape> v;
    for (int i = 0; i < 640; ++i) {
        double a[3], b[3], c[3], n[3] = {0, 0, 1};
        for (int k = 0; k < 3; ++k) {
            a[k] = u(g);
            b[k] = a[k] + u(g);
            c[k] = a[k] + u(g);
        }
        v.push_back(tri(a, b, c, n, 0));
    }
    volatile int sink = 0;
    auto time = [&](bool fast) {
        const auto t0 = std::chrono::steady_clock::now();
        for (int it = 0; it < 200; ++it)
            for (const FlatShape& s : v) {
                Box3 b;
                sink += fast ? classify_class(s, 5500.0) : classify(s, b, 5500.0);
            }
        return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / 200;
    };
    const double slow_us = time(false), fast_us = time(true);
    std::printf("%s: %ld records, %ld bounded, %ld mismatches; 640 triangles: classify %.1f us, classify_class %.1f us\n",
                bad ? "class_check FAILED" : "class_check ok", total, bounded, bad, slow_us, fast_us);
    return bad ? 1 : 0;
}

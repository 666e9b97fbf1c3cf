// accel_bound.h — the accelerator's conservative shape bounds, shared by the
// host builder (accel.cpp) and the device refit (rt_kernels.hip, rt_refit), so
// that a box grown on the device is the box the host would have built.
//
// classify() decides whether the reference test can return an INNER hit of a
// shape only inside a finite box, and gives that box: every point the test can
// report as a hit, for ray origins up to origin_lim, lies inside it.
//
// Relative padding: the float error of every quantity the reference test
// computes is ~1e-7 of the coordinates' magnitude (1e-3 of it for the
// barycentric solve on the thinnest triangle admitted); 1e-3 of (size +
// magnitude) covers them with room, for ray origins up to origin_lim.
//
// A plane-based hit point computed from a ray with origin o lies within
// ~4u(|D| + |o|) of the plane (u = 2^-24) and its projection inside the shape,
// wherever the rounding puts it along a grazing ray, so those bounds hold for
// any such origin. The sphere root does not: D = bb^2 - 4*aa*cc cancels, and
// the computed point lies within sqrt(r^2 + k*L^2) of the centre, L = |o - c|
// (measured: k <= 4.4e-7, from L = 10 to 1e4). Spheres get that extra margin
// with kSphereErr = 4e-6 and the largest L an accelerated origin can have.
//
// Origin-relative error: the padded slab test (accel_math.h) errs by about
// u*|o| in space, and a plane-based hit point by about 4u*|o|; for a small
// shape far from the largest origin that exceeds the size-relative padding, so
// every box also gets kOriginErr * origin_lim (~8x the ~5e-7 * origin_lim of
// both errors together, for |o| up to sqrt(3) * origin_lim).
#pragma once

#include <math.h>

#include "../../include/rt_flat.h"
#include "accel_math.h"  // RTA_HD

namespace rta {

struct Box3 {
    float lo[3], hi[3];
};

constexpr double kPadRel = 1e-3;
constexpr double kMinSin2 = 1e-3;    // thinnest triangle bounded (sin^2 of its corner angle)
constexpr double kMinCos = 0.05;     // steepest stored plane bounded (cos to the vertices' plane)
constexpr double kCosRef = 0.5;      // below it the padding scales with 1/cos
constexpr double kSphereErr = 4e-6;  // k of the sphere-root error above, with room
constexpr double kOriginRel = 4.0;   // origin_lim = kOriginRel * (scene magnitude + 1)
constexpr double kOriginErr = 4e-6;  // padding per unit of origin_lim (origin-relative error above)
// Origin bound of an MT accelerator (in place of kOriginRel): rays from farther
// take the always-enter mode and a camera beyond it renders the frame on k_packet.
#ifndef RTA_MT_ORIGIN_REL
#define RTA_MT_ORIGIN_REL 3.0
#endif
constexpr double kOriginRelMt = RTA_MT_ORIGIN_REL;
constexpr double kU = 5.9604644775390625e-08;  // 2^-24

enum { UNBOUNDED = 0, BOUNDED = 1, NEVER = 2 };

struct D3 {
    double x, y, z;
};
RTA_HD D3 d3(rt_vec3 v) { return D3{v.x, v.y, v.z}; }
RTA_HD D3 operator+(D3 a, D3 b) { return D3{a.x + b.x, a.y + b.y, a.z + b.z}; }
RTA_HD D3 operator-(D3 a, D3 b) { return D3{a.x - b.x, a.y - b.y, a.z - b.z}; }
RTA_HD D3 operator*(D3 a, double s) { return D3{a.x * s, a.y * s, a.z * s}; }
RTA_HD double dot(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
RTA_HD D3 cross(D3 a, D3 b) { return D3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
RTA_HD bool finite3(D3 a) { return isfinite(a.x) && isfinite(a.y) && isfinite(a.z); }
RTA_HD double maxabs(D3 a) { return fmax(fmax(fabs(a.x), fabs(a.y)), fabs(a.z)); }

// float normalize exactly as the kernels do it (only used to rebuild the
// wall basis; the box is then padded, so bit-exactness is not required).
RTA_HD void fnormalize(float v[3]) {
    float s = 1.0f / sqrtf(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    v[0] *= s;
    v[1] *= s;
    v[2] *= s;
}

struct BoxAcc {
    double lo[3], hi[3];
    RTA_HD BoxAcc() {
        for (int i = 0; i < 3; ++i) {
            lo[i] = INFINITY;
            hi[i] = -INFINITY;
        }
    }
    RTA_HD void add(D3 p) {
        const double v[3] = {p.x, p.y, p.z};
        for (int i = 0; i < 3; ++i) {
            lo[i] = fmin(lo[i], v[i]);
            hi[i] = fmax(hi[i], v[i]);
        }
    }
    RTA_HD Box3 padded(double pad) const {
        Box3 b;
        for (int i = 0; i < 3; ++i) {
            // round outwards after padding
            b.lo[i] = nextafterf(static_cast<float>(lo[i] - pad), -INFINITY);
            b.hi[i] = nextafterf(static_cast<float>(hi[i] + pad), INFINITY);
        }
        return b;
    }
    RTA_HD double extent() const { return fmax(fmax(hi[0] - lo[0], hi[1] - lo[1]), hi[2] - lo[2]); }
    RTA_HD double mag() const {
        double m = 0;
        for (int i = 0; i < 3; ++i) m = fmax(m, fmax(fabs(lo[i]), fabs(hi[i])));
        return m;
    }
};

// `amp`: error amplification of the shape's hit point (>= 1; the lift of a
// triangle onto a steep stored plane divides its errors by the cosine).
RTA_HD Box3 finish(const BoxAcc& acc, double origin_lim, double amp = 1.0) {
    return acc.padded(amp * (kPadRel * (acc.extent() + acc.mag() + 1.0) + kOriginErr * origin_lim) + 1e-6);
}

// Moller-Trumbore (gpu_shader.comp:170-195) accepts a hit when
// |a| = |e1 . (d x e2)| >= 1e-5, an absolute threshold, and reports o + t d with
// t, u, v each computed through f = 1/a, so on grazing rays from afar the hit
// can stray far from the triangle (tests/test_accel_cpu.py). The accelerator
// bounds the stray per ray (AccelHost::lmt, accel_math.h mt_pad). First-order
// float error bounds of the dot and cross products (u = 2^-24; |da| <= 7u D X,
// eu <= (9u D S E2 + 1.5 * 7u D X) / A, ev likewise with E1; the round-2 form of
// this bound took the worst origin and |cos| >= 0.03 and forced entry below):
// with D = |d|, S >= |o - p1|, X = |e1||e2|, c = |cos(d, n)| and
// A = max(1e-5, D c |e1 x e2|) - 7u D X the smallest |a| an accepted hit can
// have (|a| = D c |e1 x e2| exactly, the computed one is >= 1e-5 and within
// 7u D X of it),
//   X* = p1 + u* e1 + v* e2 lies within Q = eu E1 + ev E2
//      = u D X (18 S + 10.5 (E1 + E2)) / A of the triangle, and
//   the computed t is within r |t*| + dl of t*, r = 7.07 u D X / A + 3u,
//      dl = 9.09 u X S / A (the 2u T part is below the static box padding).
// For r < 1/2, an accepted hit at t > 0 with distance below l therefore
// implies that the ray enters the triangle's box padded by
// P = Q + D dl / (1 - r) before parameter l / (|d| (1 - r)): X* is inside the
// box padded by Q, and the ray point D dl / (1 - r) before X* (or the origin,
// when t* is smaller) is then inside the box padded by P. mt_pad takes P
// twice (safety 2) and, per local node, the worst triangle below it: the
// smallest |e1 x e2| and cosine (the grazing cone), the largest X, E1 + E2 and
// |p1 - Z|, with S = |o - Z| + |p1 - Z|. No |cos| threshold, no origin bound beyond
// the static box's: a ray grazing a node's cone gets the 1e-5 floor's pad, and
// only a node whose floor is below 2.5e-6 (triangles with X > ~6) is entered
// whatever its box says.
struct MtTri {
    double cr, X, esum, p1[3];
};

// The static box of a triangle under per-ray MT padding: the triangle's own
// box with the size/origin padding of `finish`, and its MtTri constants.
RTA_HD int classify_mt_tight(const FlatShape& s, Box3& out, double origin_lim, MtTri& m) {
    const float e1f[3] = {s.triP2.x - s.triP1.x, s.triP2.y - s.triP1.y, s.triP2.z - s.triP1.z};
    const float e2f[3] = {s.triP3.x - s.triP1.x, s.triP3.y - s.triP1.y, s.triP3.z - s.triP1.z};
    const D3 p1 = d3(s.triP1), e1{e1f[0], e1f[1], e1f[2]}, e2{e2f[0], e2f[1], e2f[2]};
    if (!finite3(p1) || !finite3(e1) || !finite3(e2)) return UNBOUNDED;
    const double E1 = sqrt(dot(e1, e1)), E2 = sqrt(dot(e2, e2)), cr = sqrt(dot(cross(e1, e2), cross(e1, e2)));
    if (!(cr > 0) || !isfinite(cr) || !(E1 * E2 < 1e30)) return UNBOUNDED;
    m.cr = cr;
    m.X = E1 * E2;
    m.esum = E1 + E2;
    m.p1[0] = p1.x;
    m.p1[1] = p1.y;
    m.p1[2] = p1.z;
    BoxAcc acc;
    acc.add(p1);
    acc.add(p1 + e1);
    acc.add(p1 + e2);
    out = finish(acc, origin_lim);
    return BOUNDED;
}

// UNBOUNDED: no finite bound; BOUNDED: `out` is set; NEVER: the reference test
// never returns INNER. origin_lim: largest |coordinate| of a ray origin the
// bound must hold for (0 for the build's first pass, which only measures the
// scene's magnitude). mt: triangles take the Moller-Trumbore test
// (classify_mt_tight, the static part of their bound; the other shapes' tests
// do not depend on it).
RTA_HD int classify(const FlatShape& s, Box3& out, double origin_lim, bool mt = false) {
    if (mt && s.type == RT_TRIANGLE) {
        MtTri m;
        return classify_mt_tight(s, out, origin_lim, m);
    }
    BoxAcc acc;
    switch (s.type) {
        case RT_SPHERE: {
            D3 c = d3(s.sphereCenter);
            double r = fabs(static_cast<double>(s.sphereRadius));
            if (!finite3(c) || !isfinite(r)) return UNBOUNDED;
            const double L = sqrt(3.0) * origin_lim + sqrt(dot(c, c));
            const double R = sqrt(r * r + kSphereErr * L * L);
            acc.add(c - D3{R, R, R});
            acc.add(c + D3{R, R, R});
            out = finish(acc, origin_lim);
            return BOUNDED;
        }
        case RT_WALL: {
            float n[3] = {s.planeNormal.x, s.planeNormal.y, s.planeNormal.z};
            // the intersection basis of gpu_shader.comp:305-307
            float u[3] = {n[1] * 0.f - 1.f * n[2], n[2] * 0.f - 0.f * n[0], n[0] * 1.f - 0.f * n[1]};
            fnormalize(u);
            if (sqrtf(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]) < 1e-5f) {  // NaN stays NaN (:306)
                u[0] = n[1] * 0.f - 0.f * n[2];
                u[1] = n[2] * 1.f - 0.f * n[0];
                u[2] = n[0] * 0.f - 1.f * n[1];
                fnormalize(u);
            }
            D3 N{n[0], n[1], n[2]}, U{u[0], u[1], u[2]};
            D3 V = cross(N, U);
            double vl = sqrt(dot(V, V));
            if (!finite3(U) || !(vl > 0) || !isfinite(vl)) return UNBOUNDED;  // ±Y: NaN basis, never rejected
            V = V * (1.0 / vl);
            D3 st = d3(s.wallStart);
            double nn = dot(N, N), W = s.wallWidth, H = s.wallHeight, D = s.planeD;
            if (!finite3(st) || !(nn > 0) || !isfinite(W) || !isfinite(H) || !isfinite(D)) return UNBOUNDED;
            D3 c0 = st - N * ((dot(N, st) + D) / nn);  // start projected on the stored plane
            acc.add(c0);
            acc.add(c0 + U * W);
            acc.add(c0 + V * H);
            acc.add(c0 + U * W + V * H);
            out = finish(acc, origin_lim);
            return BOUNDED;
        }
        case RT_TRIANGLE: {
            // gpu_shader.comp:196-240: the hit point p lies on the STORED plane
            // (N, D); the barycentric solve then projects p orthogonally onto
            // the vertices' own plane. So the INNER points are the stored-plane
            // points whose projection falls inside the triangle: the triangle
            // lifted along its own normal nt onto the stored plane. The stored
            // plane need not pass through the vertices (updateWheelAnimations,
            // src/main.cpp:1084-1109, moves vertices and keeps the old plane);
            // it must only not be nearly perpendicular to them (|cos| >=
            // kMinCos); below kCosRef the padding grows as 1/|cos|, the float
            // error of the lift.
            D3 p1 = d3(s.triP1), p2 = d3(s.triP2), p3 = d3(s.triP3), N = d3(s.planeNormal);
            double D = s.planeD;
            if (!finite3(p1) || !finite3(p2) || !finite3(p3) || !finite3(N) || !isfinite(D)) return UNBOUNDED;
            D3 e1 = p2 - p1, e2 = p3 - p1, cr = cross(e1, e2);
            double d00 = dot(e1, e1), d11 = dot(e2, e2), c2 = dot(cr, cr);
            if (!(d00 > 0) || !(d11 > 0) || !(c2 >= kMinSin2 * d00 * d11)) return UNBOUNDED;  // thin: error unbounded
            D3 nt = cr * (1.0 / sqrt(c2));
            double nl = sqrt(dot(N, N)), cn = dot(N, nt);
            if (!(nl > 1e-6 && nl < 1e6) || !(fabs(cn) >= kMinCos * nl)) return UNBOUNDED;
            const D3 q[3] = {p1, p2, p3};
            for (int i = 0; i < 3; ++i) {
                const double h = -(dot(N, q[i]) + D) / cn;  // q + h*nt lies on the stored plane
                if (!isfinite(h)) return UNBOUNDED;
                acc.add(q[i] + nt * h);
            }
            out = finish(acc, origin_lim, fmax(1.0, kCosRef * nl / fabs(cn)));
            return BOUNDED;
        }
        case RT_PLANE:
            return UNBOUNDED;
        default:
            return NEVER;  // get_intersection has no branch for it (gpu_shader.comp:246-325)
    }
}

// classify's class alone, without the box: what rt_animate needs per moved shape
// and frame to decide whether the accelerator must be rebuilt. Triangles (the
// animated bulk) take the same double operations as classify up to the squared
// forms of its two square-root tests, decided outright unless a value lies
// within a relative 1e-9 of its threshold (the double rounding of either form is
// ~1e-15); those, and the other shape types, run classify itself. So the class
// is classify's whatever the input (tests/native/class_check.cpp), at a tenth of
// its cost: no square roots, no divisions, no box or outward rounding (640 wheel
// triangles: 113 -> ~10 us on the host).
RTA_HD int classify_class(const FlatShape& s, double origin_lim) {
    if (s.type == RT_TRIANGLE) {
        const D3 p1 = d3(s.triP1), p2 = d3(s.triP2), p3 = d3(s.triP3), N = d3(s.planeNormal);
        const double D = s.planeD;
        if (!finite3(p1) || !finite3(p2) || !finite3(p3) || !finite3(N) || !isfinite(D)) return UNBOUNDED;
        const D3 e1 = p2 - p1, e2 = p3 - p1, cr = cross(e1, e2);
        const double d00 = dot(e1, e1), d11 = dot(e2, e2), c2 = dot(cr, cr);
        if (!(d00 > 0) || !(d11 > 0) || !(c2 >= kMinSin2 * d00 * d11)) return UNBOUNDED;  // as classify
        constexpr double m = 1e-9;
        const double nn = dot(N, N);  // classify: 1e-6 < sqrt(nn) < 1e6
        const bool n_lo = nn > 1e-12 * (1 + m), n_hi = nn < 1e12 * (1 - m);
        const bool n_out = nn < 1e-12 * (1 - m) || nn > 1e12 * (1 + m);
        // classify: |N . cr / sqrt(c2)| >= kMinCos sqrt(nn), i.e. (N . cr)^2 >= kMinCos^2 nn c2
        const double dn = dot(N, cr), lhs = dn * dn, rhs = kMinCos * kMinCos * nn * c2;
        if (n_out) return UNBOUNDED;
        if (n_lo && n_hi && isfinite(lhs) && isfinite(rhs) && rhs > 0) {
            if (lhs >= rhs * (1 + m)) return BOUNDED;  // h = -(N.q + D) / cn is then finite: |cn| >= 5e-8
            if (lhs <= rhs * (1 - m)) return UNBOUNDED;
        }
    }
    Box3 b;
    return classify(s, b, origin_lim);
}

}  // namespace rta

// accel_math.h — the accelerator's conservative ray tests, shared by the
// device walk (rt_kernels.hip) and the CPU emulation that checks it
// (tests/native/accel_check.cpp), so both run the same float operations.
//
// None of these tests decides a result. They only skip work that provably
// cannot change it (accel.h): local boxes are padded by at least
// 1e-3*(extent + scene magnitude + 1) + 1e-6 around every INNER hit point,
// the distance limit carries a 0.2 % margin, and the cone thresholds carry
// 2 mrad. The float error of the fused forms below is orders of magnitude
// smaller than those margins for every ray they are used on:
//   * slab: t = fma(lo, inv, -o*inv). Its error is about 6e-8*|o| in space,
//     below the kOriginErr*origin_lim part of every box's padding
//     (accel_bound.h) when |o| <= origin_lim (AccelHost).
//   * |inv| is clamped to kInvCap. A hit at parameter t on a clamped axis
//     then still lies inside the slab, because pad*kInvCap >= 1e17 > 2t for
//     unit-length directions (0.5 <= |d| <= 2) and such origins.
// Rays outside those bounds (origins on far-away plane hits, or odd
// direction lengths) get inv = 0, o*inv = 0, which makes every padded box
// pass: exact, only slower.
#pragma once

#include <cmath>

#if defined(__HIP__)
#include <hip/hip_runtime.h>
#define RTA_HD __host__ __device__ __forceinline__
#else
#define RTA_HD inline
#endif

namespace rta {

constexpr float kInvCap = 1e20f;     // |1/d| clamp of the padded slab test
constexpr float kConeEps = 1e-5f;    // rounding allowance of the cone test (the margin is 2e-3 rad)
constexpr double kConeMargin = 2e-3;  // radians beyond float error of N.d and of the cone test (build_cones)
constexpr float kPruneRel = 1.002f;  // distance margin for skipping a box

struct RayC {
    float ix, iy, iz;  // clamped 1/d (0 in the always-enter mode)
    float ox, oy, oz;  // o * inv
    float dx, dy, dz;  // d / |d|
    float rdl;         // 1 / |d|
    int dq;            // rint(127 d/|d|) as 3 signed bytes, byte 3 = -128 (cone_culls_q)
    // Moller-Trumbore walks only (mt_ray; dead, so free, in the other instances)
    float mox, moy, moz;  // the origin
    float so, on;         // |o - Z| rounded up (mt_origin_dist), |o|_1
    float dlen;           // |d| rounded up
};

// Quantized back-face cones (the barycentric accelerator's wide nodes,
// rt_kernels.hip wide_kids): one 32-bit word per child, bytes 0-2 the axis as
// a_q = rint(127 a) (signed), byte 3 a threshold t8. With the ray's
// d_q = rint(127 d/|d|), the integer dot(a_q, d_q) equals 127^2 a.d up to
//   127 (|a| |d_q - 127 d/|d|| + |a_q - 127 a|) + |a_q - 127 a| |d_q - 127 d/|d||
//   <= 127 (1.0000001 * 0.5001 * sqrt(3) + 0.5 * sqrt(3)) + 0.751 < 221
// (0.5001 covers the float d/|d| and the product 127 d). The word culls when
// dot(a_q, d_q) < 128 t8, i.e. when one dot4 with d_q's byte 3 = -128 is
// negative; t8 = floor((127^2 thr - 222) / 128) makes that imply a.d < thr,
// the float cone's own condition (cone_culls without its rounding allowance).
// |dot(a_q, d_q)| <= 127.87^2 < 16384, so t8 = -128 never culls.
constexpr int kConeNp = static_cast<int>(0x80000000u);     // kNoPrune child: a_q = 0, t8 = -128
constexpr int kConeNever = static_cast<int>(0x81000000u);  // never culls: a_q = 0, t8 = -127

RTA_HD int sdot4(int a, int b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_sdot4(a, b, 0, false);
#else
    int s = 0;
    for (int i = 0; i < 4; ++i)
        s += static_cast<int>(static_cast<signed char>((a >> (8 * i)) & 0xff)) *
             static_cast<int>(static_cast<signed char>((b >> (8 * i)) & 0xff));
    return s;
#endif
}

RTA_HD bool cone_culls_q(int w, int dq) { return sdot4(w, dq) < 0; }

// The ray's d_q (RayC::dq). A NaN component gives 0 there: such a ray has no
// INNER hit (every shape test compares against N.d), so what it culls is moot.
RTA_HD int ray_dq(float dx, float dy, float dz) {
    auto b = [](float v) {
        const float r = std::rint(127.0f * v);
        return (r >= -127.0f && r <= 127.0f) ? static_cast<int>(r) & 0xff : 0;
    };
    return b(dx) | (b(dy) << 8) | (b(dz) << 16) | static_cast<int>(0x80000000u);
}

// The cone word of a float cone (axis, thr) as AccelHost holds it (the host's
// build, the device's refit).
RTA_HD int cone_word(float ax, float ay, float az, float thr) {
    if (thr <= -6.0f) return kConeNp;  // kNoPrune (accel.h)
    const double t = std::floor((16129.0 * static_cast<double>(thr) - 222.0) / 128.0);
    if (!(t > -128.0) || !std::isfinite(ax) || !std::isfinite(ay) || !std::isfinite(az)) return kConeNever;
    const double a[3] = {ax, ay, az};
    if (!(std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]) <= 1.0000001)) return kConeNever;  // the bound needs |a| ~ 1
    int w = 0;
    for (int i = 0; i < 3; ++i) w |= (static_cast<int>(std::nearbyint(127.0 * a[i])) & 0xff) << (8 * i);
    return w | ((static_cast<int>(t > 127.0 ? 127.0 : t) & 0xff) << 24);
}

RTA_HD float clamp_inv(float d) {
    return std::fabs(d) < 1.0f / kInvCap ? std::copysign(kInvCap, d) : 1.0f / d;
}

// origin_lim: AccelHost::origin_lim, the largest origin the padding is built for.
RTA_HD RayC ray_consts(float ox, float oy, float oz, float dx, float dy, float dz, float origin_lim) {
    const float dl = std::sqrt(dx * dx + dy * dy + dz * dz);
    const float om = std::fmax(std::fmax(std::fabs(ox), std::fabs(oy)), std::fabs(oz));
    const bool ok = om <= origin_lim && dl >= 0.5f && dl <= 2.0f;
    RayC c;
    c.ix = ok ? clamp_inv(dx) : 0.0f;
    c.iy = ok ? clamp_inv(dy) : 0.0f;
    c.iz = ok ? clamp_inv(dz) : 0.0f;
    c.ox = ok ? ox * c.ix : 0.0f;
    c.oy = ok ? oy * c.iy : 0.0f;
    c.oz = ok ? oz * c.iz : 0.0f;
    c.rdl = 1.0f / dl;
    c.dx = dx * c.rdl;
    c.dy = dy * c.rdl;
    c.dz = dz * c.rdl;
    c.dq = ray_dq(c.dx, c.dy, c.dz);
    return c;
}

// Distance limit l (best hit so far, or the light distance) as a ray parameter.
RTA_HD float t_limit(float l, float rdl) { return (l * kPruneRel + 1e-6f) * rdl; }

// Padded-box test: the ray's forward part meets the box at a parameter no
// larger than tl. te = entry parameter (>= 0), for ordering and pruning.
RTA_HD bool box_enter(const RayC& c, float lx, float ly, float lz, float hx, float hy, float hz, float tl,
                      float& te) {
    const float x0 = std::fma(lx, c.ix, -c.ox), x1 = std::fma(hx, c.ix, -c.ox);
    const float y0 = std::fma(ly, c.iy, -c.oy), y1 = std::fma(hy, c.iy, -c.oy);
    const float z0 = std::fma(lz, c.iz, -c.oz), z1 = std::fma(hz, c.iz, -c.oz);
    const float tn = std::fmax(std::fmax(std::fmin(x0, x1), std::fmin(y0, y1)), std::fmax(std::fmin(z0, z1), 0.0f));
    const float tf = std::fmin(std::fmin(std::fmax(x0, x1), std::fmax(y0, y1)), std::fmin(std::fmax(z0, z1), tl));
    te = tn;
    return tn <= tf;
}

// box_enter with the exit parameter too.
RTA_HD bool box_span(const RayC& c, float lx, float ly, float lz, float hx, float hy, float hz, float tl, float& tn,
                     float& tf) {
    const float x0 = std::fma(lx, c.ix, -c.ox), x1 = std::fma(hx, c.ix, -c.ox);
    const float y0 = std::fma(ly, c.iy, -c.oy), y1 = std::fma(hy, c.iy, -c.oy);
    const float z0 = std::fma(lz, c.iz, -c.oz), z1 = std::fma(hz, c.iz, -c.oz);
    tn = std::fmax(std::fmax(std::fmin(x0, x1), std::fmin(y0, y1)), std::fmax(std::fmin(z0, z1), 0.0f));
    tf = std::fmin(std::fmin(std::fmax(x0, x1), std::fmax(y0, y1)), std::fmin(std::fmax(z0, z1), tl));
    return tn <= tf;
}

// Back-face cone (accel.h, build_cones): no shape below can give an INNER hit
// (N.d > 0 is required) when dot(axis, d/|d|) < thr.
RTA_HD bool cone_culls(const RayC& c, float ax, float ay, float az, float thr) {
    return std::fma(ax, c.dx, std::fma(ay, c.dy, az * c.dz)) < thr - kConeEps;
}

constexpr float kU24 = 5.9604645e-08f;
// |o - Z| rounded up (AccelHost::mt_z), once per ray.
RTA_HD float mt_origin_dist(float ox, float oy, float oz, const float* z) {
    const float x = ox - z[0], y = oy - z[1], w = oz - z[2];
    return 1.0001f * std::sqrt(x * x + y * y + w * w) + 1e-6f;
}

// The Moller-Trumbore walk's origin terms of RayC.
RTA_HD void mt_ray(RayC& c, float ox, float oy, float oz, const float* z) {
    c.mox = ox;
    c.moy = oy;
    c.moz = oz;
    c.so = mt_origin_dist(ox, oy, oz, z);
    c.on = std::fabs(ox) + std::fabs(oy) + std::fabs(oz);
    c.dlen = 1.0001f / c.rdl;
}

// 1/x within 1 ulp (v_rcp_f32 on the device); every use below carries a
// relative margin of 1e-4 or more, so the rounding does not matter.
RTA_HD float rcp(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rcpf(x);
#else
    return 1.0f / x;
#endif
}

// Moller-Trumbore per-ray padding (the derivation above accel_bound.h MtTri).
// k: the node's grazing cone (axis, s = 2 sin(psi/2) + margin); m: its
// AccelHost::lmt constants {cr_min, u X_max, M_max, 18 M_max + 10.5 Esum_max,
// w, h0} (M = |p1 - Z|; w, h0: mt_slab); so: |o - Z| of the ray. Returns false when no finite bound holds (the walk
// enters at parameter 0); else `pad` to add to the node's static box on every
// side and `lf` (>= 1) to multiply the distance limit by.
constexpr int kMtPadF = 6;  // floats per local node in AccelHost::lmt
RTA_HD bool mt_pad(const RayC& c, float so, const float* k, const float* m, float& pad, float& lf, float& q2,
                   float& pt, float& ilf) {
    const float D = c.dlen;
    const float cn = std::fabs(std::fma(k[0], c.dx, std::fma(k[1], c.dy, k[2] * c.dz))) - k[3];
    const float A = std::fmax(1e-5f, D * std::fmax(cn, 0.0f) * m[0]) - 7.0f * D * m[1];
    if (!(A > 2.5e-6f)) return false;
    const float ia = 1.0001f * rcp(A);
    const float r = 7.07f * D * m[1] * ia + 3.0f * kU24;
    if (!(r < 0.5f)) return false;
    const float q = D * m[1] * std::fma(18.0f, so, m[3]) * ia;
    const float dl = 9.09f * m[1] * (so + m[2]) * ia;
    lf = 1.0001f * rcp(1.0f - r);
    // 1 / lf from below without a second reciprocal: (1 - r) / 1.0001 times 0.99999
    // (0.99989 * 1.0001 = 0.999990), against a rounding of rcp and the products of a few ulp
    ilf = (1.0f - r) * 0.99989f;
    q2 = 2.0f * q;
    pt = 2.0f * D * dl * lf;
    pad = q2 + pt;
    return pad < 1e30f;
}
RTA_HD bool mt_pad(const RayC& c, float so, const float* k, const float* m, float& pad, float& lf, float& q2,
                   float& pt) {
    float ilf;
    return mt_pad(c, so, k, m, pad, lf, q2, pt, ilf);
}

// The node's slab along its cone axis a: every triangle below lies within
// |a.x - w| <= h0 (m[4] = w, m[5] = h0), and its plane within angle theta of
// a's, 2 sin(theta/2) <= k[3]. X* (in T's plane, within Q of T) is then within
// h0 + Q k[3] of w along a (taken with 2Q, as the box takes it), and the ray point the box test stands for (within
// D dl lf of X* along the ray) within a further D dl lf |a.d/|d||. So the ray
// segment must meet that slab too: true when [t0, t1] (the box's interval)
// meets it. q2 = 2Q, pt = 2 D dl lf (mt_pad's two parts of pad); on >= |o|_1.
RTA_HD bool mt_slab(float ox, float oy, float oz, float on, const RayC& c, const float* k, const float* m,
                    float q2, float pt, float t0, float t1) {
    const float dn = std::fma(k[0], c.dx, std::fma(k[1], c.dy, k[2] * c.dz));
    const float s0 = std::fma(k[0], ox, std::fma(k[1], oy, std::fma(k[2], oz, -m[4])));
    const float hw = std::fma(q2, k[3], m[5]) + pt * std::fabs(dn) + 4.0f * kU24 * (on + std::fabs(m[4])) + 1e-6f;
    const float iv = c.rdl * rcp(dn);  // 1 / (a.d): +-inf when parallel
    const float ta = (-hw - s0) * iv, tb = (hw - s0) * iv;
    const float lo = std::fmax(t0, std::fmin(ta, tb)), hi = std::fmin(t1, std::fmax(ta, tb));
    return !(lo > hi + 1e-4f * std::fabs(hi) + 1e-6f);
}

}  // namespace rta

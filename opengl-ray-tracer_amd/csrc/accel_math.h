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
constexpr float kPruneRel = 1.002f;  // distance margin for skipping a box

struct RayC {
    float ix, iy, iz;  // clamped 1/d (0 in the always-enter mode)
    float ox, oy, oz;  // o * inv
    float dx, dy, dz;  // d / |d|
    float rdl;         // 1 / |d|
    int dq;            // rint(127 d/|d|) as 3 signed bytes, byte 3 = -128 (cone_culls_q)
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

// Host: the cone word of a float cone (axis, thr) as AccelHost holds it.
inline int cone_word(float ax, float ay, float az, float thr) {
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

// Back-face cone (accel.h, build_cones): no shape below can give an INNER hit
// (N.d > 0 is required) when dot(axis, d/|d|) < thr.
RTA_HD bool cone_culls(const RayC& c, float ax, float ay, float az, float thr) {
    return std::fma(ax, c.dx, std::fma(ay, c.dy, az * c.dz)) < thr - kConeEps;
}

}  // namespace rta

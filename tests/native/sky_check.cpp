// sky_check: rtg::sky_band (csrc/sky_rows.h) against the shader's own arithmetic.
// For random cameras (positions, targets, fov, aspect) and random root boxes, every
// pixel of every row outside the band gets a camera ray (getRay, gpu_shader.comp
// :155-168, in float as the kernels compute it) that misses the box under the GLSL
// slab test (:364-377, GLSL min/max). Also reports how many rows the band keeps.
// Exits non-zero on any violation.
#include <cmath>
#include <cstdio>
#include <random>

#include "../../opengl-ray-tracer_amd/csrc/sky_rows.h"

struct V3 {
    float x, y, z;
};
static V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static V3 mul(float s, V3 a) { return {s * a.x, s * a.y, s * a.z}; }
static float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static V3 norm(V3 a) { return mul(1.0f / std::sqrt(dot(a, a)), a); }
static V3 cross(V3 a, V3 b) { return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y}; }
static float gmin(float a, float b) { return (b < a) ? b : a; }
static float gmax(float a, float b) { return (a < b) ? b : a; }

static bool slab(V3 o, V3 d, const float lo[3], const float hi[3]) {
    const V3 inv{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    const float t0[3] = {(lo[0] - o.x) * inv.x, (lo[1] - o.y) * inv.y, (lo[2] - o.z) * inv.z};
    const float t1[3] = {(hi[0] - o.x) * inv.x, (hi[1] - o.y) * inv.y, (hi[2] - o.z) * inv.z};
    const float tmin = gmax(gmax(gmin(t0[0], t1[0]), gmin(t0[1], t1[1])), gmin(t0[2], t1[2]));
    const float tmax = gmin(gmin(gmax(t0[0], t1[0]), gmax(t0[1], t1[1])), gmax(t0[2], t1[2]));
    return tmax >= tmin && tmax > 0.0f;
}

int main() {
    std::mt19937 g(7);
    std::uniform_real_distribution<float> u(-1, 1);
    long bad = 0, cases = 0, rows_total = 0, rows_sky = 0;
    const int W = 320, H = 180;
    // 3000 cameras within 40 of the origin, 1500 at distances 1e3-1e5 looking at a
    // box near it or near themselves (getRay's rounding grows with |pos|), some with a
    // non-unit Front (the shader uses the uploaded vector as it is)
    for (int it = 0; it < 4500; ++it) {
        FlatCamera cam{};
        const bool far = it >= 3000;
        const float dist = far ? std::pow(10.0f, 3.0f + 2.0f * (u(g) + 1) / 2) : 40.0f;
        V3 pos{dist * u(g), dist * u(g), dist * u(g)}, tgt{5 * u(g), 5 * u(g), 5 * u(g)};
        if (far && it % 2) tgt = add(pos, V3{30 * u(g), 30 * u(g), 30 * u(g)});  // a box near the camera
        const float fs = far && it % 3 == 0 ? 0.5f + 2.5f * (u(g) + 1) / 2 : 1.0f;
        const V3 fu = norm(sub(tgt, pos)), r = norm(cross(fu, V3{0, 1, 0})), up = norm(cross(r, fu));
        const V3 f = mul(fs, fu);
        cam.Position = {pos.x, pos.y, pos.z};
        cam.Front = {f.x, f.y, f.z};
        cam.Right = {r.x, r.y, r.z};
        cam.Up = {up.x, up.y, up.z};
        cam.fov = 30 + 60 * (u(g) + 1) / 2;
        cam.aspectRatio = static_cast<float>(W) / H;
        float lo[3], hi[3];
        const V3 bc = far && it % 2 ? tgt : V3{10 * u(g), 10 * u(g), 10 * u(g)};
        const float cc[3] = {bc.x, bc.y, bc.z};
        for (int a = 0; a < 3; ++a) {
            const float e = 0.1f + 10 * (u(g) + 1);
            lo[a] = cc[a] - e;
            hi[a] = cc[a] + e;
        }
        if (it % 7 == 0) lo[1] = hi[1] = 25.0f;  // a flat floor (zero-thickness box)
        int y0, y1;
        if (!rtg::sky_band(cam, lo, hi, H, static_cast<float>(H), &y0, &y1)) continue;
        ++cases;
        const float hgt = 2.0f * std::tan((cam.fov / 2.0f) * 0.01745329251994329576923690768489f);
        const float wid = hgt * cam.aspectRatio;
        for (int y = 0; y < H; ++y) {
            ++rows_total;
            if (y >= y0 && y < y1) continue;
            ++rows_sky;
            for (int x = 0; x < W; ++x) {
                const float nx = 2.0f * static_cast<float>(x) / W - 1.0f, ny = 1.0f - 2.0f * static_cast<float>(y) / H;
                const V3 p = add(add(add(pos, f), mul(nx * wid / 2.0f, r)), mul(ny * hgt / 2.0f, up));
                if (slab(pos, norm(sub(p, pos)), lo, hi)) {
                    if (bad < 5) std::printf("VIOLATION case %d row %d x %d (band [%d, %d))\n", it, y, x, y0, y1);
                    ++bad;
                }
            }
        }
    }
    std::printf("%s: %ld cases, %ld of %ld rows outside the band, %ld violations\n",
                bad ? "sky_check FAILED" : "sky_check ok", cases, rows_sky, rows_total, bad);
    return bad ? 1 : 0;
}

// sky_rows.h — which image rows can only be background (host; rt_group.hip, tests).
//
// gpu_shader.comp:440-458: a camera ray that misses the root node's box hits
// nothing and the pixel is the background gradient of its row (:436), exactly
// (acc = 0 + 1 * bg). getRay (:155-168) puts the rays of image row y in one plane
// through the camera position: P = pos + front + ndcX w/2 right + ndcY h/2 up, so
// every direction of the row lies in the plane spanned by (front + ndcY h/2 up)
// and right, whose normal is n(ndcY) = right x front + ndcY h/2 (right x up). If
// all 8 corners of the root box lie strictly on one side of that plane, no ray of
// the row can enter the box. The side test takes an angular margin so that the
// conclusion holds for the float rays too: getRay forms P = pos + front + ... in
// float and subtracts pos again, so a ray's direction is off the exact plane by up
// to ~u (|pos| + |front| + w/2 |right| + h/2 |up|) / |P - pos| (u = 2^-24), which
// grows with the camera's distance from the origin; the margin is 1e-4 rad plus 32
// times that bound, with |P - pos| >= |front| for the orthogonal camera frames
// updateCameraVectors makes (others get no band). The slab test's own rounding is
// ~2u of the corner directions, inside the 1e-4. n is linear in ndcY and the rows that meet a box form one band
// (the planes turn about the axis through pos along `right`), so the scan stops at
// the first row from the top and from the bottom that may meet it.
//
// rt_group uses it to keep sky rows off the links: a peer sends only its rows
// inside the band and rank 0 writes the background for the others
// (rt_group_dispatch, k_unstripe). Every rank computes the same band from the same
// camera and box with the same double operations.
#ifndef RT_SKY_ROWS_H
#define RT_SKY_ROWS_H

#include <cmath>

#include "../../include/rt_flat.h"

namespace rtg {

// Rows [*y_lo, *y_hi) may meet the box [lo, hi]; every other row of the
// width x height frame (resY as in the shader) can only be background. Returns
// false (and the whole frame) when the inputs are not finite, the box is empty,
// or the planes degenerate.
inline bool sky_band(const FlatCamera& cam, const float lo[3], const float hi[3], int height, float resY, int* y_lo,
                     int* y_hi) {
    *y_lo = 0;
    *y_hi = height;
    const double R[3] = {cam.Right.x, cam.Right.y, cam.Right.z}, F[3] = {cam.Front.x, cam.Front.y, cam.Front.z},
                 U[3] = {cam.Up.x, cam.Up.y, cam.Up.z}, o[3] = {cam.Position.x, cam.Position.y, cam.Position.z};
    auto cross = [](const double a[3], const double b[3], double r[3]) {
        r[0] = a[1] * b[2] - a[2] * b[1];
        r[1] = a[2] * b[0] - a[0] * b[2];
        r[2] = a[0] * b[1] - a[1] * b[0];
    };
    double n0[3], n1[3];
    cross(R, F, n0);
    cross(R, U, n1);
    // h = 2 tan(radians(fov / 2)) as the shader (:156); only its size matters here
    const double h = 2.0 * std::tan(static_cast<double>(cam.fov) / 2.0 * 0.017453292519943295);
    for (int a = 0; a < 3; ++a) {
        if (!std::isfinite(lo[a]) || !std::isfinite(hi[a]) || !(lo[a] <= hi[a])) return false;
        if (!std::isfinite(R[a]) || !std::isfinite(F[a]) || !std::isfinite(U[a]) || !std::isfinite(o[a])) return false;
    }
    if (!std::isfinite(h) || !(resY > 0) || height <= 0) return false;
    auto dot = [](const double a[3], const double b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; };
    auto l1 = [](const double a[3]) { return std::fabs(a[0]) + std::fabs(a[1]) + std::fabs(a[2]); };
    const double fl = std::sqrt(dot(F, F)), rl = std::sqrt(dot(R, R)), ul = std::sqrt(dot(U, U));
    // |P - pos| >= |front| needs right and up orthogonal to front (to 1e-3)
    if (!(fl > 0) || std::fabs(dot(R, F)) > 1e-3 * rl * fl || std::fabs(dot(U, F)) > 1e-3 * ul * fl) return false;
    const double w = h * std::fabs(static_cast<double>(cam.aspectRatio));
    if (!std::isfinite(w)) return false;
    const double ang = 1e-4 + 32.0 * 5.9604644775390625e-08 * (l1(o) + l1(F) + 0.5 * w * l1(R) + 0.5 * h * l1(U)) / fl;
    // per corner: s(ndcY) = a + ndcY b, the side of the corner; m its margin
    double ca[8], cb[8], cm[8];
    for (int k = 0; k < 8; ++k) {
        const double c[3] = {(k & 1 ? hi[0] : lo[0]) - o[0], (k & 2 ? hi[1] : lo[1]) - o[1],
                             (k & 4 ? hi[2] : lo[2]) - o[2]};
        ca[k] = n0[0] * c[0] + n0[1] * c[1] + n0[2] * c[2];
        cb[k] = 0.5 * h * (n1[0] * c[0] + n1[1] * c[1] + n1[2] * c[2]);
        cm[k] = std::sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
    }
    auto sky = [&](int y) {
        const double ny = 1.0 - 2.0 * y / static_cast<double>(resY);
        // |n(ny)| bounds the normal's length for the margin
        const double nn[3] = {n0[0] + 0.5 * h * ny * n1[0], n0[1] + 0.5 * h * ny * n1[1], n0[2] + 0.5 * h * ny * n1[2]};
        const double nl = std::sqrt(nn[0] * nn[0] + nn[1] * nn[1] + nn[2] * nn[2]);
        if (!(nl > 0)) return false;
        int pos = 0, neg = 0;
        for (int k = 0; k < 8; ++k) {
            const double s = ca[k] + ny * cb[k], m = ang * nl * cm[k] + 1e-9;
            pos += s > m;
            neg += s < -m;
        }
        return pos == 8 || neg == 8;
    };
    int a = 0, b = height;
    while (a < b && sky(a)) ++a;
    while (b > a && sky(b - 1)) --b;
    *y_lo = a;
    *y_hi = b;
    return true;
}

}  // namespace rtg

#endif

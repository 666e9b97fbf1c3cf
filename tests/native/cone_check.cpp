// Conservativeness of the quantized back-face cones (accel_math.h cone_word /
// cone_culls_q / ray_dq, the wide nodes of rt_kernels.hip): whenever the
// quantized test culls, the float cone's own condition a.d < thr holds for the
// exact unit direction (evaluated in long double). Random unit axes, thresholds
// over the range build_cones emits (-sin(theta + margin), plus the never-cull
// and kNoPrune codes) and random directions of lengths 0.5-2, biased toward
// the cull boundary. Also checks the special words and the host sdot4.
#include <cmath>
#include <cstdio>
#include <random>

#include "../../opengl-ray-tracer_amd/csrc/accel_math.h"

namespace {
int fails = 0;
void check(bool ok, const char* what) {
    if (!ok && fails++ < 10) std::printf("FAIL %s\n", what);
}
}  // namespace

int main() {
    std::mt19937_64 rng(12345);
    std::uniform_real_distribution<double> u(-1.0, 1.0), len(0.5, 2.0), th(0.0, 1.5707);
    auto unit = [&](double v[3]) {
        for (;;) {
            for (int i = 0; i < 3; ++i) v[i] = u(rng);
            const double l = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
            if (l > 0.1 && l <= 1.0) {
                for (int i = 0; i < 3; ++i) v[i] /= l;
                return;
            }
        }
    };
    // special words
    check(rta::cone_word(0.f, 0.f, 1.f, -8.f) == rta::kConeNp, "kNoPrune -> kConeNp");
    check(rta::cone_word(0.f, 0.f, 0.f, -4.f) == rta::kConeNever, "never-cull -> kConeNever");
    check(rta::cone_word(0.f, 0.f, 1.f, NAN) == rta::kConeNever, "NaN threshold -> kConeNever");
    check(rta::cone_word(NAN, 0.f, 1.f, -0.1f) == rta::kConeNever, "NaN axis -> kConeNever");
    check(rta::cone_word(1.f, 1.f, 0.f, -0.1f) == rta::kConeNever, "non-unit axis -> kConeNever");
    check(rta::sdot4(static_cast<int>(0x80ff7f01u), static_cast<int>(0x80ff7f01u)) == 1 + 127 * 127 + 1 + 128 * 128,
          "host sdot4");
    long long culls = 0, trials = 0, dirs = 0;
    for (int a = 0; a < 20000; ++a) {
        double ax[3];
        unit(ax);
        const float fa[3] = {static_cast<float>(ax[0]), static_cast<float>(ax[1]), static_cast<float>(ax[2])};
        const float thr = static_cast<float>(-std::sin(th(rng)));
        const int w = rta::cone_word(fa[0], fa[1], fa[2], thr);
        for (int k = 0; k < 200; ++k) {
            double d[3];
            unit(d);
            if (k & 1) {  // near the boundary: d = cos(phi) a + sin(phi) p with a.d ~ thr
                double p[3] = {d[1] * ax[2] - d[2] * ax[1], d[2] * ax[0] - d[0] * ax[2], d[0] * ax[1] - d[1] * ax[0]};
                const double pl = std::sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]);
                if (!(pl > 1e-6)) continue;
                const double c = static_cast<double>(thr) + 0.03 * u(rng), s = std::sqrt(std::max(0.0, 1 - c * c));
                for (int i = 0; i < 3; ++i) d[i] = c * ax[i] + s * p[i] / pl;
            }
            const double l = len(rng);
            const float fd[3] = {static_cast<float>(d[0] * l), static_cast<float>(d[1] * l), static_cast<float>(d[2] * l)};
            const rta::RayC rc = rta::ray_consts(0.f, 0.f, 0.f, fd[0], fd[1], fd[2], 1e30f);
            ++dirs;
            if (!rta::cone_culls_q(w, rc.dq)) continue;
            ++culls;
            const long double dl = std::sqrt(static_cast<long double>(fd[0]) * fd[0] +
                                             static_cast<long double>(fd[1]) * fd[1] +
                                             static_cast<long double>(fd[2]) * fd[2]);
            const long double dot = (static_cast<long double>(fa[0]) * fd[0] + static_cast<long double>(fa[1]) * fd[1] +
                                     static_cast<long double>(fa[2]) * fd[2]) / dl;
            ++trials;
            check(dot < thr, "quantized cull implies a.d < thr");
        }
        // the special words never cull
        double d[3];
        unit(d);
        const rta::RayC rc = rta::ray_consts(0.f, 0.f, 0.f, static_cast<float>(d[0]), static_cast<float>(d[1]),
                                             static_cast<float>(d[2]), 1e30f);
        check(!rta::cone_culls_q(rta::kConeNp, rc.dq) && !rta::cone_culls_q(rta::kConeNever, rc.dq),
              "special words never cull");
        const rta::RayC anti = rta::ray_consts(0.f, 0.f, 0.f, -fa[0], -fa[1], -fa[2], 1e30f);
        check(!rta::cone_culls_q(rta::cone_word(fa[0], fa[1], fa[2], -4.f), anti.dq), "thr -4 never culls");
    }
    std::printf("cone_check %s: %lld of %lld directions culled, all inside the float cone's bound\n",
                fails ? "FAILED" : "ok", culls, dirs);
    (void)trials;
    return fails ? 1 : 0;
}

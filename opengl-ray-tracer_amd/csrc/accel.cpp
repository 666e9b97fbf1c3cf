// accel.cpp — host-side builder of the exact-result accelerator. See accel.h
// for the contract; the bounds below are what makes skipping a shape safe.
#include "accel.h"
#include "accel_bound.h"

#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <numeric>
#include <exception>
#include <thread>

namespace rta {
namespace {

Box3 empty_box() {
    Box3 b;
    for (int i = 0; i < 3; ++i) {
        b.lo[i] = INFINITY;
        b.hi[i] = -INFINITY;
    }
    return b;
}

void grow(Box3& a, const Box3& b) {
    for (int i = 0; i < 3; ++i) {
        a.lo[i] = std::min(a.lo[i], b.lo[i]);
        a.hi[i] = std::max(a.hi[i], b.hi[i]);
    }
}

float area(const Box3& b) {
    float e[3];
    for (int i = 0; i < 3; ++i) e[i] = std::max(0.f, b.hi[i] - b.lo[i]);
    return e[0] * e[1] + e[1] * e[2] + e[2] * e[0];
}

struct Item {
    int shape, seq;
    Box3 box;
    float c[3];
    float n[3] = {0, 0, 0};  // MT: the triangle's unit normal, either orientation (hn)
    bool hn = false;
    bool big = false;  // MT: |e1||e2| > kMtBigX (its 1e-5 floor bound is loose or absent)
};

// MT triangles with |e1||e2| above this are kept apart from the rest at the
// first split of a local tree (mt_pad takes a node's worst |e1||e2| with its
// smallest |e1 x e2|, so mixing them would leave every ancestor unbounded).
#ifndef RTA_MT_BIG_X
#define RTA_MT_BIG_X 4.0
#endif
constexpr double kMtBigX = RTA_MT_BIG_X;


// MT builds (AccelHost::mt): the orientation-free normal cone of the items a
// predicate selects, as the build's cost model sees it (build_cones_mt computes
// the walk's conservative cones afterwards). theta < 0: no triangle.
struct NCone {
    double a[3] = {0, 0, 0};
    double theta = -1;
};

template <class F>
NCone normal_cone(const std::vector<Item>& items, int b, int e, F sel) {
    NCone c;
    const float* ref = nullptr;
    double s[3] = {0, 0, 0};
    for (int i = b; i < e; ++i) {
        const Item& it = items[i];
        if (!it.hn || !sel(it)) continue;
        if (!ref) ref = it.n;
        const double f = (it.n[0] * ref[0] + it.n[1] * ref[1] + it.n[2] * ref[2]) < 0 ? -1.0 : 1.0;
        for (int a = 0; a < 3; ++a) s[a] += f * it.n[a];
    }
    if (!ref) return c;
    const double l = std::sqrt(s[0] * s[0] + s[1] * s[1] + s[2] * s[2]);
    if (!(l > 1e-9)) {
        c.theta = 1.5708;
        return c;
    }
    for (int a = 0; a < 3; ++a) c.a[a] = s[a] / l;
    c.theta = 0;
    for (int i = b; i < e; ++i) {
        const Item& it = items[i];
        if (!it.hn || !sel(it)) continue;
        const double d = std::fabs(it.n[0] * c.a[0] + it.n[1] * c.a[1] + it.n[2] * c.a[2]);
        c.theta = std::max(c.theta, std::acos(std::min(1.0, d)));
    }
    return c;
}

// MT: a normal split is taken while it costs less than kMtNormalBias times the
// spatial one, and local leaves hold up to kMtLeaf prims. The cost model prices
// grazing for uniformly spread directions (kMtBuildPsi); camera and reflection
// rays are not. Round 2 (forced grazing entry) measured bias 4 best against 1, 2
// and 8 (profiles/r02zz3_abf_mt_*); round 3 (per-ray padding) re-measured leaves
// of 2 against 1 and 4 (profiles/r03j_ab_mt_variants.txt), and the bias and
// kMtBuildPsi as neutral in the CPU emulation (node steps per car camera ray).
#ifndef RTA_MT_NORMAL_BIAS
#define RTA_MT_NORMAL_BIAS 4.0
#endif
constexpr double kMtNormalBias = RTA_MT_NORMAL_BIAS;
#ifndef RTA_MT_LEAF
#define RTA_MT_LEAF 2
#endif
constexpr int kMtLeaf = RTA_MT_LEAF;  // MT local leaves hold at most this many prims
#ifndef RTA_MT_BUILD_PSI
#define RTA_MT_BUILD_PSI 0.032
#endif
constexpr double kMtBuildPsi = RTA_MT_BUILD_PSI;  // the cost model's grazing margin (rad)

struct LocalBuilder {
    AccelHost& out;
    std::vector<Item> items;
    int max_depth_seen = 0;

    // MT cost of one side of a split: the chance that a ray which reaches the
    // parent enters the child -- its grazing cone's chance for uniform directions,
    // sin(theta + psi), where the walk enters whatever the box says, plus the box's
    // share of the parent's area otherwise -- times the child's items.
    template <class F>
    double mt_side_cost(int b, int e, float parent_area, F sel) const {
        Box3 box = empty_box();
        int n = 0;
        for (int i = b; i < e; ++i)
            if (sel(items[i])) {
                grow(box, items[i].box);
                ++n;
            }
        if (n == 0) return 0;
        const NCone c = normal_cone(items, b, e, sel);
        const double psi = kMtBuildPsi;
        const double g = c.theta < 0 ? 0.0 : std::sin(std::min(1.5707963, c.theta + psi));
        const double f = parent_area > 0 ? std::min(1.0, static_cast<double>(area(box)) / parent_area) : 1.0;
        return n * (g + (1 - g) * f);
    }

    // MT: split [b, e) by normal orientation (2-means on orientation-free normals,
    // seeded by the cone axis and the normal farthest from it). Returns the seeds.
    bool normal_seeds(int b, int e, const NCone& pc, double s0[3], double s1[3]) const {
        double worst = 2;
        int far = -1;
        for (int i = b; i < e; ++i) {
            if (!items[i].hn) continue;
            const double d = std::fabs(items[i].n[0] * pc.a[0] + items[i].n[1] * pc.a[1] + items[i].n[2] * pc.a[2]);
            if (d < worst) {
                worst = d;
                far = i;
            }
        }
        if (far < 0) return false;
        for (int a = 0; a < 3; ++a) {
            s0[a] = pc.a[a];
            s1[a] = items[far].n[a];
        }
        for (int iter = 0; iter < 3; ++iter) {
            double m0[3] = {0, 0, 0}, m1[3] = {0, 0, 0};
            for (int i = b; i < e; ++i) {
                const Item& it = items[i];
                if (!it.hn) continue;
                const double d0 = it.n[0] * s0[0] + it.n[1] * s0[1] + it.n[2] * s0[2];
                const double d1 = it.n[0] * s1[0] + it.n[1] * s1[1] + it.n[2] * s1[2];
                const bool left = std::fabs(d0) >= std::fabs(d1);
                const double f = (left ? d0 : d1) < 0 ? -1.0 : 1.0;
                for (int a = 0; a < 3; ++a) (left ? m0 : m1)[a] += f * it.n[a];
            }
            const double l0 = std::sqrt(m0[0] * m0[0] + m0[1] * m0[1] + m0[2] * m0[2]);
            const double l1 = std::sqrt(m1[0] * m1[0] + m1[1] * m1[1] + m1[2] * m1[2]);
            if (!(l0 > 1e-9) || !(l1 > 1e-9)) break;
            for (int a = 0; a < 3; ++a) {
                s0[a] = m0[a] / l0;
                s1[a] = m1[a] / l1;
            }
        }
        return true;
    }

    int leaf(int b, int e) {
        int k = static_cast<int>(out.lbox.size());
        Box3 box = empty_box();
        for (int i = b; i < e; ++i) grow(box, items[i].box);
        out.lbox.push_back(box);
        out.la.push_back(-(static_cast<int>(out.prim_shape.size()) + 1));
        out.lb.push_back(e - b);
        // keep the reference order inside a leaf (cheaper ties, same result)
        std::sort(items.begin() + b, items.begin() + e, [](const Item& x, const Item& y) { return x.seq < y.seq; });
        for (int i = b; i < e; ++i) {
            out.prim_shape.push_back(items[i].shape);
            out.prim_seq.push_back(items[i].seq);
        }
        ++out.local_leaves;
        return k;
    }

    // Binned SAH over centroids; `budget` = levels still allowed.
    int build(int b, int e, int depth, int budget) {
        max_depth_seen = std::max(max_depth_seen, depth);
        const int n = e - b;
        if (n <= (out.mt ? kMtLeaf : 4) || budget <= 0) return leaf(b, e);
        if (out.mt) {
            const int nb = static_cast<int>(std::count_if(items.begin() + b, items.begin() + e,
                                                          [](const Item& x) { return x.big; }));
            if (nb > 0 && nb < n) {
                auto it = std::partition(items.begin() + b, items.begin() + e, [](const Item& x) { return x.big; });
                return inner(b, static_cast<int>(it - items.begin()), e, 0, depth, budget);
            }
        }
        Box3 box = empty_box();
        float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int i = b; i < e; ++i) {
            grow(box, items[i].box);
            for (int a = 0; a < 3; ++a) {
                clo[a] = std::min(clo[a], items[i].c[a]);
                chi[a] = std::max(chi[a], items[i].c[a]);
            }
        }
        int axis = 0;
        for (int a = 1; a < 3; ++a)
            if (chi[a] - clo[a] > chi[axis] - clo[axis]) axis = a;
        int mid = b;
        const float ext = chi[axis] - clo[axis];
        if (ext > 0) {
            constexpr int kBins = 16;
            int cnt[kBins] = {0};
            Box3 bb[kBins];
            for (auto& x : bb) x = empty_box();
            auto bin_of = [&](const Item& it) {
                const float f = (it.c[axis] - clo[axis]) / ext * kBins;
                if (!(f >= 1.0f)) return 0;  // NaN never converts to int
                return f >= static_cast<float>(kBins - 1) ? kBins - 1 : static_cast<int>(f);
            };
            for (int i = b; i < e; ++i) {
                int k = bin_of(items[i]);
                ++cnt[k];
                grow(bb[k], items[i].box);
            }
            float best = INFINITY;
            int best_k = -1;
            Box3 lacc = empty_box();
            int lcnt = 0;
            float lcost[kBins];
            for (int k = 0; k < kBins - 1; ++k) {
                grow(lacc, bb[k]);
                lcnt += cnt[k];
                lcost[k] = lcnt ? area(lacc) * lcnt : 0.f;
            }
            Box3 racc = empty_box();
            int rcnt = 0;
            for (int k = kBins - 1; k >= 1; --k) {
                grow(racc, bb[k]);
                rcnt += cnt[k];
                float c = lcost[k - 1] + (rcnt ? area(racc) * rcnt : 0.f);
                if (rcnt && rcnt < n && c < best) {
                    best = c;
                    best_k = k;
                }
            }
            bool by_normal = false;
            double s0[3], s1[3];
            auto normal_left = [&](const Item& x) {
                if (!x.hn) return true;
                return std::fabs(x.n[0] * s0[0] + x.n[1] * s0[1] + x.n[2] * s0[2]) >=
                       std::fabs(x.n[0] * s1[0] + x.n[1] * s1[1] + x.n[2] * s1[2]);
            };
            if (out.mt) {
                // MT: a spatial split leaves wide grazing cones, which rays enter
                // wherever they are; a split by normal orientation tightens them. The
                // cheaper of the two by mt_side_cost.
                const NCone pc = normal_cone(items, b, e, [](const Item&) { return true; });
                const float pa = area(box);
                double sc = INFINITY;
                if (best_k > 0)
                    sc = mt_side_cost(b, e, pa, [&](const Item& x) { return bin_of(x) < best_k; }) +
                         mt_side_cost(b, e, pa, [&](const Item& x) { return !(bin_of(x) < best_k); });
                if (pc.theta > 0.02 && normal_seeds(b, e, pc, s0, s1)) {
                    int nl = 0;
                    for (int i = b; i < e; ++i) nl += normal_left(items[i]) ? 1 : 0;
                    if (nl > 0 && nl < n) {
                        const double nc = mt_side_cost(b, e, pa, normal_left) +
                                          mt_side_cost(b, e, pa, [&](const Item& x) { return !normal_left(x); });
                        by_normal = nc < sc * kMtNormalBias;
                    }
                }
            }
            if (by_normal) {
                auto it = std::partition(items.begin() + b, items.begin() + e, normal_left);
                mid = static_cast<int>(it - items.begin());
            } else if (best_k > 0) {
                auto it = std::partition(items.begin() + b, items.begin() + e,
                                         [&](const Item& x) { return bin_of(x) < best_k; });
                mid = static_cast<int>(it - items.begin());
            }
        }
        if (mid <= b || mid >= e) {  // all centroids equal or no useful split: halve by count
            mid = b + n / 2;
            std::nth_element(items.begin() + b, items.begin() + mid, items.begin() + e,
                             [&](const Item& x, const Item& y) { return x.c[axis] < y.c[axis]; });
        }
        return inner(b, mid, e, axis, depth, budget);
    }

    int inner(int b, int mid, int e, int axis, int depth, int budget) {
        Box3 box = empty_box();
        for (int i = b; i < e; ++i) grow(box, items[i].box);
        const int k = static_cast<int>(out.lbox.size());
        out.lbox.push_back(box);
        out.la.push_back(0);
        out.lb.push_back(0);
        const int l = build(b, mid, depth + 1, budget - 1);
        const int r = build(mid, e, depth + 1, budget - 1);
        out.la[k] = l;
        out.lb[k] = r | (axis << 30);
        return k;
    }
};

}  // namespace


namespace {

struct Cone {
    double a[3];
    double theta;  // half angle; > pi/2 = full
    bool full() const { return theta >= 1.5; }
};

Cone full_cone() { return Cone{{0, 0, 0}, 10.0}; }

// The INNER-capable normal of a shape: np = N.d must be > 0 for plane, wall
// and (barycentric) triangle hits; spheres have every direction.
Cone shape_cone(const FlatShape& s) {
    if (s.type != RT_WALL && s.type != RT_TRIANGLE) return full_cone();
    double n[3] = {s.planeNormal.x, s.planeNormal.y, s.planeNormal.z};
    double l = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
    if (!(l > 1e-20) || !std::isfinite(l)) return full_cone();
    return Cone{{n[0] / l, n[1] / l, n[2] / l}, 0.0};
}

Cone merge(const Cone& x, const Cone& y) {
    if (x.full() || y.full()) return full_cone();
    double a[3] = {x.a[0] + y.a[0], x.a[1] + y.a[1], x.a[2] + y.a[2]};
    double l = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
    if (!(l > 1e-6)) return full_cone();
    for (double& v : a) v /= l;
    auto ang = [&](const double* b) {
        double c = a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
        return std::acos(std::max(-1.0, std::min(1.0, c)));
    };
    Cone c{{a[0], a[1], a[2]}, std::max(ang(x.a) + x.theta, ang(y.a) + y.theta)};
    return c.full() ? full_cone() : c;
}

}  // namespace

// Moller-Trumbore: the unit normal of e1 x e2 (edges as the device computes
// them, float), either orientation (|cos| decides); `none` for other shapes.
bool mt_normal(const FlatShape& s, double n[3]) {
    if (s.type != RT_TRIANGLE) return false;
    const float e1[3] = {s.triP2.x - s.triP1.x, s.triP2.y - s.triP1.y, s.triP2.z - s.triP1.z};
    const float e2[3] = {s.triP3.x - s.triP1.x, s.triP3.y - s.triP1.y, s.triP3.z - s.triP1.z};
    const double c[3] = {static_cast<double>(e1[1]) * e2[2] - static_cast<double>(e1[2]) * e2[1],
                         static_cast<double>(e1[2]) * e2[0] - static_cast<double>(e1[0]) * e2[2],
                         static_cast<double>(e1[0]) * e2[1] - static_cast<double>(e1[1]) * e2[0]};
    const double l = std::sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
    if (!(l > 0) || !std::isfinite(l)) return false;
    for (int i = 0; i < 3; ++i) n[i] = c[i] / l;
    return true;
}

// Grazing cones (AccelHost::mt): per node the axis and half angle of the
// triangle normals below, orientation-free (each normal is flipped towards the
// running axis before merging).
struct GCone {
    double a[3] = {0, 0, 0};
    double theta = -1;  // < 0: no triangle below
};

GCone gmerge(const GCone& x, const GCone& y) {
    if (x.theta < 0) return y;
    if (y.theta < 0) return x;
    if (x.theta >= 1.5 || y.theta >= 1.5) return GCone{{0, 0, 0}, 10.0};
    double ya[3] = {y.a[0], y.a[1], y.a[2]};
    if (x.a[0] * ya[0] + x.a[1] * ya[1] + x.a[2] * ya[2] < 0)
        for (double& v : ya) v = -v;
    double a[3] = {x.a[0] + ya[0], x.a[1] + ya[1], x.a[2] + ya[2]};
    double l = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
    if (!(l > 1e-6)) return GCone{{0, 0, 0}, 10.0};
    for (double& v : a) v /= l;
    auto ang = [&](const double* b) {
        double c = a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
        return std::acos(std::max(-1.0, std::min(1.0, c)));
    };
    return GCone{{a[0], a[1], a[2]}, std::max(ang(x.a) + x.theta, ang(ya) + y.theta)};
}

namespace {

// Host threads for the builds' independent halves (at most 16: the GPU box's CPU
// share per GPU). 1 on a one-core host; RTA_BUILD_THREADS overrides it (1-64; the
// accelerator is the same for every count, tests/test_accel_cpu.py).
int build_threads() {
    if (const char* e = std::getenv("RTA_BUILD_THREADS")) {
        const int v = std::atoi(e);
        if (v >= 1) return std::min(v, 64);
    }
    const unsigned h = std::thread::hardware_concurrency();
    return static_cast<int>(std::max(1u, std::min(16u, h)));
}

// fn(i0, i1) over [0, n) in contiguous chunks on up to build_threads() threads (the
// calling one included); chunk c is [c n / T, (c + 1) n / T).
template <class F>
void parallel_chunks(int n, int min_per_thread, F fn) {
    const int T = std::max(1, std::min(build_threads(), n / std::max(1, min_per_thread)));
    if (T <= 1) {
        fn(0, n, 0);
        return;
    }
    std::vector<std::thread> th;
    std::vector<std::exception_ptr> err(T);  // rethrown on the calling thread after every join
    for (int c = 1; c < T; ++c)
        th.emplace_back([&, c] {
            try {
                fn(static_cast<int>(static_cast<long long>(c) * n / T),
                   static_cast<int>(static_cast<long long>(c + 1) * n / T), c);
            } catch (...) {
                err[c] = std::current_exception();
            }
        });
    try {
        fn(0, static_cast<int>(static_cast<long long>(n) / T), 0);
    } catch (...) {
        err[0] = std::current_exception();
    }
    for (auto& t : th) t.join();
    for (auto& e : err)
        if (e) std::rethrow_exception(e);
}

}  // namespace

void build_cones_mt(const FlatShape* shapes, AccelHost& A) {
    const size_t M = A.lbox.size();
    A.lcone.assign(4 * M, 0.f);
    std::vector<GCone> cones(M);
    std::vector<char> done(M, 0);
    std::function<const GCone&(size_t)> get = [&](size_t j) -> const GCone& {
        if (done[j]) return cones[j];
        GCone c;
        if (A.la[j] < 0) {
            const int st = -A.la[j] - 1, n = A.lb[j];
            for (int i = 0; i < n; ++i) {
                GCone one;
                if (mt_normal(shapes[A.prim_shape[st + i]], one.a)) one.theta = 0.0;
                c = gmerge(c, one);
            }
        } else {
            c = gmerge(get(static_cast<size_t>(A.la[j])), get(static_cast<size_t>(A.lb[j] & 0x3fffffff)));
        }
        cones[j] = c;
        done[j] = 1;
        return cones[j];
    };
    // Per-ray padding (accel_bound.h, MtTri; accel_math.h mt_pad): the cone's
    // s = 2 sin(theta/2) bounds |n - axis| for every normal below, so
    // |cos(d, n)| >= |d . axis| - s; the node constants take the worst triangle.
    // per prim its MT constants, on the build threads (min/max per chunk, exact in any order)
    const int np = static_cast<int>(A.prim_shape.size());
    std::vector<MtTri> tri(A.prim_shape.size());
    std::vector<char> has(A.prim_shape.size(), 0);
    const int nt = build_threads();
    std::vector<double> zr(6 * static_cast<size_t>(nt));
    for (int c = 0; c < nt; ++c)
        for (int a = 0; a < 3; ++a) {
            zr[6 * c + a] = INFINITY;
            zr[6 * c + 3 + a] = -INFINITY;
        }
    parallel_chunks(np, 4096, [&](int p0, int p1, int c) {
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int p = p0; p < p1; ++p) {
            const FlatShape& s = shapes[A.prim_shape[p]];
            Box3 b;
            if (s.type != RT_TRIANGLE || classify_mt_tight(s, b, 0.0, tri[p]) != BOUNDED) continue;
            has[p] = 1;
            if (tri[p].X > kMtBigX) continue;  // Z: the centre of the bulk, not of a large ground quad
            for (int a = 0; a < 3; ++a) {
                lo[a] = std::min(lo[a], tri[p].p1[a]);
                hi[a] = std::max(hi[a], tri[p].p1[a]);
            }
        }
        for (int a = 0; a < 3; ++a) {
            zr[6 * c + a] = lo[a];
            zr[6 * c + 3 + a] = hi[a];
        }
    });
    double zlo[3] = {INFINITY, INFINITY, INFINITY}, zhi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int c = 0; c < nt; ++c)
        for (int a = 0; a < 3; ++a) {
            zlo[a] = std::min(zlo[a], zr[6 * c + a]);
            zhi[a] = std::max(zhi[a], zr[6 * c + 3 + a]);
        }
    for (int a = 0; a < 3; ++a) A.mt_z[a] = std::isfinite(zlo[a]) ? static_cast<float>(0.5 * (zlo[a] + zhi[a])) : 0.f;
    struct Agg {
        double cr = INFINITY, X = 0, esum = 0, m = 0;
    };
    // slab along the cone axis (mt_slab): min/max of a . vertex over the triangles below
    auto slab = [&](size_t j, const float* ax, double& w, double& h0) {
        double lo = INFINITY, hi = -INFINITY;
        std::function<void(size_t)> rec = [&](size_t b) {
            if (A.la[b] < 0) {
                const int st = -A.la[b] - 1, n = A.lb[b];
                for (int i = 0; i < n; ++i) {
                    if (!has[st + i]) {  // a sphere (or other shape) below: its hits are not in any slab
                        lo = -INFINITY;
                        hi = INFINITY;
                        continue;
                    }
                    const FlatShape& s = shapes[A.prim_shape[st + i]];
                    for (const rt_vec3& v : {s.triP1, s.triP2, s.triP3}) {
                        const double x = static_cast<double>(ax[0]) * v.x + static_cast<double>(ax[1]) * v.y +
                                         static_cast<double>(ax[2]) * v.z;
                        lo = std::min(lo, x);
                        hi = std::max(hi, x);
                    }
                }
            } else {
                rec(static_cast<size_t>(A.la[b]));
                rec(static_cast<size_t>(A.lb[b] & 0x3fffffff));
            }
        };
        rec(j);
        const bool fin = std::isfinite(lo) && std::isfinite(hi);
        w = fin ? 0.5 * (lo + hi) : 0.0;
        h0 = fin ? 0.5 * (hi - lo) : INFINITY;
    };
    std::vector<Agg> agg(M);
    std::vector<char> adone(M, 0);
    std::function<const Agg&(size_t)> aget = [&](size_t j) -> const Agg& {
        if (adone[j]) return agg[j];
        Agg g;
        auto merge_in = [&](const Agg& x) {
            g.cr = std::min(g.cr, x.cr);
            g.X = std::max(g.X, x.X);
            g.esum = std::max(g.esum, x.esum);
            g.m = std::max(g.m, x.m);
        };
        if (A.la[j] < 0) {
            const int st = -A.la[j] - 1, n = A.lb[j];
            for (int i = 0; i < n; ++i) {
                if (!has[st + i]) continue;
                const MtTri& t = tri[st + i];
                const double dz[3] = {t.p1[0] - A.mt_z[0], t.p1[1] - A.mt_z[1], t.p1[2] - A.mt_z[2]};
                merge_in(Agg{t.cr, t.X, t.esum, std::sqrt(dz[0] * dz[0] + dz[1] * dz[1] + dz[2] * dz[2])});
            }
        } else {
            merge_in(aget(static_cast<size_t>(A.la[j])));
            merge_in(aget(static_cast<size_t>(A.lb[j] & 0x3fffffff)));
        }
        agg[j] = g;
        adone[j] = 1;
        return agg[j];
    };
    A.lmt.assign(kMtPadF * M, 0.f);
    auto mt_record = [&](size_t j) {
        const GCone& c = cones[j];
        float* o = &A.lcone[4 * j];
        o[0] = static_cast<float>(c.a[0]);
        o[1] = static_cast<float>(c.a[1]);
        o[2] = static_cast<float>(c.a[2]);
        o[3] = (c.theta < 0 || c.theta >= 1.5) ? 2.f : static_cast<float>(2.0 * std::sin(0.5 * c.theta + 1e-6) + 2e-5);
        const Agg& g = agg[j];
        float* m = &A.lmt[kMtPadF * j];
        if (!(g.X > 0)) {  // no triangle below: pad 0, no slab
            m[5] = INFINITY;
            return;
        }
        const double up = 1.0 + 1e-5;
        m[0] = static_cast<float>(g.cr * (1.0 - 1e-5));
        m[1] = static_cast<float>(kU * g.X * up);
        m[2] = static_cast<float>(g.m * up + 1e-5);
        m[3] = static_cast<float>((18.0 * g.m + 10.5 * g.esum) * up + 1e-5);
        double w, h0;
        slab(j, o, w, h0);
        m[4] = static_cast<float>(w);
        m[5] = static_cast<float>(h0 * up + 1e-5 * (std::fabs(w) + 1.0));
        // (measured in tests/native/accel_check: skipping the slab of wide cones,
        // sin > 0.3, or of nodes thicker along the axis than 1/4 of their box
        // raises the car's node steps per camera ray from 79 to 94)
    };
    for (size_t j = 0; j < M; ++j) {  // every node's cone and aggregate first (memoised recursion)
        get(j);
        aget(j);
    }
    // then each node's record on the build threads: its slab walks its own subtree
    // (read-only), so the nodes are independent
    parallel_chunks(static_cast<int>(M), 1024, [&](int j0, int j1, int) {
        for (size_t j = static_cast<size_t>(j0); j < static_cast<size_t>(j1); ++j) mt_record(j);
    });
}

void build_cones(const FlatShape* shapes, AccelHost& A) {
    if (A.mt) {
        build_cones_mt(shapes, A);
        return;
    }
    const size_t M = A.lbox.size();
    A.lcone.assign(4 * M, 0.f);
    std::vector<Cone> cones(M, full_cone());
    auto store = [&](size_t j) {
        const Cone& c = cones[j];
        float* o = &A.lcone[4 * j];
        const double t = c.theta + kConeMargin;
        if (c.full() || t >= 1.5707) {
            o[0] = o[1] = o[2] = 0.f;
            o[3] = -4.f;
        } else {
            o[0] = static_cast<float>(c.a[0]);
            o[1] = static_cast<float>(c.a[1]);
            o[2] = static_cast<float>(c.a[2]);
            o[3] = static_cast<float>(-std::sin(t));
        }
    };
    // The builders number every tree in preorder (a node, its left subtree, then its
    // right one), so a node's subtree is the index range [j, j + size): subtrees of at
    // most M / 64 nodes are independent units, each merged children first (descending
    // index) on the build threads, then the nodes above them. Each node's cone is the
    // same merge of its children's as in the recursion below (which forests not in
    // preorder take).
    std::vector<int> size(M, 1);
    bool pre = true;
    for (size_t j = M; j-- > 0 && pre;) {
        if (A.la[j] < 0) continue;
        const size_t l = static_cast<size_t>(A.la[j]), r = static_cast<size_t>(A.lb[j] & 0x3fffffff);
        pre = l == j + 1 && r == l + static_cast<size_t>(size[l]) && r < M;
        if (pre) size[j] = 1 + size[l] + size[r];
    }
    if (pre && M >= 32768) {  // (smaller: threads cost more than they save)
        auto one = [&](size_t j) {
            if (A.la[j] < 0) {
                const int st = -A.la[j] - 1, n = A.lb[j];
                Cone c = n > 0 ? shape_cone(shapes[A.prim_shape[st]]) : full_cone();
                for (int i = 1; i < n; ++i) c = merge(c, shape_cone(shapes[A.prim_shape[st + i]]));
                cones[j] = c;
            } else {
                cones[j] = merge(cones[static_cast<size_t>(A.la[j])], cones[static_cast<size_t>(A.lb[j] & 0x3fffffff)]);
            }
            store(j);
        };
        const size_t unit = std::max<size_t>(64, M / 64);
        std::vector<std::pair<size_t, size_t>> units;  // [first, end) of each unit subtree
        std::vector<size_t> top;                      // the nodes above them, ascending
        for (size_t j = 0; j < M;) {
            if (static_cast<size_t>(size[j]) <= unit) {
                units.push_back({j, j + static_cast<size_t>(size[j])});
                j += static_cast<size_t>(size[j]);
            } else {
                top.push_back(j++);
            }
        }
        parallel_chunks(static_cast<int>(units.size()), 4, [&](int u0, int u1, int) {
            for (int u = u0; u < u1; ++u)
                for (size_t j = units[u].second; j-- > units[u].first;) one(j);
        });
        for (size_t q = top.size(); q-- > 0;) one(top[q]);
        return;
    }
    std::vector<char> done(M, 0);
    std::function<const Cone&(size_t)> get = [&](size_t j) -> const Cone& {
        if (done[j]) return cones[j];
        Cone c;
        if (A.la[j] < 0) {
            const int st = -A.la[j] - 1, n = A.lb[j];
            c = n > 0 ? shape_cone(shapes[A.prim_shape[st]]) : full_cone();
            for (int i = 1; i < n; ++i) c = merge(c, shape_cone(shapes[A.prim_shape[st + i]]));
        } else {
            c = merge(get(static_cast<size_t>(A.la[j])), get(static_cast<size_t>(A.lb[j] & 0x3fffffff)));
        }
        cones[j] = c;
        done[j] = 1;
        return cones[j];
    };
    for (size_t j = 0; j < M; ++j) {
        get(j);
        store(j);
    }
}

namespace {

// Inner height of binary local node j: the stack entries a binary walk pushes
// below it on its deepest path (0 for a leaf).
int inner_height(const AccelHost& A, int j, std::vector<int>& memo) {
    if (j < 0 || A.la[j] < 0) return 0;
    if (memo[j] >= 0) return memo[j];
    const int h = 1 + std::max(inner_height(A, A.la[j], memo), inner_height(A, A.lb[j] & 0x3fffffff, memo));
    memo[j] = h;
    return h;
}

// Collapses the binary local tree below binary inner node j into wide nodes:
// a wide node takes j's children, then repeatedly replaces its largest inner
// child (surface area) by that child's two children, up to kWide. A lane walk
// pushes every entered child but the nearest, so a wide node of k children
// adds k - 1 entries to the stack below it; `budget` bounds that sum along
// every path (the expansion stops early where the budget requires). Returns
// the wide id; `pend` = the bound reached.
int make_wide(AccelHost& A, int j, int budget, std::vector<int>& memo, int& pend) {
    auto inner = [&](int b) { return b >= 0 && A.la[b] >= 0; };
    // at most 2 kWide children: fixed arrays, no allocation per wide node
    struct Slots {
        int v[2 * kWide];
        int n = 0;
        int size() const { return n; }
        int& operator[](int i) { return v[i]; }
        int operator[](int i) const { return v[i]; }
    };
    Slots slots;
    slots.v[slots.n++] = A.la[j];
    slots.v[slots.n++] = A.lb[j] & 0x3fffffff;
    auto need = [&](const Slots& sl) {
        int m = 0;
        for (int i = 0; i < sl.n; ++i) m = std::max(m, inner_height(A, sl.v[i], memo));
        return sl.n - 1 + m;
    };
    const int max_kids = A.mt ? kWide : kWideKids;
    static_assert(kWideKids <= 2 * kWide, "Slots holds the widest node");
    for (;;) {
        if (slots.size() >= max_kids) break;
        int pick = -1;
        float best = -1.f;
        for (int s2 = 0; s2 < slots.size(); ++s2)
            if (inner(slots[s2]) && area(A.lbox[slots[s2]]) > best) {
                best = area(A.lbox[slots[s2]]);
                pick = s2;
            }
        if (pick < 0) break;
        Slots next = slots;
        const int b = next[pick];
        next[pick] = A.la[b];
        next.v[next.n++] = A.lb[b] & 0x3fffffff;
        if (need(next) > budget) break;  // deeper expansion would exceed the stack budget
        slots = next;
    }
    // one record of kWide children, or two consecutive ones (a pair: up to 2 kWide)
    const int w = static_cast<int>(A.wchild.size()) / kWide;
    const int recs = static_cast<int>(slots.size()) > kWide ? 2 : 1;
    A.wchild.resize(A.wchild.size() + recs * kWide, -1);
    A.wsub.resize(A.wsub.size() + recs * kWide, -1);
    A.wpair.resize(A.wpair.size() + recs, 0);
    A.wpair[w] = recs == 2;
    const int own = static_cast<int>(slots.size()) - 1;
    int below = 0;
    for (int s2 = 0; s2 < static_cast<int>(slots.size()); ++s2) {
        A.wchild[kWide * w + s2] = slots[s2];
        if (inner(slots[s2])) {
            int p = 0;
            const int sub = make_wide(A, slots[s2], budget - own, memo, p);
            A.wsub[kWide * w + s2] = sub;
            below = std::max(below, p);
        }
    }
    pend = own + below;
    return w;
}

}  // namespace

namespace {

// An atom of the scene tree: the bounded shapes of a small reference leaf
// (kept together), one bounded shape of a large leaf, or up to four unbounded
// shapes of one leaf (infinite box). `first`/`n` index SceneBuilder::ap.
struct Atom {
    int ref, first, n;
    Box3 box;
    float c[3];
};

// Binned SAH over atom centroids (cost = box area x shapes), into T's
// lbox / la / lb / prim_shape / prim_seq (the layout of a local tree, so the
// cone and wide-collapse passes apply). A leaf holds atoms of one reference
// leaf only (n == 1, or all of one leaf with <= 4 shapes). Splits fall back to
// the median where the SAH choice would let the height exceed `hmax`.
#ifndef RT_ITEM_MAX
#define RT_ITEM_MAX 4
#endif
// Shapes of one reference leaf kept together in one scene-tree item (at most; <= 7
// for the few-leaf item codes).
constexpr int kItemMax = RT_ITEM_MAX;

struct SceneBuilder {
    AccelHost& T;
    std::vector<Atom>& atoms;                     // partitioned in place: sub-builders own disjoint ranges
    const std::vector<std::pair<int, int>>& ap;  // (shape, seq)
    std::vector<int> leaf_ref;                    // per node: reference leaf of a leaf, -1 inner
    int hmax = 0, height = 0;
    int par = 0;  // levels below this one whose two halves may still be built on two threads

    // Appends a sub-builder's tree (its nodes and prims numbered from 0, root first)
    // after this one's, as the sequential build would have numbered it; returns the
    // index of its root.
    int splice(const SceneBuilder& o) {
        const int off = static_cast<int>(T.lbox.size()), poff = static_cast<int>(T.prim_shape.size());
        T.lbox.insert(T.lbox.end(), o.T.lbox.begin(), o.T.lbox.end());
        for (size_t j = 0; j < o.T.la.size(); ++j) {
            const int a = o.T.la[j], b = o.T.lb[j];
            if (a >= 0) {  // inner: left, right | axis << 30
                T.la.push_back(a + off);
                T.lb.push_back(((b & 0x3fffffff) + off) | (b & ~0x3fffffff));
            } else {  // leaf: -(start + 1), count
                T.la.push_back(a - poff);
                T.lb.push_back(b);
            }
        }
        T.prim_shape.insert(T.prim_shape.end(), o.T.prim_shape.begin(), o.T.prim_shape.end());
        T.prim_seq.insert(T.prim_seq.end(), o.T.prim_seq.begin(), o.T.prim_seq.end());
        leaf_ref.insert(leaf_ref.end(), o.leaf_ref.begin(), o.leaf_ref.end());
        height = std::max(height, o.height);
        return off;
    }

    int leaf(int b, int e) {
        const int k = static_cast<int>(T.lbox.size());
        Box3 box = empty_box();
        thread_local std::vector<std::pair<int, int>> ps;  // reused: one leaf per atom on config 5
        ps.clear();
        for (int i = b; i < e; ++i) {
            grow(box, atoms[i].box);
            for (int q = atoms[i].first; q < atoms[i].first + atoms[i].n; ++q) ps.push_back(ap[q]);
        }
        std::sort(ps.begin(), ps.end(), [](const auto& x, const auto& y) { return x.second < y.second; });
        T.lbox.push_back(box);
        T.la.push_back(-(static_cast<int>(T.prim_shape.size()) + 1));
        T.lb.push_back(static_cast<int>(ps.size()));
        leaf_ref.push_back(atoms[b].ref);
        for (auto [si, seq] : ps) {
            T.prim_shape.push_back(si);
            T.prim_seq.push_back(seq);
        }
        return k;
    }

    int inner(const Box3& box, int l, int r, int axis) {
        const int k = static_cast<int>(T.lbox.size());
        T.lbox.push_back(box);
        T.la.push_back(l);
        T.lb.push_back(r | (axis << 30));
        leaf_ref.push_back(-1);
        return k;
    }

    static constexpr int kParAtoms = 8192;   // halves smaller than this stay on one thread
    static constexpr int kParAxes = 16384;   // nodes this large sweep their 3 axes on 3 threads

    // bounded = false: atoms with infinite boxes, split by count only.
    int build(int b, int e, int depth, bool bounded) {
        height = std::max(height, depth);
        const int n = e - b;
        bool same = true;
        int tot = 0;
        for (int i = b; i < e; ++i) {
            same = same && atoms[i].ref == atoms[b].ref;
            tot += atoms[i].n;
        }
        if (n == 1 || (same && tot <= kItemMax)) return leaf(b, e);
        Box3 box = empty_box();
        float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int i = b; i < e; ++i) {
            grow(box, atoms[i].box);
            for (int a = 0; a < 3; ++a) {
                clo[a] = std::min(clo[a], atoms[i].c[a]);
                chi[a] = std::max(chi[a], atoms[i].c[a]);
            }
        }
        int axis = 0;
        for (int a = 1; a < 3; ++a)
            if (chi[a] - clo[a] > chi[axis] - clo[axis]) axis = a;
        const int room = hmax - depth - 1;
        // a side of x atoms fits below this level (its binary height ceil(log2 x) <= room)
        const long long fit = room < 0 ? -1 : room >= 62 ? LLONG_MAX : 1LL << room;
        // 256 bins (measured against 32: config 3 -1.4 %, config 2 -2.5 %, config 5 equal;
        // 1024 gains nothing more)
        constexpr int kMaxBins = 256;
        constexpr int kBins = kMaxBins;
        auto bin_of = [&](const Atom& it, int ax) {
            const float ext = chi[ax] - clo[ax];
            const float f = (it.c[ax] - clo[ax]) / ext * kBins;
            // non-finite centres (inf - inf, x / inf) go to bin 0; never convert NaN to int
            if (!(f >= 1.0f)) return 0;
            return f >= static_cast<float>(kBins - 1) ? kBins - 1 : static_cast<int>(f);
        };
        float best = INFINITY;
        int best_k = -1, best_axis = -1;
        // per-thread bin counters, all zero between uses: the sparse sweep clears the bins
        // it touched, the dense one clears every bin (not 2 KB zeroed per axis and node:
        // config 5's scene tree has ~45k inner nodes)
        thread_local int cnt[kMaxBins] = {0}, acnt[kMaxBins] = {0};
        for (int ax = 0; bounded && n < kBins && ax < 3; ++ax) {
            if (!(chi[ax] - clo[ax] > 0)) continue;
            Box3 bb[kMaxBins];
            {
                // Few atoms: only the bins they occupy are set up and swept. Growing by
                // an empty bin is the identity and every boundary inside a run of empty
                // bins makes the same partition at the same cost, so the split found
                // (best_k included: the first of a run scanning down is the next occupied
                // bin) is the dense sweep's (scene-tree hashes equal on configs 2, 3, 5,
                // the 222-strip road and three soups). Config 5's whole accelerator build
                // (93k atoms): 2.1 s -> 0.36 s on the host.
                // the occupied bins in ascending order from a bitmap (no sort)
                unsigned long long occ[kMaxBins / 64] = {};
                for (int i = b; i < e; ++i) {
                    const int k = bin_of(atoms[i], ax);
                    if (acnt[k] == 0) {
                        occ[k >> 6] |= 1ull << (k & 63);
                        bb[k] = empty_box();
                    }
                    cnt[k] += atoms[i].n;
                    ++acnt[k];
                    grow(bb[k], atoms[i].box);
                }
                int used[kMaxBins], nu = 0;
                for (int w = 0; w < kMaxBins / 64; ++w)
                    for (unsigned long long m = occ[w]; m; m &= m - 1) used[nu++] = 64 * w + __builtin_ctzll(m);
                Box3 lacc = empty_box();
                int lcnt = 0, lat = 0;
                float lcost[kMaxBins];
                int lats[kMaxBins];
                for (int j = 0; j < nu; ++j) {
                    grow(lacc, bb[used[j]]);
                    lcnt += cnt[used[j]];
                    lat += acnt[used[j]];
                    lcost[j] = lcnt ? area(lacc) * lcnt : 0.f;
                    lats[j] = lat;
                }
                Box3 racc = empty_box();
                int rcnt = 0, rat = 0;
                for (int j = nu - 1; j >= 1; --j) {
                    const int k = used[j];
                    grow(racc, bb[k]);
                    rcnt += cnt[k];
                    rat += acnt[k];
                    const float c = lcost[j - 1] + (rcnt ? area(racc) * rcnt : 0.f);
                    if (rat && rat < n && c < best && lats[j - 1] <= fit && rat <= fit) {
                        best = c;
                        best_k = k;
                        best_axis = ax;
                    }
                }
                for (int j = 0; j < nu; ++j) cnt[used[j]] = acnt[used[j]] = 0;
            }
        }
        if (bounded && n >= kBins) {
            // Many atoms: every bin. Each axis's cheapest boundary (the first of equal
            // costs in sweep order), then the axes in order, a later one only if strictly
            // cheaper: the sequential sweep's choice. The axes of the largest nodes run on
            // three threads.
            float ab[3] = {INFINITY, INFINITY, INFINITY};
            int ak[3] = {-1, -1, -1};
            auto dense = [&](int ax) {
                if (!(chi[ax] - clo[ax] > 0)) return;
                Box3 bb[kMaxBins];
                for (auto& x : bb) x = empty_box();
                for (int i = b; i < e; ++i) {
                    const int k = bin_of(atoms[i], ax);
                    cnt[k] += atoms[i].n;
                    ++acnt[k];
                    grow(bb[k], atoms[i].box);
                }
                Box3 lacc = empty_box();
                int lcnt = 0, lat = 0;
                float lcost[kMaxBins];
                int lats[kMaxBins];
                for (int k = 0; k < kBins - 1; ++k) {
                    grow(lacc, bb[k]);
                    lcnt += cnt[k];
                    lat += acnt[k];
                    lcost[k] = lcnt ? area(lacc) * lcnt : 0.f;
                    lats[k] = lat;
                }
                Box3 racc = empty_box();
                int rcnt = 0, rat = 0;
                for (int k = kBins - 1; k >= 1; --k) {
                    grow(racc, bb[k]);
                    rcnt += cnt[k];
                    rat += acnt[k];
                    const float c = lcost[k - 1] + (rcnt ? area(racc) * rcnt : 0.f);
                    if (rat && rat < n && c < ab[ax] && lats[k - 1] <= fit && rat <= fit) {
                        ab[ax] = c;
                        ak[ax] = k;
                    }
                }
                std::fill(cnt, cnt + kBins, 0);  // this thread's counters
                std::fill(acnt, acnt + kBins, 0);
            };
            if (par > 0 && n >= kParAxes) {
                std::exception_ptr err[2];
                std::thread t1([&] {
                    try {
                        dense(1);
                    } catch (...) {
                        err[0] = std::current_exception();
                    }
                });
                std::thread t2([&] {
                    try {
                        dense(2);
                    } catch (...) {
                        err[1] = std::current_exception();
                    }
                });
                dense(0);
                t1.join();
                t2.join();
                for (auto& x : err)
                    if (x) std::rethrow_exception(x);
            } else {
                for (int ax = 0; ax < 3; ++ax) dense(ax);
            }
            for (int ax = 0; ax < 3; ++ax)
                if (ak[ax] >= 0 && ab[ax] < best) {
                    best = ab[ax];
                    best_k = ak[ax];
                    best_axis = ax;
                }
        }
        int mid = b;
        if (best_k > 0) {
            axis = best_axis;
            auto it = std::partition(atoms.begin() + b, atoms.begin() + e,
                                     [&](const Atom& x) { return bin_of(x, axis) < best_k; });
            mid = static_cast<int>(it - atoms.begin());
        }
        if (mid <= b || mid >= e) {  // median (no useful SAH split, height bound, or unbounded atoms)
            mid = b + n / 2;
            if (bounded)
                std::nth_element(atoms.begin() + b, atoms.begin() + mid, atoms.begin() + e,
                                 [&](const Atom& x, const Atom& y) { return x.c[axis] < y.c[axis]; });
        }
        const int k = inner(box, 0, 0, axis);
        int l, r;
        if (par > 0 && n >= kParAtoms) {
            // the halves on two threads, each into its own arrays, then appended in the
            // sequential order: the same tree, node for node (tools/native/accel_time.cpp)
            AccelHost tl, tr;
            SceneBuilder L{tl, atoms, ap, {}, hmax, 0, par - 1}, R{tr, atoms, ap, {}, hmax, 0, par - 1};
            std::exception_ptr err;  // an exception on the helper thread (bad_alloc) reaches the caller
            std::thread th([&] {
                try {
                    L.build(b, mid, depth + 1, bounded);
                } catch (...) {
                    err = std::current_exception();
                }
            });
            try {
                R.build(mid, e, depth + 1, bounded);
            } catch (...) {
                th.join();
                throw;
            }
            th.join();
            if (err) std::rethrow_exception(err);
            l = splice(L);
            r = splice(R);
        } else {
            l = build(b, mid, depth + 1, bounded);
            r = build(mid, e, depth + 1, bounded);
        }
        T.la[k] = l;
        T.lb[k] = r | (axis << 30);
        return k;
    }
};

bool boxes_nest(const FlatNode& p, const FlatNode& ch) {
    const float plo[3] = {p.boundsMin.x, p.boundsMin.y, p.boundsMin.z};
    const float phi[3] = {p.boundsMax.x, p.boundsMax.y, p.boundsMax.z};
    const float clo[3] = {ch.boundsMin.x, ch.boundsMin.y, ch.boundsMin.z};
    const float chi[3] = {ch.boundsMax.x, ch.boundsMax.y, ch.boundsMax.z};
    for (int a = 0; a < 3; ++a)
        if (!(plo[a] <= clo[a] && clo[a] <= phi[a] && plo[a] <= chi[a] && chi[a] <= phi[a])) return false;
    return true;
}

}  // namespace

// Builds out.st (accel.h, SceneTree) when the reference tree's boxes nest
// (out.st.wroot = -1 otherwise); st.max_stack <= cap sizes its LDS stack.
// Binary height bound of the scene tree (median splits below it).
constexpr int kSceneHeight = 40;

static thread_local double prof_t0 = 0;  // a rebuild thread may build beside another context
static void prof(const char* what) {
    static const bool on = std::getenv("RTA_BUILD_PROFILE") != nullptr;
    if (!on) return;
    const double t = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
    std::fprintf(stderr, "  %-28s %8.2f ms\n", what, t - prof_t0);
    prof_t0 = t;
}

static void build_scene_tree(const FlatShape* shapes, const FlatNode* nodes, int N, const int* idx,
                             const std::vector<char>& reach, const std::vector<int>& seq_base,
                             const std::vector<int>& scls, const std::vector<Box3>& sbox, int cap, AccelHost& out) {
    SceneTree& st = out.st;
    st = SceneTree();
    out.st_cone.clear();
    if (N <= 0 || N >= (1 << 28)) return;
    for (int k = 0; k < N; ++k) {
        const FlatNode& nd = nodes[k];
        if (!reach[k] || nd.leftChild == -1) continue;
        if (!boxes_nest(nd, nodes[nd.leftChild]) || !boxes_nest(nd, nodes[nd.rightChild])) return;
    }
    st.nested = 1;
    AccelHost T;
    T.mt = out.mt;  // the scene tree's cones follow the accelerator's triangle test
    std::vector<Atom> atoms;
    std::vector<std::pair<int, int>> ap;
    int par = 0;  // thread levels: 2^par halves at most in flight
    while ((2 << par) <= build_threads()) ++par;
    SceneBuilder sb{T, atoms, ap, {}, kSceneHeight, 0, par};
    std::vector<Atom> unb;
    const Box3 inf_box{{-INFINITY, -INFINITY, -INFINITY}, {INFINITY, INFINITY, INFINITY}};
    // An unbounded shape is tested only when the ray passes its reference leaf's
    // exact box; that box, padded like the shape bounds, contains every such
    // ray's slab interval (accel_math.h), though not necessarily the hit.
    auto leaf_pad = [&](const FlatNode& nd) {
        BoxAcc acc;
        for (int q = 0; q < 8; ++q)
            acc.add(D3{(q & 1) ? nd.boundsMax.x : nd.boundsMin.x, (q & 2) ? nd.boundsMax.y : nd.boundsMin.y,
                       (q & 4) ? nd.boundsMax.z : nd.boundsMin.z});
        Box3 b = finish(acc, out.origin_lim);
        for (int a = 0; a < 3; ++a)
            if (!(b.lo[a] <= b.hi[a])) return inf_box;  // NaN from infinite bounds: no bound at all
        return b;
    };
    // Atoms per reference leaf, in chunks of leaves on the build threads, each into its
    // own arrays (Atom::first relative to its own ap), then appended in leaf order: the
    // sequential pass's atoms and ap exactly.
    std::vector<int> rleaves;
    for (int k = 0; k < N; ++k)
        if (reach[k] && nodes[k].leftChild == -1) rleaves.push_back(k);
    struct Chunk {
        std::vector<Atom> bounded, unbounded;
        std::vector<std::pair<int, int>> ap;
    };
    std::vector<Chunk> chunks(static_cast<size_t>(std::max(1, build_threads())));
    parallel_chunks(static_cast<int>(rleaves.size()), 2048, [&](int q0, int q1, int c) {
        Chunk& C = chunks[c];
        // per-leaf scratch, reused (no allocation per leaf or per atom)
        std::vector<int> bnd;
        std::vector<std::pair<int, int>> ub, ps;
        for (int q = q0; q < q1; ++q) {
            const int k = rleaves[q];
            const FlatNode& nd = nodes[k];
            bnd.clear();
            ub.clear();
            for (int i = 0; i < std::max(0, nd.numShapes); ++i) {
                const int si = idx[nd.startShapeIdx + i];
                if (scls[si] == NEVER) continue;
                if (scls[si] == UNBOUNDED) ub.push_back({si, seq_base[k] + i});
                else bnd.push_back(i);
            }
            // an atom of n (shape, seq) pairs starting at p
            auto add = [&](std::vector<Atom>& dst, const std::pair<int, int>* p, int n, const Box3& box) {
                Atom at{k, static_cast<int>(C.ap.size()), n, box, {0.f, 0.f, 0.f}};
                for (int a = 0; a < 3; ++a) at.c[a] = std::isfinite(box.lo[a]) ? 0.5f * (box.lo[a] + box.hi[a]) : 0.f;
                C.ap.insert(C.ap.end(), p, p + n);
                dst.push_back(at);
            };
            if (bnd.size() <= static_cast<size_t>(kItemMax)) {
                if (!bnd.empty()) {
                    Box3 box = empty_box();
                    ps.clear();
                    for (int i : bnd) {
                        const int si = idx[nd.startShapeIdx + i];
                        grow(box, sbox[si]);
                        ps.push_back({si, seq_base[k] + i});
                    }
                    add(C.bounded, ps.data(), static_cast<int>(ps.size()), box);
                }
            } else {
                for (int i : bnd) {
                    const int si = idx[nd.startShapeIdx + i];
                    const std::pair<int, int> one{si, seq_base[k] + i};
                    add(C.bounded, &one, 1, sbox[si]);
                }
            }
            for (size_t q2 = 0; q2 < ub.size(); q2 += 4)
                add(C.unbounded, ub.data() + q2, static_cast<int>(std::min(ub.size(), q2 + 4) - q2), leaf_pad(nd));
        }
    });
    for (Chunk& C : chunks) {
        const int off = static_cast<int>(ap.size());
        for (Atom& at : C.bounded) at.first += off;
        for (Atom& at : C.unbounded) at.first += off;
        ap.insert(ap.end(), C.ap.begin(), C.ap.end());
        sb.atoms.insert(sb.atoms.end(), C.bounded.begin(), C.bounded.end());
        unb.insert(unb.end(), C.unbounded.begin(), C.unbounded.end());
    }
    const int nb = static_cast<int>(sb.atoms.size()), nu = static_cast<int>(unb.size());
    prof("  scene: atoms");
    if (nb + nu == 0) return;
    sb.atoms.insert(sb.atoms.end(), unb.begin(), unb.end());
    // bounded atoms under one SAH tree, unbounded ones under another whose
    // boxes carry no distance bound (kNoPrune: entered at parameter 0)
    int root, unb_root = -1;
    if (nb > 0 && nu > 0) {
        root = sb.inner(inf_box, 0, 0, 0);
        const int l = sb.build(0, nb, 1, true);
        unb_root = sb.build(nb, nb + nu, 1, true);
        T.la[root] = l;
        T.lb[root] = unb_root;
    } else {
        root = sb.build(0, nb + nu, 0, true);
        if (nu > 0) unb_root = root;
    }
    st.height = sb.height;
    prof("  scene: SAH build");
    build_cones(shapes, T);
    prof("  scene: cones");
    if (unb_root >= 0) {  // the unbounded subtree is built last: its nodes are [unb_root, end)
        for (size_t j = static_cast<size_t>(unb_root); j < T.lbox.size(); ++j) T.lcone[4 * j + 3] = kNoPrune;
    }
    // Full 4-wide collapse: the walks have no static stack bound on the scene
    // tree (a lane that runs out of entries walks the reference tree instead,
    // rt_kernels.hip lane_walk), so max_stack only sizes the LDS stack.
    int pend = 0;
    if (T.la[root] >= 0) {
        std::vector<int> memo(T.lbox.size(), -1);
        st.wroot = make_wide(T, root, 1 << 20, memo, pend);
    } else {
        st.wroot = 0;
        T.wchild.assign(kWide, -1);
        T.wsub.assign(kWide, -1);
        T.wpair.assign(1, 0);
        T.wchild[0] = root;
    }
    st.max_stack = std::min(pend + 2, cap);
    // merge: the scene tree's prims follow the local ones
    const int P0 = static_cast<int>(out.prim_shape.size());
    out.prim_shape.insert(out.prim_shape.end(), T.prim_shape.begin(), T.prim_shape.end());
    out.prim_seq.insert(out.prim_seq.end(), T.prim_seq.begin(), T.prim_seq.end());
    // T's arrays move into st (T ends here)
    st.box = std::move(T.lbox);
    st.a = std::move(T.la);
    st.b = std::move(T.lb);
    st.item_of.assign(st.box.size(), -1);
    for (size_t j = 0; j < st.box.size(); ++j) {
        if (st.a[j] >= 0) continue;
        const int start = -st.a[j] - 1 + P0;
        st.a[j] = -(start + 1);
        st.item_of[j] = static_cast<int>(st.item_ref.size());
        st.item_ref.push_back(sb.leaf_ref[j]);
        st.item_start.push_back(start);
        st.item_count.push_back(st.b[j]);
    }
    st.wchild = std::move(T.wchild);
    st.wsub = std::move(T.wsub);
    st.wpair = std::move(T.wpair);
    out.st_cone = std::move(T.lcone);
}

// Wide collapse of every local tree within the lane stack budget `cap`;
// returns the stack bound of the lane walk over them.
static int build_wide(AccelHost& A, const std::vector<int>& ref_depth, int cap) {
    A.wchild.clear();
    A.wsub.clear();
    A.wpair.clear();
    A.wroot.assign(A.local_root.size(), -1);
    std::vector<int> memo(A.lbox.size(), -1);
    int need = 0;
    for (size_t k = 0; k < A.local_root.size(); ++k) {
        const int r = A.local_root[k];
        if (r < 0 || A.la[r] < 0) continue;
        const int budget = std::max(cap - ref_depth[k] - 2, inner_height(A, r, memo));
        int pend = 0;
        A.wroot[k] = make_wide(A, r, budget, memo, pend);
        need = std::max(need, ref_depth[k] + pend + 2);
    }
    return need;
}

void parallel_for(int n, int min_per_thread, const std::function<void(int, int)>& fn) {
    parallel_chunks(n, min_per_thread, [&](int i0, int i1, int) { fn(i0, i1); });
}

bool build_accel(const FlatShape* shapes, int S, const FlatNode* nodes, int N, const int* idx, int I,
                 int leaf_threshold, int stack_cap, AccelHost& out, bool mt) {
    (void)I;
    prof_t0 = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
    out = AccelHost();
    out.mt = mt;
    out.content.assign(N, empty_box());
    out.flags.assign(N, 0);
    out.plain_start.assign(N, 0);
    out.plain_count.assign(N, 0);
    out.local_root.assign(N, -1);
    if (N == 0) return true;

    std::vector<Box3> sbox(S);
    std::vector<int> scls(S);
    // shapes classified independently, in chunks on the build threads (max is exact
    // in any order)
    std::vector<float> mag(build_threads(), 0.f);
    parallel_chunks(S, 4096, [&](int i0, int i1, int c) {
        float m = 0.f;  // one store per chunk: the threads' slots of `mag` share a cache line
        for (int i = i0; i < i1; ++i) {
            scls[i] = classify(shapes[i], sbox[i], 0.0, mt);
            if (scls[i] == BOUNDED)
                for (int a = 0; a < 3; ++a) m = std::max({m, std::fabs(sbox[i].lo[a]), std::fabs(sbox[i].hi[a])});
        }
        mag[c] = m;
    });
    for (float m : mag) out.scene_mag = std::max(out.scene_mag, m);
    out.origin_lim = static_cast<float>((mt ? kOriginRelMt : kOriginRel) * (out.scene_mag + 1.0));
    parallel_chunks(S, 4096, [&](int i0, int i1, int) {
        for (int i = i0; i < i1; ++i) scls[i] = classify(shapes[i], sbox[i], out.origin_lim, mt);
    });
    out.shape_cls = scls;
    out.shape_box = sbox;
    prof("classify");

    // Reference walk order (gpu_shader.comp:384-426: pop right first): the
    // rank of each leaf's shapes, and each node's depth (pending stack bound).
    std::vector<int> seq_base(N, -1), depth(N, 0);
    std::vector<char> reach(N, 0);
    {
        std::vector<std::pair<int, int>> st{{N - 1, 1}};
        int running = 0;
        while (!st.empty()) {
            auto [k, d] = st.back();
            st.pop_back();
            reach[k] = 1;
            depth[k] = std::max(depth[k], d);
            const FlatNode& nd = nodes[k];
            if (nd.leftChild == -1) {
                if (seq_base[k] < 0) {
                    seq_base[k] = running;
                    running += std::max(0, nd.numShapes);
                }
            } else {
                st.push_back({nd.leftChild, d + 1});
                st.push_back({nd.rightChild, d + 1});
            }
        }
    }

    // Leaves: always-tested prims and local BVHs. Each leaf is worked out on its own
    // (build threads, chunks of leaves), then appended in node order exactly as one
    // sequential pass would: plain prims first, then the local tree, its nodes and prims
    // renumbered by where they land (the same accelerator: tools/native/accel_time.cpp).
    struct LeafOut {
        Box3 content;
        int flags = 0, bounded = 0;
        std::vector<std::pair<int, int>> plain;  // (shape, seq)
        std::unique_ptr<AccelHost> loc;         // the local tree, numbered from 0 (root 0)
    };
    std::vector<int> leaves;
    for (int k = 0; k < N; ++k)
        if (reach[k] && nodes[k].leftChild == -1) leaves.push_back(k);
    std::vector<LeafOut> lo(leaves.size());
    std::vector<char> too_deep(build_threads(), 0);
    parallel_chunks(static_cast<int>(leaves.size()), 256, [&](int q0, int q1, int c) {
        std::vector<Item> bounded;  // per leaf, reused (moved out only into a local build)
        for (int q = q0; q < q1; ++q) {
            const int k = leaves[q];
            const FlatNode& nd = nodes[k];
            LeafOut& L = lo[q];
            bounded.clear();
            Box3 content = empty_box();
            bool unb = false;
            for (int i = 0; i < std::max(0, nd.numShapes); ++i) {
                const int si = idx[nd.startShapeIdx + i];
                const int seq = seq_base[k] + i;
                if (scls[si] == NEVER) continue;
                if (scls[si] == UNBOUNDED) {
                    L.plain.push_back({si, seq});
                    unb = true;
                    continue;
                }
                grow(content, sbox[si]);
                Item it{si, seq, sbox[si], {}};
                for (int a = 0; a < 3; ++a) it.c[a] = 0.5f * (sbox[si].lo[a] + sbox[si].hi[a]);
                double nn[3];
                if (mt && mt_normal(shapes[si], nn)) {
                    it.hn = true;
                    for (int a = 0; a < 3; ++a) it.n[a] = static_cast<float>(nn[a]);
                    MtTri mtt;
                    Box3 tb;
                    it.big = classify_mt_tight(shapes[si], tb, 0.0, mtt) == BOUNDED && mtt.X > kMtBigX;
                }
                bounded.push_back(it);
            }
            L.content = content;
            L.flags = (unb || mt) ? 0 : 8;  // MT boxes hold for non-grazing rays only: no content culling
            if (static_cast<int>(bounded.size()) <= leaf_threshold) {
                for (const Item& it : bounded) L.plain.push_back({it.shape, it.seq});
                std::sort(L.plain.begin(), L.plain.end(), [](auto& a, auto& b) { return a.second < b.second; });
                bounded.clear();
            }
            if (!bounded.empty()) {
                const int budget = stack_cap - depth[k] - 2;
                if (budget < 1) {
                    too_deep[c] = 1;
                    continue;
                }
                L.loc = std::make_unique<AccelHost>();
                L.loc->mt = mt;
                LocalBuilder lb{*L.loc, std::move(bounded)};
                lb.build(0, static_cast<int>(lb.items.size()), 0, budget);
                L.bounded = static_cast<int>(lb.items.size());
            }
        }
    });
    prof("leaf builds");
    for (char t : too_deep)
        if (t) return false;
    int max_stack = 1;
    for (size_t q = 0; q < leaves.size(); ++q) {
        const int k = leaves[q];
        LeafOut& L = lo[q];
        out.content[k] = L.content;
        out.flags[k] = L.flags;
        out.plain_start[k] = static_cast<int>(out.prim_shape.size());
        out.plain_count[k] = static_cast<int>(L.plain.size());
        for (auto [si, seq] : L.plain) {
            out.prim_shape.push_back(si);
            out.prim_seq.push_back(seq);
        }
        out.always_prims += static_cast<int>(L.plain.size());
        if (L.loc) {
            const AccelHost& o = *L.loc;
            const int off = static_cast<int>(out.lbox.size()), poff = static_cast<int>(out.prim_shape.size());
            out.lbox.insert(out.lbox.end(), o.lbox.begin(), o.lbox.end());
            for (size_t j2 = 0; j2 < o.la.size(); ++j2) {
                const int a = o.la[j2], b = o.lb[j2];
                if (a >= 0) {  // inner: left, right | axis << 30
                    out.la.push_back(a + off);
                    out.lb.push_back(((b & 0x3fffffff) + off) | (b & ~0x3fffffff));
                } else {  // leaf: -(start + 1), count
                    out.la.push_back(a - poff);
                    out.lb.push_back(b);
                }
            }
            out.prim_shape.insert(out.prim_shape.end(), o.prim_shape.begin(), o.prim_shape.end());
            out.prim_seq.insert(out.prim_seq.end(), o.prim_seq.begin(), o.prim_seq.end());
            out.local_leaves += o.local_leaves;
            out.local_root[k] = off;  // the local root is its tree's first node
            out.bounded_prims += L.bounded;
            L.loc.reset();
        }
        max_stack = std::max(max_stack, depth[k] + 1);
    }

    // Content boxes of inner nodes (children first) and the visit-order hint.
    std::vector<char> done(N, 0);
    std::function<void(int)> visit = [&](int k) {
        if (done[k]) return;
        done[k] = 1;
        const FlatNode& nd = nodes[k];
        if (nd.leftChild == -1) return;
        visit(nd.leftChild);
        visit(nd.rightChild);
        const int l = nd.leftChild, r = nd.rightChild;
        Box3 c = out.content[l];
        grow(c, out.content[r]);
        out.content[k] = c;
        const bool bounded = (out.flags[l] & 8) && (out.flags[r] & 8);
        int axis = 0;
        float best = -1.f;
        for (int a = 0; a < 3; ++a) {
            float dl = 0.5f * (out.content[l].lo[a] + out.content[l].hi[a]);
            float dr = 0.5f * (out.content[r].lo[a] + out.content[r].hi[a]);
            float g = std::fabs(dl - dr);
            if (std::isfinite(g) && g > best) {
                best = g;
                axis = a;
            }
        }
        float cl = 0.5f * (out.content[l].lo[axis] + out.content[l].hi[axis]);
        float crr = 0.5f * (out.content[r].lo[axis] + out.content[r].hi[axis]);
        const int swap = (std::isfinite(cl) && std::isfinite(crr) && cl > crr) ? 1 : 0;
        out.flags[k] = axis | (swap << 2) | (bounded ? 8 : 0);
    };
    prof("leaves");
    visit(N - 1);
    prof("content boxes");
    build_cones(shapes, out);
    prof("cones");
    max_stack = std::max(max_stack, build_wide(out, depth, kLaneStack));
    prof("wide");
    if (max_stack > stack_cap) return false;
    // MT: no scene tree. Its inner boxes bound hits, and an MT hit strays from its
    // triangle on grazing rays; the reference tree's exact boxes decide which leaves
    // are tested independently of the triangle test, so MT rays walk those (with the
    // grazing-cone local BVHs inside large leaves).
    if (!mt)
        build_scene_tree(shapes, nodes, N, idx, reach, seq_base, scls, sbox, std::min(stack_cap, kLaneStack), out);
    prof("scene tree");
    if (out.st.wroot >= 0) max_stack = std::max(max_stack, out.st.max_stack);
    out.max_stack = max_stack;
    return max_stack <= stack_cap;
}

}  // namespace rta

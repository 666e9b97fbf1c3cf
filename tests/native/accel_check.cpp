// accel_check.cpp — TEST HARNESS: scalar CPU emulation of k_accel's walk over
// the accelerator built by the product's accel.cpp, for checking the
// accelerator's exactness rules on CPU (tests/test_accel_cpu.py compares its
// closest-hit choice with the oracle's reference walk). Not product code.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../opengl-ray-tracer_amd/csrc/accel.h"
#include "../../opengl-ray-tracer_amd/csrc/accel_math.h"

namespace {
struct V { float x, y, z; };
V mk(float x, float y, float z) { return V{x, y, z}; }
V operator+(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
V operator-(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V operator*(float s, V a) { return {s * a.x, s * a.y, s * a.z}; }
float dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
V cross(V a, V b) { return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y}; }
V normalize(V a) { float s = 1.0f / std::sqrt(dot(a, a)); return {a.x * s, a.y * s, a.z * s}; }
float dist(V a, V b) { V d = b - a; return std::sqrt(dot(d, d)); }
float gmin(float a, float b) { return (b < a) ? b : a; }
float gmax(float a, float b) { return (a < b) ? b : a; }
V fv(rt_vec3 v) { return {v.x, v.y, v.z}; }

struct Best { float d; int seq; V p; int shape; };

bool g_mt = false;  // Moller-Trumbore triangles (out_info[6] = 1)
const bool g_slab = std::getenv("ACNOSLAB") == nullptr;
constexpr int kMtF = rta::kMtPadF;
float g_pad_scale = 1.0f;  // out_info[7] == 777: the MT per-ray padding switched off (the test's teeth)

// INNER hit of a shape, GLSL semantics (barycentric, or Moller-Trumbore when g_mt), or false.
bool isect(const FlatShape& s, V o, V d, V& p) {
    if (g_mt && s.type == 3) {  // gpu_shader.comp:170-195, the device's mt_hit operations
        V p1 = fv(s.triP1), e1 = fv(s.triP2) - p1, e2 = fv(s.triP3) - p1;
        V hh = cross(d, e2);
        float a = dot(e1, hh);
        if (std::fabs(a) < 1e-5f) return false;
        float fi = 1.0f / a;
        V sv = o - p1;
        float u = fi * dot(sv, hh);
        if (u < 0.0f || u > 1.0f) return false;
        V q = cross(sv, e1);
        float v = fi * dot(d, q);
        if (v < 0.0f || u + v > 1.0f) return false;
        float t = fi * dot(e2, q);
        if (!(t > 0.0f)) return false;
        p = o + t * d;
        return true;
    }
    if (s.type == 0) {
        V c = fv(s.sphereCenter), oc = o - c;
        float aa = dot(d, d), bb = 2.0f * dot(d, oc), cc = dot(oc, oc) - s.sphereRadius * s.sphereRadius;
        float D = bb * bb - 4.0f * aa * cc;
        if (!(D > 0.0f)) return false;
        float t1 = (-bb - std::sqrt(D)) / (2.0f * aa);
        if (!(t1 > 0.0f)) return false;
        p = o + t1 * d;
        return true;
    }
    if (s.type < 1 || s.type > 3) return false;
    V n = fv(s.planeNormal);
    float np = dot(n, d);
    if (np == 0.0f) return false;
    float t = -(s.planeD + dot(n, o)) / np;
    if (!(t > 0.0f) || !(np > 0.0f)) return false;
    p = o + t * d;
    if (s.type == 2) {
        V u = normalize(cross(n, mk(0, 1, 0)));
        if (std::sqrt(dot(u, u)) < 1e-5f) u = normalize(cross(n, mk(1, 0, 0)));
        V v = normalize(cross(n, u));
        V lp = p - fv(s.wallStart);
        float up = dot(lp, u), vp = dot(lp, v);
        if (up < 0.0f || up > s.wallWidth || vp < 0.0f || vp > s.wallHeight) return false;
    } else if (s.type == 3) {
        V p1 = fv(s.triP1), e1 = fv(s.triP2) - p1, e2 = fv(s.triP3) - p1, tp = p - p1;
        float d00 = dot(e1, e1), d01 = dot(e1, e2), d11 = dot(e2, e2), d20 = dot(tp, e1), d21 = dot(tp, e2);
        float den = d00 * d11 - d01 * d01;
        float v = (d11 * d20 - d01 * d21) / den, w = (d00 * d21 - d01 * d20) / den, u = 1.0f - v - w;
        if (u < 0.0f || v < 0.0f || w < 0.0f) return false;
    }
    return true;
}

bool ref_aabb(V o, V inv, const rt_vec3& lo, const rt_vec3& hi) {
    float tx0 = (lo.x - o.x) * inv.x, tx1 = (hi.x - o.x) * inv.x;
    float ty0 = (lo.y - o.y) * inv.y, ty1 = (hi.y - o.y) * inv.y;
    float tz0 = (lo.z - o.z) * inv.z, tz1 = (hi.z - o.z) * inv.z;
    float tmin = gmax(gmax(gmin(tx0, tx1), gmin(ty0, ty1)), gmin(tz0, tz1));
    float tmax = gmin(gmin(gmax(tx0, tx1), gmax(ty0, ty1)), gmax(tz0, tz1));
    return tmax >= tmin && tmax > 0.0f;
}

// The device walk's conservative tests (accel_math.h), same float operations.
bool padded(const rta::RayC& c, const rta::Box3& b, float l) {
    float te;
    return rta::box_enter(c, b.lo[0], b.lo[1], b.lo[2], b.hi[0], b.hi[1], b.hi[2], rta::t_limit(l, c.rdl), te);
}
}  // namespace

extern "C" {

// FNV-1a over every field of the accelerator built for the scene (0 if it cannot be
// built): equal hashes mean the same accelerator.
unsigned long long accel_hash(const FlatShape* shapes, int S, const FlatNode* nodes, int N, const int* idx, int I,
                              int mt) {
    rta::AccelHost A;
    if (!rta::build_accel(shapes, S, nodes, N, idx, I, 8, 64, A, mt != 0)) return 0;
    unsigned long long h = 1469598103934665603ull;
    auto bytes = [&](const void* p, size_t n) {
        const unsigned char* c = static_cast<const unsigned char*>(p);
        for (size_t i = 0; i < n; ++i) h = (h ^ c[i]) * 1099511628211ull;
    };
    auto v = [&](const auto& x) {
        const size_t n = x.size();
        bytes(&n, sizeof n);
        if (n) bytes(x.data(), n * sizeof(x[0]));
    };
    auto sc = [&](const auto& x) { bytes(&x, sizeof x); };
    v(A.prim_shape); v(A.prim_seq); v(A.content); v(A.flags); v(A.plain_start); v(A.plain_count);
    v(A.local_root); v(A.lbox); v(A.la); v(A.lb); v(A.lcone); v(A.wchild); v(A.wsub); v(A.wroot); v(A.wpair);
    sc(A.max_stack); sc(A.scene_mag); sc(A.origin_lim); sc(A.always_prims); sc(A.bounded_prims);
    sc(A.local_leaves);
    v(A.st.box); v(A.st.a); v(A.st.b); v(A.st.item_of); v(A.st.item_ref); v(A.st.item_start);
    v(A.st.item_count); v(A.st.wchild); v(A.st.wsub); v(A.st.wpair); sc(A.st.wroot); sc(A.st.max_stack); sc(A.st.height);
    sc(A.st.nested); v(A.st_cone); v(A.lmt); sc(A.mt_z);
    return h;
}

// For each ray (o[i], d[i]): the accelerated closest hit (shape index or -1)
// and the rays' shadow query against lim[i]. Returns -1 if the accelerator
// cannot be built for this tree. out_info[8] (in): 1 = rays take the scene
// tree where the device would; out: [9] scene tree built, [10] rays that took
// it, [11] the reference boxes nest.
int accel_check(const FlatShape* shapes, int S, const FlatNode* nodes, int N, const int* idx, int I,
                const float* o, const float* d, const float* lim, int R, int* out_shape, float* out_d,
                int* out_shadow, int* out_info) {
    rta::AccelHost A;
    g_mt = out_info[6] != 0;
    g_pad_scale = out_info[7] == 777 ? 0.0f : 1.0f;
    if (!rta::build_accel(shapes, S, nodes, N, idx, I, 8, 64, A, g_mt)) return -1;
    out_info[0] = static_cast<int>(A.lbox.size());
    out_info[1] = A.always_prims;
    out_info[2] = A.bounded_prims;
    out_info[3] = A.max_stack;
    const bool use_tree = out_info[8] != 0;
    bool boxes_finite = true;
    for (int k = 0; k < N; ++k)
        for (float v : {nodes[k].boundsMin.x, nodes[k].boundsMin.y, nodes[k].boundsMin.z, nodes[k].boundsMax.x,
                        nodes[k].boundsMax.y, nodes[k].boundsMax.z})
            if (std::isnan(v)) boxes_finite = false;
    constexpr int kSceneBase = 1 << 29;
    // ACSTAT: wide-node visits per depth below the local roots
    // children of the node whose first record is w: kWide, or 2 kWide for a pair (accel.h wpair)
    auto kids = [](const std::vector<char>& pair, int w) {
        return rta::kWide * (w < static_cast<int>(pair.size()) && pair[w] ? 2 : 1);
    };
    std::vector<int> wdepth(A.wchild.size() / rta::kWide, 0);
    for (size_t w = 0; w < wdepth.size(); ++w)
        for (int s2 = 0; s2 < kids(A.wpair, static_cast<int>(w)); ++s2)
            if (A.wsub[rta::kWide * w + s2] >= 0) wdepth[A.wsub[rta::kWide * w + s2]] = wdepth[w] + 1;
    long long per_depth[64] = {0}, forced_depth[64] = {0};
    long long tests = 0, scene_rays = 0, pops = 0, forced = 0;
    for (int r = 0; r < R; ++r) {
        long long nodes_before = 0;
        V ro = mk(o[3 * r], o[3 * r + 1], o[3 * r + 2]), rd = mk(d[3 * r], d[3 * r + 1], d[3 * r + 2]);
        V inv = mk(1.0f / rd.x, 1.0f / rd.y, 1.0f / rd.z);
        rta::RayC rc = rta::ray_consts(ro.x, ro.y, ro.z, rd.x, rd.y, rd.z, A.origin_lim);
        rta::mt_ray(rc, ro.x, ro.y, ro.z, A.mt_z);  // the device's MT ray terms
        const float so = rc.so, on = rc.on;
        for (int pass = 0; pass < 2; ++pass) {
            const bool shadow = pass == 1;
            Best b{1e20f, 0x7fffffff, mk(0, 0, 0), -1};
            bool hit_shadow = false;
            std::vector<int> st;
            // Scene tree (accel.h, SceneTree): taken by the rays the device sends
            // there (rt_kernels.hip, use_scene) when out_info[8] asks for it.
            const bool fast = boxes_finite && std::fabs(ro.x) < 3.0e38f && std::fabs(ro.y) < 3.0e38f &&
                              std::fabs(ro.z) < 3.0e38f && std::fabs(inv.x) < 3.0e38f &&
                              std::fabs(inv.y) < 3.0e38f && std::fabs(inv.z) < 3.0e38f && inv.x != 0.0f &&
                              inv.y != 0.0f && inv.z != 0.0f;
            const bool scene = use_tree && A.st.wroot >= 0 && fast && rc.ix != 0.0f;
            if (scene) ++scene_rays;
            if (scene) st.push_back(-(A.st.wroot + 1) - kSceneBase);
            else if (N > 0) st.push_back(N - 1);
            while (!st.empty() && !(shadow && hit_shadow)) {
                int code = st.back();
                st.pop_back();
                const float l = shadow ? lim[r] : b.d;
                auto scan = [&](int start, int cnt) {
                    for (int i = 0; i < cnt && !(shadow && hit_shadow); ++i) {
                        const int si = A.prim_shape[start + i], seq = A.prim_seq[start + i];
                        V p;
                        ++tests;
                        if (!isect(shapes[si], ro, rd, p)) continue;
                        float dd = dist(ro, p);
                        if (shadow) {
                            if (dd < lim[r]) hit_shadow = true;
                        } else if (dd < b.d || (dd == b.d && seq < b.seq)) {
                            b = Best{dd, seq, p, si};
                        }
                    }
                };
                if (std::getenv("ACDBG")) std::printf("pop %d lim %g best %d %g\n", code, l, b.shape, b.d);
                ++nodes_before;
                ++pops;
                if (code <= -kSceneBase) {
                    // scene-tree wide node: padded boxes and cones; an item tests its
                    // reference leaf's exact box before its shapes
                    const int w = -(code + kSceneBase) - 1;
                    for (int s2 = 0; s2 < kids(A.st.wpair, w); ++s2) {
                        const int j = A.st.wchild[rta::kWide * w + s2];
                        if (j < 0) continue;
                        const float* k = &A.st_cone[4 * j];
                        // (MT accelerators build no scene tree)
                        if (!padded(rc, A.st.box[j], k[3] <= rta::kNoPrune ? INFINITY : l)) continue;
                        if (rta::cone_culls_q(rta::cone_word(k[0], k[1], k[2], k[3]), rc.dq)) continue;  // the device's quantized cone
                        const int sub = A.st.wsub[rta::kWide * w + s2];
                        if (sub >= 0) {
                            st.push_back(-(sub + 1) - kSceneBase);
                            continue;
                        }
                        const int it = A.st.item_of[j];
                        const FlatNode& rl = nodes[A.st.item_ref[it]];
                        if (ref_aabb(ro, inv, rl.boundsMin, rl.boundsMax)) scan(A.st.item_start[it], A.st.item_count[it]);
                    }
                } else if (code >= 0) {
                    const FlatNode& nd = nodes[code];
                    if (!ref_aabb(ro, inv, nd.boundsMin, nd.boundsMax)) continue;
                    if ((A.flags[code] & 8) && !padded(rc, A.content[code], l)) continue;
                    if (nd.leftChild == -1) {
                        scan(A.plain_start[code], A.plain_count[code]);
                        const int lr = A.local_root[code];
                        if (lr >= 0 && A.wroot[code] >= 0) st.push_back(-(A.wroot[code] + 1));  // wide root
                        else if (lr >= 0 && (g_mt || padded(rc, A.lbox[lr], l))) scan(-A.la[lr] - 1, A.lb[lr]);
                    } else {
                        st.push_back(nd.leftChild);
                        st.push_back(nd.rightChild);
                    }
                } else {
                    // wide local node (accel.h, build_wide): each child's padded
                    // box and back-face cone, tested at the wide node
                    const int w = -code - 1;
                    ++per_depth[std::min(63, wdepth[w])];
                    for (int s2 = 0; s2 < kids(A.wpair, w); ++s2) {
                        const int j = A.wchild[rta::kWide * w + s2];
                        if (j < 0) continue;
                        const float* k = &A.lcone[4 * j];
                        if (g_mt) {
                            float pad, lf, q2, pt;
                            if (rta::mt_pad(rc, so, k, &A.lmt[kMtF * j], pad, lf, q2, pt)) {
                                if (g_pad_scale != 1.0f) {  // mutation check only (out_info[7] = 777)
                                    pad *= g_pad_scale, q2 *= g_pad_scale, pt *= g_pad_scale;
                                    lf = 1.0f;
                                }
                                rta::Box3 b = A.lbox[j];
                                for (int a = 0; a < 3; ++a) {
                                    b.lo[a] -= pad;
                                    b.hi[a] += pad;
                                }
                                float tn, tf;
                                if (!rta::box_span(rc, b.lo[0], b.lo[1], b.lo[2], b.hi[0], b.hi[1], b.hi[2],
                                                   rta::t_limit(l * lf, rc.rdl), tn, tf))
                                    continue;
                                if (g_slab && rc.ix != 0.0f && A.lmt[kMtF * j + 5] < 3e38f && !rta::mt_slab(ro.x, ro.y, ro.z, on, rc, k, &A.lmt[kMtF * j], q2, pt, tn, tf)) continue;
                            } else {
                                ++forced;
                                ++forced_depth[std::min(63, wdepth[w])];
                            }
                        } else {
                            if (!padded(rc, A.lbox[j], l)) continue;
                            if (rta::cone_culls_q(rta::cone_word(k[0], k[1], k[2], k[3]), rc.dq)) continue;  // the device's quantized cone
                        }
                        if (A.la[j] < 0) scan(-A.la[j] - 1, A.lb[j]);
                        else st.push_back(-(A.wsub[rta::kWide * w + s2] + 1));
                    }
                }
            }
            if (shadow) out_shadow[r] = hit_shadow ? 1 : 0;
            else { out_shape[r] = b.shape; out_d[r] = b.d; }
            if (out_info[7] == 12345 && pass == (lim[r] < 1e19f ? 1 : 0)) out_shape[r] = static_cast<int>(nodes_before);
        }
    }
    out_info[4] = static_cast<int>(tests / (R > 0 ? R : 1));
    out_info[5] = static_cast<int>(pops / (R > 0 ? R : 1));
    if (std::getenv("ACSTAT"))
        for (int k = 0; k < 64; ++k)
            if (per_depth[k]) std::printf("depth %d: %.2f visits/ray %.2f forced\n", k, double(per_depth[k]) / R, double(forced_depth[k]) / R);
    if (std::getenv("ACSTAT")) std::printf("pops/ray %.1f forced/ray %.2f tests/ray %.1f\n", double(pops) / R, double(forced) / R, double(tests) / R);
    out_info[9] = A.st.wroot >= 0 ? 1 : 0;
    out_info[10] = static_cast<int>(scene_rays);
    out_info[11] = A.st.nested;
    return 0;
}
}

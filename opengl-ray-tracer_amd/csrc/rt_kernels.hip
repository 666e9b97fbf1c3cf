// rt_kernels.hip — the MI355X (gfx950) render kernels and the C ABI of
// include/rt_api.h (librtamd.so).
//
// Kernels
//   k_pack_shapes / k_pack_nodes : AoS FlatShape/FlatNode (the reference's SSBO
//       records) -> the HBM layout of rt_device.h (run once per upload).
//   k_lane<STATS>   : one ray per lane walking the reference's own traversal
//       (stack in LDS, right child first, closest-hit shadow rays). It is the
//       literal restatement of gpu_shader.comp and, with STATS, counts the work
//       that shader performs (node loads, primitive tests, material fetches).
//   k_packet        : the production kernel. A wave64 renders an 8x8 pixel tile
//       as one packet: the tree walk order of gpu_shader.comp:384-426 does not
//       depend on the ray, so the wave walks it once with a 64-bit active mask
//       per stack entry (the stack lives in the wave's VGPR lanes: entry j in
//       lane j, readlane/writelane), node and shape records are wave-uniform
//       scalar loads, and each lane keeps exactly the state, order and
//       tie-breaking of its own reference walk. Shadow rays stop per lane at the
//       first occluder closer than the light (equivalent to the reference's
//       closest-hit test).
//
// Launch geometry: 256-thread blocks = 4 waves side by side = 32 x 8 pixels;
// grid = ceil(W/32) x ceil(rows/8). Every kernel is compiled with
// -ffp-contract=off (Makefile) so its float sequence is the oracle's.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <limits>
#include <atomic>
#include <memory>
#include <new>
#include <thread>
#include <vector>

#include "../../include/rt_api.h"
#include "accel.h"
#include "accel_math.h"
#include "lbvh.h"
#include "rt_device.h"
#include "group_wait.h"
#include "rt_internal.h"

using namespace rtd;

namespace {

constexpr int kBlock = 256;
constexpr int kTileW = 32;  // pixels per block row (4 waves x 8)
constexpr int kTileH = 8;
constexpr int kMaxStack = 64;  // gpu_shader.comp:384
constexpr int kRing = 1024;
constexpr int kLeafScan = 8;   // leaves with more shapes get a local BVH (accel.h)    // dispatch timings kept between rt_kernel_times calls

// Stats slots, in rt_stats field order.
enum {
    ST_PIXELS = 0, ST_CLOSEST, ST_SHADOW, ST_NODES,
    ST_BVH0, ST_BVH1, ST_BVH2, ST_BVH3,
    ST_BR0, ST_BR1, ST_BR2, ST_BR3,
    ST_UPD, ST_HITS, ST_COUNT
};

// ---------------------------------------------------------------------------
// Pack kernels

// The ray-independent part of a shape's intersection record (GeoRec).
__device__ GeoRec pack_geo(const FlatShape& s, int si) {
    GeoRec g;
    for (int k = 0; k < 18; ++k) g.f[k] = 0.f;
    g.type = s.type;
    g.idx = si;
    if (s.type == RT_SPHERE) {
        g.f[0] = s.sphereCenter.x; g.f[1] = s.sphereCenter.y; g.f[2] = s.sphereCenter.z;
        g.f[3] = s.sphereRadius;
    } else {
        V n = mk(s.planeNormal.x, s.planeNormal.y, s.planeNormal.z);
        g.f[0] = n.x; g.f[1] = n.y; g.f[2] = n.z; g.f[3] = s.planeD;
        if (s.type == RT_WALL) {
            g.f[4] = s.wallStart.x; g.f[5] = s.wallStart.y; g.f[6] = s.wallStart.z;
            g.f[7] = s.wallWidth; g.f[8] = s.wallHeight;
            // gpu_shader.comp:305-307, a function of the normal only.
            V u = normalize(cross(n, mk(0.f, 1.f, 0.f)));
            if (len(u) < 1e-5f) u = normalize(cross(n, mk(1.f, 0.f, 0.f)));
            V v = normalize(cross(n, u));
            g.f[9] = u.x; g.f[10] = u.y; g.f[11] = u.z;
            g.f[12] = v.x; g.f[13] = v.y; g.f[14] = v.z;
        } else if (s.type == RT_TRIANGLE) {
            V p1 = mk(s.triP1.x, s.triP1.y, s.triP1.z);
            V e1 = mk(s.triP2.x, s.triP2.y, s.triP2.z) - p1;
            V e2 = mk(s.triP3.x, s.triP3.y, s.triP3.z) - p1;
            // gpu_shader.comp:218-229, ray-independent part.
            float d00 = dot(e1, e1), d01 = dot(e1, e2), d11 = dot(e2, e2);
            g.f[4] = p1.x; g.f[5] = p1.y; g.f[6] = p1.z;
            g.f[7] = e1.x; g.f[8] = e1.y; g.f[9] = e1.z;
            g.f[10] = e2.x; g.f[11] = e2.y; g.f[12] = e2.z;
            g.f[13] = d00; g.f[14] = d01; g.f[15] = d11;
            g.f[16] = d00 * d11 - d01 * d01;
        }
    }
    return g;
}

__device__ __forceinline__ void store_geo(float4* out, const GeoRec& g) {
    const float4* in = reinterpret_cast<const float4*>(&g);
    for (int k = 0; k < 5; ++k) out[k] = in[k];
}

// PrimRec (rt_device.h) of a shape's GeoRec and its rank in the reference walk.
__device__ __forceinline__ PrimRec pack_prim(const GeoRec& g, int seq) {
    PrimRec p;
    for (int k = 0; k < 15; ++k) p.f[k] = g.f[k];
    int type = g.type;
    if (type == 3) {
        p.f[13] = g.f[14];  // d01
        p.f[14] = g.f[16];  // d00 * d11 - d01 * d01
    } else if (type < 0 || type > 3) {  // no INNER hit (get_intersection: NONE)
        type = 1;
        p.f[0] = p.f[1] = p.f[2] = __int_as_float(0x7fc00000);
    }
    p.st = (seq << 2) | type;
    return p;
}

__device__ __forceinline__ void store_prim(float4* prims, int j, const PrimRec& p) {
    const float4* in = reinterpret_cast<const float4*>(&p);
    float4* out = prims + 4 * static_cast<size_t>(j);
    for (int k = 0; k < 4; ++k) out[k] = in[k];
}

__device__ __forceinline__ void store_mat(float4* mat, int j, const FlatMaterial& m) {
    mat[2 * j] = make_float4(m.color.x, m.color.y, m.color.z, m.fresnelStrength);
    mat[2 * j + 1] =
        make_float4(m.ambientStrength, m.diffuseStrength, m.specularStrength, static_cast<float>(m.shininess));
}

__global__ void k_pack_shapes(const FlatShape* __restrict__ src, int S, const int* __restrict__ idx, int I,
                              float4* __restrict__ geo_lin, float4* __restrict__ geo_leaf,
                              float4* __restrict__ mat) {
    int j = blockIdx.x * blockDim.x + threadIdx.x;
    int total = S + I;
    if (j >= total) return;
    const bool leaf_slot = j >= S;
    const int si = leaf_slot ? idx[j - S] : j;
    const FlatShape& s = src[si];
    const GeoRec g = pack_geo(s, si);
    store_geo(leaf_slot ? geo_leaf + 5 * static_cast<size_t>(j - S) : geo_lin + 5 * static_cast<size_t>(j), g);
    if (!leaf_slot) store_mat(mat, j, s.material);
}

__global__ void k_pack_nodes(const FlatNode* __restrict__ src, int N, float4* __restrict__ nodes) {
    int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= N) return;
    const FlatNode& n = src[k];
    int a, b;
    if (n.leftChild == -1) {
        a = -(n.startShapeIdx + 1);
        b = n.numShapes;
    } else {
        a = n.leftChild;
        b = n.rightChild;
    }
    nodes[2 * k] = make_float4(n.boundsMin.x, n.boundsMin.y, n.boundsMin.z, __int_as_float(a));
    nodes[2 * k + 1] = make_float4(n.boundsMax.x, n.boundsMax.y, n.boundsMax.z, __int_as_float(b));
}

// ---------------------------------------------------------------------------
// Shared per-pixel plumbing

struct PixelCoord {
    int x, r, y;
    bool active;
};

__device__ __forceinline__ PixelCoord pixel_of(const KParams& kp) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    PixelCoord pc;
    pc.x = blockIdx.x * kTileW + wave * 8 + (lane & 7);
    pc.r = blockIdx.y * kTileH + (lane >> 3);
    pc.active = pc.x < kp.width && pc.r < kp.out_rows;
    pc.y = pc.active ? image_row(kp, pc.r) : 0;
    pc.active = pc.active && pc.y < kp.height;
    return pc;
}

// Background gradient (gpu_shader.comp:436).
__device__ __forceinline__ V background(const KParams& kp, int y) {
    return mix(mk(0.05f, 0.07f, 0.1f), mk(0.5f, 0.7f, 1.0f), static_cast<float>(y) / kp.resY);
}

__device__ __forceinline__ Ray primary_ray(const KParams& kp, int x, int y) {
    return get_ray(kp, 2.0f * static_cast<float>(x) / kp.resX - 1.0f, 1.0f - 2.0f * static_cast<float>(y) / kp.resY);
}

struct Counters {
    unsigned c[ST_COUNT];
};

// Lighting of one bounce (gpu_shader.comp:482-516): adds to acc/att and
// updates the ray; returns true if the path continues.
__device__ __forceinline__ bool shade_bounce(const KParams& kp, Ray& ray, V hp, V hn, const Mat& m, bool shadow,
                                             V& acc, V& att, float offset_reflect) {
    V pc = phong(hp, hn, ray.d, kp.light_pos, kp.light_color, m);
    if (shadow) pc = pc * 0.3f;
    acc = acc + mulv(att, pc);
    if (m.specular > 0.0f) {
        V rd = reflect(ray.d, hn);
        ray.o = hp + hn * offset_reflect;
        ray.d = rd;
        if (kp.useFresnel) {
            float fr = powf(1.0f - gmax(dot(-ray.d, hn), 0.0f), 5.0f);
            fr = gmin(gmax(fr, 0.0f), 0.8f);
            float rw = m.fresnel * fr;
            float mw = 1.0f - rw;
            att = mulv(att, mix(m.color, mk(1.f, 1.f, 1.f), rw));
            acc = acc + mulv(mw * m.color, pc);
        } else {
            att = att * m.specular;
        }
        return true;
    }
    return false;
}

// ---------------------------------------------------------------------------
// k_lane: the reference walk, one ray per lane.

struct LaneHit {
    bool found;
    float d;
    V p;
    int slot;
};

template <bool STATS>
__device__ LaneHit lane_closest_bvh(const KParams& kp, const float4* __restrict__ nodes,
                                    const float4* __restrict__ geo, Ray r, int* stk, Counters& c) {
    LaneHit res{false, 1e20f, mk(0.f, 0.f, 0.f), -1};
    if (kp.N <= 0) return res;
    const V inv = inv_dir(r.d);
    int sp = 0;
    stk[0] = kp.N - 1;
    sp = 1;
    while (sp > 0) {
        --sp;
        const int k = stk[sp * kBlock];
        const float4 a = nodes[2 * k], b = nodes[2 * k + 1];
        if (STATS) c.c[ST_NODES]++;
        if (!ray_aabb(r.o, inv, mk(a.x, a.y, a.z), mk(b.x, b.y, b.z))) continue;
        const int ia = __float_as_int(a.w), ib = __float_as_int(b.w);
        if (ia < 0) {
            const int start = -ia - 1;
            for (int i = 0; i < ib; ++i) {
                const GeoRec g = load_rec(geo, start + i);
                if (STATS && g.type >= 0 && g.type < 4) c.c[ST_BVH0 + g.type]++;
                const Hit h = intersect(g, r, kp.useMT);
                if (h.type == INNER) {
                    const float d = dist(r.o, h.p);
                    if (d < res.d) {
                        res = LaneHit{true, d, h.p, start + i};
                        if (STATS) c.c[ST_UPD]++;
                    }
                }
            }
        } else {
            if (sp + 2 > kp.max_stack) return LaneHit{false, 1e20f, mk(0.f, 0.f, 0.f), -1};
            stk[sp * kBlock] = ia;
            stk[(sp + 1) * kBlock] = ib;
            sp += 2;
        }
    }
    return res;
}

template <bool STATS>
__device__ LaneHit lane_closest_brute(const KParams& kp, const float4* __restrict__ geo, Ray r, Counters& c) {
    LaneHit res{false, 1e20f, mk(0.f, 0.f, 0.f), -1};
    for (int i = 0; i < kp.S; ++i) {
        const GeoRec g = load_rec(geo, i);
        if (STATS && g.type >= 0 && g.type < 4) c.c[ST_BR0 + g.type]++;
        const Hit h = intersect(g, r, kp.useMT);
        if (h.type == INNER) {
            const float d = dist(r.o, h.p);
            if (d < res.d) {
                res = LaneHit{true, d, h.p, i};
                if (STATS) c.c[ST_UPD]++;
            }
        }
    }
    return res;
}

// Brute-force shadow loop (gpu_shader.comp:569-580): stops at the first
// INNER hit nearer than the light.
template <bool STATS>
__device__ bool lane_shadow_brute(const KParams& kp, const float4* __restrict__ geo, Ray sr, float ld, Counters& c) {
    for (int i = 0; i < kp.S; ++i) {
        const GeoRec g = load_rec(geo, i);
        if (STATS && g.type >= 0 && g.type < 4) c.c[ST_BR0 + g.type]++;
        const Hit h = intersect(g, sr, kp.useMT);
        if (h.type == INNER && dist(sr.o, h.p) < ld) return true;
    }
    return false;
}

template <bool STATS>
__global__ __launch_bounds__(kBlock) void k_lane(const float4* __restrict__ geo_leaf,
                                                 const float4* __restrict__ geo_lin,
                                                 const float4* __restrict__ mat,
                                                 const float4* __restrict__ nodes, KParams kp) {
    extern __shared__ int lds_stack[];
    int* stk = lds_stack + threadIdx.x;  // entry s of this lane at stk[s * kBlock]
    const PixelCoord pc = pixel_of(kp);
    Counters c;
    if (STATS)
        for (int i = 0; i < ST_COUNT; ++i) c.c[i] = 0;
    if (pc.active) {
        const V bg = background(kp, pc.y);
        Ray ray = primary_ray(kp, pc.x, pc.y);
        V acc = mk(0.f, 0.f, 0.f), att = mk(1.f, 1.f, 1.f);
        if (STATS) c.c[ST_PIXELS]++;
        const float shadow_off = kp.useBVH ? 1e-3f : 1e-5f;  // :469 vs :565
        for (int depth = 0; depth < kp.maxBounces; ++depth) {
            if (STATS) c.c[ST_CLOSEST]++;
            LaneHit hit = kp.useBVH ? lane_closest_bvh<STATS>(kp, nodes, geo_leaf, ray, stk, c)
                                    : lane_closest_brute<STATS>(kp, geo_lin, ray, c);
            if (!hit.found) {
                acc = acc + mulv(att, bg);
                break;
            }
            if (STATS) c.c[ST_HITS]++;
            const GeoRec g = load_rec(kp.useBVH ? geo_leaf : geo_lin, hit.slot);
            const V hn = shape_normal(g, hit.p);
            const Mat m = load_mat(mat, g.idx);
            Ray sr{hit.p + hn * shadow_off, normalize(kp.light_pos - hit.p)};
            const float ld = dist(kp.light_pos, hit.p);
            bool shadow;
            if (STATS) c.c[ST_SHADOW]++;
            if (kp.useBVH) {
                // Full closest-hit walk, as gpu_shader.comp:473-480.
                LaneHit sh = lane_closest_bvh<STATS>(kp, nodes, geo_leaf, sr, stk, c);
                shadow = sh.found && sh.d < ld;
            } else {
                shadow = lane_shadow_brute<STATS>(kp, geo_lin, sr, ld, c);
            }
            if (!shade_bounce(kp, ray, hit.p, hn, m, shadow, acc, att, 1e-3f)) break;
        }
        store_px(kp, pc.r, pc.x, make_float4(acc.x, acc.y, acc.z, 1.0f));
    }
    if (STATS) {
        for (int i = 0; i < ST_COUNT; ++i) {
            unsigned long long v = c.c[i];
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
            if ((threadIdx.x & 63) == 0 && v) atomicAdd(kp.stats + i, v);
        }
    }
}

// ---------------------------------------------------------------------------
// k_packet: the wave64 packet walk.

__device__ __forceinline__ int lane_id() { return __lane_id(); }
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Wave-uniform stack of (node, 64-bit mask) held in three VGPRs: entry j in lane j.
struct WaveStack {
    int node, lo, hi;
    int sp;  // uniform
    __device__ __forceinline__ void push(int k, unsigned long long m) {
        const bool mine = lane_id() == sp;  // v_writelane equivalent
        node = mine ? k : node;
        lo = mine ? static_cast<int>(m & 0xffffffffu) : lo;
        hi = mine ? static_cast<int>(m >> 32) : hi;
        ++sp;
    }
    __device__ __forceinline__ void pop(int& k, unsigned long long& m) {
        --sp;
        k = __builtin_amdgcn_readlane(node, sp);
        const unsigned l = static_cast<unsigned>(__builtin_amdgcn_readlane(lo, sp));
        const unsigned h = static_cast<unsigned>(__builtin_amdgcn_readlane(hi, sp));
        m = (static_cast<unsigned long long>(h) << 32) | l;
    }
};

__device__ __forceinline__ bool lane_in(unsigned long long m) { return (m >> lane_id()) & 1ull; }

// Closest hit for every lane in `active` (reference walk order per lane).
__device__ LaneHit packet_closest_bvh(const KParams& kp, const float4* __restrict__ nodes,
                                      const float4* __restrict__ geo, const Ray& r, bool active) {
    LaneHit res{false, 1e20f, mk(0.f, 0.f, 0.f), -1};
    const unsigned long long m0 = __ballot(active);
    if (kp.N <= 0 || m0 == 0) return res;
    const V inv = inv_dir(r.d);
    WaveStack st{0, 0, 0, 0};
    st.push(kp.N - 1, m0);
    while (st.sp > 0) {
        int k;
        unsigned long long m;
        st.pop(k, m);
        k = uni(k);
        const float4 a = nodes[2 * k], b = nodes[2 * k + 1];
        const bool hb = lane_in(m) && ray_aabb(r.o, inv, mk(a.x, a.y, a.z), mk(b.x, b.y, b.z));
        const unsigned long long mh = __ballot(hb);
        if (mh == 0) continue;
        const int ia = uni(__float_as_int(a.w)), ib = uni(__float_as_int(b.w));
        if (ia < 0) {
            const int start = -ia - 1;
            for (int i = 0; i < ib; ++i) {
                const GeoRec g = load_rec(geo, start + i);
                if (hb) {
                    const Hit h = intersect(g, r, kp.useMT);
                    if (h.type == INNER) {
                        const float d = dist(r.o, h.p);
                        if (d < res.d) res = LaneHit{true, d, h.p, start + i};
                    }
                }
            }
        } else {
            if (st.sp + 2 > kMaxStack) {
                // Unreachable: the host rejects trees deeper than the stack.
                return LaneHit{false, 1e20f, mk(0.f, 0.f, 0.f), -1};
            }
            st.push(ia, mh);
            st.push(ib, mh);
        }
    }
    return res;
}

// Shadow query: true iff the lane's reference closest-hit shadow walk would
// find a hit nearer than `ld` (and than the 1e20 start value). Lanes retire at
// their first such hit.
__device__ bool packet_shadow_bvh(const KParams& kp, const float4* __restrict__ nodes,
                                  const float4* __restrict__ geo, const Ray& r, float ld, bool active) {
    bool shadow = false;
    const unsigned long long m0 = __ballot(active);
    if (kp.N <= 0 || m0 == 0) return false;
    const float lim = gmin(ld, 1e20f);
    const V inv = inv_dir(r.d);
    WaveStack st{0, 0, 0, 0};
    st.push(kp.N - 1, m0);
    unsigned long long done = 0;
    while (st.sp > 0) {
        int k;
        unsigned long long m;
        st.pop(k, m);
        m &= ~done;
        if (m == 0) continue;
        k = uni(k);
        const float4 a = nodes[2 * k], b = nodes[2 * k + 1];
        const bool hb = lane_in(m) && ray_aabb(r.o, inv, mk(a.x, a.y, a.z), mk(b.x, b.y, b.z));
        const unsigned long long mh = __ballot(hb);
        if (mh == 0) continue;
        const int ia = uni(__float_as_int(a.w)), ib = uni(__float_as_int(b.w));
        if (ia < 0) {
            const int start = -ia - 1;
            bool live = hb;
            for (int i = 0; i < ib; ++i) {
                const GeoRec g = load_rec(geo, start + i);
                if (live) {
                    const Hit h = intersect(g, r, kp.useMT);
                    if (h.type == INNER && dist(r.o, h.p) < lim) {
                        shadow = true;
                        live = false;
                    }
                }
                if (__ballot(live) == 0) break;
            }
            done = __ballot(shadow);
            if ((m0 & ~done) == 0) break;
        } else {
            if (st.sp + 2 > kMaxStack) return shadow;
            st.push(ia, mh);
            st.push(ib, mh);
        }
    }
    return shadow;
}

__device__ LaneHit packet_closest_brute(const KParams& kp, const float4* __restrict__ geo, const Ray& r,
                                        bool active) {
    LaneHit res{false, 1e20f, mk(0.f, 0.f, 0.f), -1};
    if (__ballot(active) == 0) return res;
    for (int i = 0; i < kp.S; ++i) {
        const GeoRec g = load_rec(geo, i);
        if (active) {
            const Hit h = intersect(g, r, kp.useMT);
            if (h.type == INNER) {
                const float d = dist(r.o, h.p);
                if (d < res.d) res = LaneHit{true, d, h.p, i};
            }
        }
    }
    return res;
}

__device__ bool packet_shadow_brute(const KParams& kp, const float4* __restrict__ geo, const Ray& r, float ld,
                                    bool active) {
    bool live = active, shadow = false;
    if (__ballot(live) == 0) return false;
    for (int i = 0; i < kp.S; ++i) {
        const GeoRec g = load_rec(geo, i);
        if (live) {
            const Hit h = intersect(g, r, kp.useMT);
            if (h.type == INNER && dist(r.o, h.p) < ld) {
                shadow = true;
                live = false;
            }
        }
        if (__ballot(live) == 0) break;
    }
    return shadow;
}

__global__ __launch_bounds__(kBlock) void k_packet(const float4* __restrict__ geo_leaf,
                                                   const float4* __restrict__ geo_lin,
                                                   const float4* __restrict__ mat,
                                                   const float4* __restrict__ nodes, KParams kp) {
    const PixelCoord pc = pixel_of(kp);
    const V bg = background(kp, pc.y);
    Ray ray = primary_ray(kp, pc.x, pc.y);
    V acc = mk(0.f, 0.f, 0.f), att = mk(1.f, 1.f, 1.f);
    bool alive = pc.active;
    const float shadow_off = kp.useBVH ? 1e-3f : 1e-5f;
    for (int depth = 0; depth < kp.maxBounces; ++depth) {
        if (__ballot(alive) == 0) break;
        LaneHit hit = kp.useBVH ? packet_closest_bvh(kp, nodes, geo_leaf, ray, alive)
                                : packet_closest_brute(kp, geo_lin, ray, alive);
        if (alive && !hit.found) {
            acc = acc + mulv(att, bg);
            alive = false;
        }
        V hn = mk(0.f, 0.f, 0.f);
        Mat m{};
        Ray sr{mk(0.f, 0.f, 0.f), mk(0.f, 0.f, 1.f)};
        float ld = 0.f;
        if (alive) {
            const GeoRec g = load_rec(kp.useBVH ? geo_leaf : geo_lin, hit.slot);
            hn = shape_normal(g, hit.p);
            m = load_mat(mat, g.idx);
            sr = Ray{hit.p + hn * shadow_off, normalize(kp.light_pos - hit.p)};
            ld = dist(kp.light_pos, hit.p);
        }
        const bool shadow = kp.useBVH ? packet_shadow_bvh(kp, nodes, geo_leaf, sr, ld, alive)
                                      : packet_shadow_brute(kp, geo_lin, sr, ld, alive);
        if (alive) alive = shade_bounce(kp, ray, hit.p, hn, m, shadow, acc, att, 1e-3f);
    }
    if (pc.active) store_px(kp, pc.r, pc.x, make_float4(acc.x, acc.y, acc.z, 1.0f));
}

// ---------------------------------------------------------------------------
// k_accel: the packet walk over the reference tree plus the exact-result
// accelerator (accel.h). Which reference leaves a lane enters is decided by
// the reference's own box test; inside them, conservative local boxes and a
// distance margin skip shapes that cannot win; every candidate carries its
// rank in the reference walk so that ties resolve exactly as the reference's
// strict "<" in walk order does (lexicographic minimum of (distance, rank)).
// Barycentric triangle test only (the default); Moller-Trumbore frames use
// k_packet.

struct AccelPtrs {
    const float4* __restrict__ anodes;  // 4 float4 per reference node (the root's entry test)
    const float4* __restrict__ prims;   // 4 float4 per prim (PrimRec)
    const float4* __restrict__ lnodes;  // 6 float4 per local inner node: both child boxes + codes, cones
    const float4* __restrict__ wnodes;  // 8 float4 per reference inner node: both children's exact + content boxes
    const int4* __restrict__ tleaf;     // per reference leaf: plain start, plain count, local root code
    const float4* __restrict__ titems;  // 2 float4 per scene-tree item: exact box of its reference leaf + range
    int troot;                          // scene-tree root code (kLocal|w), kNoChild: reference tree only
    int scene_stack;                    // stack entries a scene-tree walk may use (<= the walk's own cap)
    int nfew;                           // > 0: items are gated by a per-ray mask over nfew reference leaves
                                        //      whose exact boxes are titems[0 .. 2*nfew) (few_mask)
    int N;
    float origin_lim;                   // AccelHost::origin_lim
    int boxes_finite;                   // no reference node box holds a NaN (ray_aabb_fast)
    int split_max;                      // lane_walk_any: split walks of waves with <= this many rays (0: off)
    int split_g;                        // ... over groups of at most this many lanes (a power of two)
    const int* __restrict__ prim_shape; // shape index per prim slot (the winner's material)
    float mt_z[3];                      // AccelHost::mt_z (Moller-Trumbore per-ray padding)
};

// Child codes of the walks' stacks and of lnodes / wnodes entries.
constexpr unsigned kLocal = 0x80000000u, kLeaf = 0x40000000u, kTopLeaf = 0x20000000u, kItem = 0x10000000u;
// A wide-node code (kLocal without kLeaf) with kPair names a node of two consecutive
// records (accel.h kWideKids, AccelHost::wpair): both are tested at one step.
constexpr unsigned kPair = 0x08000000u, kRecMask = 0x07ffffffu;
constexpr int kNoChild = 0x7fffffff;
constexpr bool kWide8 = RT_WIDE8 != 0;

// The closest hit so far: distance, rank in the reference walk, ray parameter and
// record slot. The hit point is o + t d, recomputed from t after the walk: the same
// float operations as where it was found, so the same bits (two registers fewer
// through the walks than keeping the point).
struct Best {
    float d;
    int seq;
    float t;
    int slot;
};

__device__ __forceinline__ V hit_point(const Ray& r, float t) { return r.o + t * r.d; }

__device__ __forceinline__ bool lex_better(float d, int seq, const Best& b) {
    return d < b.d || (d == b.d && seq < b.seq);
}

// gpu_shader.comp:242-328 for one candidate, taking the winner test early:
// the hit point and distance are computed exactly as the reference does, and
// the remaining (wall / barycentric) checks only run when the candidate could
// win. Same result as testing first and comparing after.
// Moller-Trumbore (gpu_shader.comp:170-195) with the same float operations as
// intersect(): t > 0 gives INNER at o + t d, whatever the triangle's facing.
__device__ __forceinline__ bool mt_hit(const float* f, const Ray& r, V& p, float& tt) {
    const V p1 = mk(f[4], f[5], f[6]), e1 = mk(f[7], f[8], f[9]), e2 = mk(f[10], f[11], f[12]);
    const V hh = cross(r.d, e2);
    const float a = dot(e1, hh);
    if (__builtin_fabsf(a) < 1e-5f) return false;
    const float fi = 1.0f / a;
    const V s = r.o - p1;
    const float u = fi * dot(s, hh);
    if (u < 0.0f || u > 1.0f) return false;
    const V q = cross(s, e1);
    const float v = fi * dot(r.d, q);
    if (v < 0.0f || u + v > 1.0f) return false;
    const float t = fi * dot(e2, q);
    if (!(t > 0.0f)) return false;
    p = hit_point(r, t);
    tt = t;
    return true;
}

// The barycentric terms of a PrimRec triangle (gpu_shader.comp:218-229): d00 and
// d11 recomputed as pack_geo computes them, d01 and the denominator stored.
__device__ __forceinline__ bool tri_inside(const float* f, V p) {
    const V e1 = mk(f[7], f[8], f[9]), e2 = mk(f[10], f[11], f[12]);
    const V tp = p - mk(f[4], f[5], f[6]);
    const float d20 = dot(tp, e1), d21 = dot(tp, e2);
    const float d00 = dot(e1, e1), d11 = dot(e2, e2);
    const float v = (d11 * d20 - f[13] * d21) / f[14];
    const float w = (d00 * d21 - f[13] * d20) / f[14];
    const float u = 1.0f - v - w;
    return !(u < 0.0f || v < 0.0f || w < 0.0f);
}

template <bool MT = false>
__device__ __forceinline__ void try_closest(const PrimRec& g, int slot, const Ray& r, Best& b) {
    const float* f = g.f;
    const int seq = g.st, type = prim_type(g);
    if (MT && type == 3) {
        V p;
        float t;
        if (!mt_hit(f, r, p, t)) return;
        const float d = dist(r.o, p);
        if (lex_better(d, seq, b)) b = Best{d, seq, t, slot};
        return;
    }
    if (type == 0) {
        V c = mk(f[0], f[1], f[2]);
        V oc = r.o - c;
        float aa = dot(r.d, r.d);
        float bb = 2.0f * dot(r.d, oc);
        float cc = dot(oc, oc) - f[3] * f[3];
        float D = bb * bb - 4.0f * aa * cc;
        if (D > 0.0f) {
            float t1 = (-bb - __builtin_sqrtf(D)) / (2.0f * aa);
            if (t1 > 0.0f) {
                V p = hit_point(r, t1);
                float d = dist(r.o, p);
                if (lex_better(d, seq, b)) b = Best{d, seq, t1, slot};
            }
        }
        return;
    }
    V n = mk(f[0], f[1], f[2]);
    const float np = dot(n, r.d);
    // INNER needs np > 0 and t = num / np > 0 (gpu_shader.comp:206-212,276-283):
    // both signs are known before the division, which only the survivors pay.
    if (!(np > 0.0f)) return;
    const float num = -(f[3] + dot(n, r.o));
    if (!(num > 0.0f)) return;
    const float t = num / np;
    if (!(t > 0.0f)) return;
    V p = hit_point(r, t);
    float d = dist(r.o, p);
    if (!lex_better(d, seq, b)) return;
    if (type == 2) {
        V lp = p - mk(f[4], f[5], f[6]);
        float up = dot(lp, mk(f[9], f[10], f[11]));
        float vp = dot(lp, mk(f[12], f[13], f[14]));
        if (up < 0.0f || up > f[7] || vp < 0.0f || vp > f[8]) return;
    } else if (type == 3) {
        if (!tri_inside(f, p)) return;
    }
    b = Best{d, seq, t, slot};
}

// Shadow candidate: an INNER hit nearer than lim (gpu_shader.comp:473-480).
template <bool MT = false>
__device__ __forceinline__ bool try_shadow(const PrimRec& g, const Ray& r, float lim) {
    const float* f = g.f;
    const int type = prim_type(g);
    if (MT && type == 3) {
        V p;
        float t;
        return mt_hit(f, r, p, t) && dist(r.o, p) < lim;
    }
    if (type == 0) {
        V c = mk(f[0], f[1], f[2]);
        V oc = r.o - c;
        float aa = dot(r.d, r.d);
        float bb = 2.0f * dot(r.d, oc);
        float cc = dot(oc, oc) - f[3] * f[3];
        float D = bb * bb - 4.0f * aa * cc;
        if (!(D > 0.0f)) return false;
        float t1 = (-bb - __builtin_sqrtf(D)) / (2.0f * aa);
        return t1 > 0.0f && dist(r.o, r.o + t1 * r.d) < lim;
    }
    V n = mk(f[0], f[1], f[2]);
    const float np = dot(n, r.d);
    if (!(np > 0.0f)) return false;  // signs first, as in try_closest
    const float num = -(f[3] + dot(n, r.o));
    if (!(num > 0.0f)) return false;
    const float t = num / np;
    if (!(t > 0.0f)) return false;
    V p = r.o + t * r.d;
    if (!(dist(r.o, p) < lim)) return false;
    if (type == 2) {
        V lp = p - mk(f[4], f[5], f[6]);
        float up = dot(lp, mk(f[9], f[10], f[11]));
        float vp = dot(lp, mk(f[12], f[13], f[14]));
        return !(up < 0.0f || up > f[7] || vp < 0.0f || vp > f[8]);
    }
    if (type == 3) return tri_inside(f, p);
    return true;
}

// Diagnostics (TIMED k_accel only): per-lane node steps and primitive tests.
struct WalkCount {
    unsigned nodes, tests;
    unsigned wnodes, wtests;  // wave iterations (TIMED diagnostics only): node steps, leaf-loop steps
};

// True in exactly one active lane: counts a wave-level iteration once.
__device__ __forceinline__ bool first_active() {
    return static_cast<int>(__lane_id()) == __builtin_ctzll(__ballot(1));
}

// Codes of the walk: a reference inner node k; kTopLeaf|k a reference leaf;
// kTopLeaf|kItem|i a scene-tree item; kLocal|j a wide node (local or scene
// tree); kLocal|kLeaf|start<<6|count a local leaf (start < 2^22, count < 64:
// bits 28-29 stay clear, so kTopLeaf and kItem are never set in a local code).
__device__ __forceinline__ int top_code(int k, int ia) { return ia < 0 ? static_cast<int>(kTopLeaf | k) : k; }

template <bool MT = false>
__device__ __forceinline__ rta::RayC ray_c(const Ray& r, const AccelPtrs& A) {
    rta::RayC c = rta::ray_consts(r.o.x, r.o.y, r.o.z, r.d.x, r.d.y, r.d.z, A.origin_lim);
    if (MT) rta::mt_ray(c, r.o.x, r.o.y, r.o.z, A.mt_z);
    return c;
}

__device__ __forceinline__ bool box_enter(const rta::RayC& c, float4 lo, float4 hi, float tl, float& te) {
    return rta::box_enter(c, lo.x, lo.y, lo.z, hi.x, hi.y, hi.z, tl, te);
}

// Scene-tree item (accel.h, SceneTree): the exact box test of its reference
// leaf (gpu_shader.comp:364-377; NaN-free for the rays that take the scene
// tree), then its prim range.
__device__ __forceinline__ bool enter_item(const AccelPtrs& A, unsigned uc, const Ray& r, const V& inv, int& start,
                                           int& count) {
    const float4* q = A.titems + 2 * static_cast<size_t>(uc & 0x0fffffffu);
    const float4 e0 = q[0], e1 = q[1];
    start = __float_as_int(e0.w);
    count = __float_as_int(e1.w);
    return ray_aabb_fast(r.o, inv, mk(e0.x, e0.y, e0.z), mk(e1.x, e1.y, e1.z));
}

// Few-leaf scenes (<= 8 reference leaves): the exact box tests of all of them
// once per walk; items are then local-leaf codes with kItem set and the leaf's
// index in bits 3-5 (no item record load on the walk).
__device__ __forceinline__ unsigned few_mask(const AccelPtrs& A, const Ray& r, const V& inv) {
    unsigned fm = 0;
    for (int i = 0; i < A.nfew; ++i) {
        const float4 e0 = A.titems[2 * i], e1 = A.titems[2 * i + 1];
        if (ray_aabb_fast(r.o, inv, mk(e0.x, e0.y, e0.z), mk(e1.x, e1.y, e1.z))) fm |= 1u << i;
    }
    return fm;
}

// A ray walks the scene tree when one is built and its slab values cannot be
// NaN (aabb_fast_ok) and the padded tests are in their bounded mode (c.ix != 0).
__device__ __forceinline__ bool use_scene(const AccelPtrs& A, bool fast, const rta::RayC& c) {
    return A.troot != kNoChild && fast && c.ix != 0.0f;
}

// The root has no parent: its own exact box decides entry (gpu_shader.comp:386-395),
// then its content box.
__device__ __forceinline__ bool enter_root(const AccelPtrs& A, const Ray& r, const V& inv, const rta::RayC& c,
                                           float tl, int& code) {
    const float4* q = A.anodes + 4 * static_cast<size_t>(A.N - 1);
    const float4 e0 = q[0], e1 = q[1], c0 = q[2], c1 = q[3];
    float te;
    code = top_code(A.N - 1, __float_as_int(e0.w));
    return ray_aabb(r.o, inv, mk(e0.x, e0.y, e0.z), mk(e1.x, e1.y, e1.z)) &&
           (!(__float_as_int(c0.w) & 8) || box_enter(c, c0, c1, tl, te));
}

// Both children of a node in hand: which the lane enters and at what parameter.
// Reference inner node: the children's exact boxes with the GLSL test (the
// reference's own entry decision, evaluated at the parent), then their content
// boxes. Local inner node: padded child boxes and back-face cones.
struct Kids {
    int ca, cb;
    float ta, tb;
    bool ha, hb;
};

__device__ __forceinline__ Kids ref_kids(const AccelPtrs& A, unsigned uc, const Ray& r, const V& inv,
                                         const rta::RayC& c, float tl, bool in, bool fast) {
    const float4* q = A.wnodes + 8 * static_cast<size_t>(uc);
    const float4 ae0 = q[0], ae1 = q[1], ac0 = q[2], ac1 = q[3];
    const float4 be0 = q[4], be1 = q[5], bc0 = q[6], bc1 = q[7];
    Kids k;
    bool ea, eb;
    if (fast) {
        ea = ray_aabb_fast(r.o, inv, mk(ae0.x, ae0.y, ae0.z), mk(ae1.x, ae1.y, ae1.z));
        eb = ray_aabb_fast(r.o, inv, mk(be0.x, be0.y, be0.z), mk(be1.x, be1.y, be1.z));
    } else {
        ea = ray_aabb(r.o, inv, mk(ae0.x, ae0.y, ae0.z), mk(ae1.x, ae1.y, ae1.z));
        eb = ray_aabb(r.o, inv, mk(be0.x, be0.y, be0.z), mk(be1.x, be1.y, be1.z));
    }
    // content boxes evaluated unconditionally (no branch between the loads and their use)
    float ta, tb;
    const bool pa = box_enter(c, ac0, ac1, tl, ta), pb = box_enter(c, bc0, bc1, tl, tb);
    const bool fa = (__float_as_int(ac0.w) & 8) != 0, fb = (__float_as_int(bc0.w) & 8) != 0;
    k.ha = in & ea & (pa | !fa);
    k.hb = in & eb & (pb | !fb);
    k.ta = fa ? ta : 0.f;
    k.tb = fb ? tb : 0.f;
    k.ca = __float_as_int(ae0.w);
    k.cb = __float_as_int(ae1.w);
    return k;
}

// A wide local node (accel.h, build_wide): up to four children, stored as
// 11 float4 (lo.x[4], lo.y[4], lo.z[4], hi.x[4], hi.y[4], hi.z[4], cone
// axis x[4], y[4], z[4], cone threshold[4], child codes[4]). Returns the
// children sorted by entry parameter, misses last (key = +inf).
struct Kids4 {
    float t[4];
    int code[4];
};

__device__ __forceinline__ void cas(Kids4& k, int i, int j) {
    const bool sw = k.t[j] < k.t[i];
    const float ti = k.t[i], tj = k.t[j];
    const int ci = k.code[i], cj = k.code[j];
    k.t[i] = sw ? tj : ti;
    k.t[j] = sw ? ti : tj;
    k.code[i] = sw ? cj : ci;
    k.code[j] = sw ? ci : cj;
}

// Two children per packed instruction (v_pk_fma_f32, v_pk_mul_f32): the same
// fma / mul per component as rta::box_enter and rta::cone_culls.
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

// The barycentric accelerator's wide node, 8 float4 = 128 B (one cache line):
// the four children's boxes as six rows (lo.x of the four, lo.y, ... hi.z), one
// quantized back-face cone word per child (accel_math.h, cone_word; kConeNp
// marks a kNoPrune child: entered at parameter 0, no distance limit) and the
// child codes. Same slab operations as rta::box_enter; the cone test is one
// dot4 per child.
__device__ __forceinline__ void wide_pair_q(const rta::RayC& c, float tl, f2 lx, f2 ly, f2 lz, f2 hx, f2 hy, f2 hz,
                                            int w0, int w1, float& t0, float& t1, bool& h0, bool& h1) {
    const f2 ix = {c.ix, c.ix}, iy = {c.iy, c.iy}, iz = {c.iz, c.iz};
    const f2 ox = {-c.ox, -c.ox}, oy = {-c.oy, -c.oy}, oz = {-c.oz, -c.oz};
    const f2 x0 = fma2(lx, ix, ox), x1 = fma2(hx, ix, ox);
    const f2 y0 = fma2(ly, iy, oy), y1 = fma2(hy, iy, oy);
    const f2 z0 = fma2(lz, iz, oz), z1 = fma2(hz, iz, oz);
    const int w[2] = {w0, w1};
    float tn[2], tf[2], te[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const bool np = w[k] == rta::kConeNp;
        tn[k] = fmaxf(fmaxf(fminf(x0[k], x1[k]), fminf(y0[k], y1[k])), fmaxf(fminf(z0[k], z1[k]), 0.0f));
        const float tz = fmaxf(z0[k], z1[k]);
        tf[k] = fminf(fminf(fmaxf(x0[k], x1[k]), fmaxf(y0[k], y1[k])), np ? fminf(tz, INFINITY) : fminf(tz, tl));
        te[k] = np ? 0.0f : tn[k];
    }
    t0 = te[0];
    t1 = te[1];
    h0 = (tn[0] <= tf[0]) & !rta::cone_culls_q(w0, c.dq);
    h1 = (tn[1] <= tf[1]) & !rta::cone_culls_q(w1, c.dq);
}

// Wide-node record stride in float4: 8 (quantized cones), 17 for the
// Moller-Trumbore accelerator: boxes (6), float grazing cones (4: axis, s),
// the per-ray padding constants (6, accel.h AccelHost::lmt) and the codes.
constexpr int kWideRec = 8, kWideRecMt = 17;
#ifndef RT_MT_UNROLL
#define RT_MT_UNROLL 4  // MT wide_kids: children per unrolled step (r03j: 1 -> 4 car MT -15 %)
#endif
constexpr int kMtUnroll = RT_MT_UNROLL;
#ifndef RT_MT_ILF
#define RT_MT_ILF 1  // MT entry parameter scaled by mt_pad's 1/lf bound, not a reciprocal (car MT -2.0 %, r04zz9)
#endif

// Float `comp` of child `sl`'s box (0-2 lo.xyz, 3-5 hi.xyz) in wide record w:
// row comp, lane sl of the SoA records; float comp of the child's 16-float
// block in the MT records (wide_kids).
__host__ __device__ __forceinline__ float* wide_box_f(float4* lnodes, int rec, int w, int sl, int comp) {
    float* base = reinterpret_cast<float*>(lnodes + rec * static_cast<size_t>(w));
    return rec == kWideRecMt ? base + 16 * sl + comp : base + 4 * comp + sl;
}


template <bool MT = false>
__device__ __forceinline__ Kids4 wide_kids(const AccelPtrs& A, unsigned uc, const rta::RayC& c, float tl, bool in) {
    const float4* q = A.lnodes + (MT ? kWideRecMt : kWideRec) * static_cast<size_t>(uc & kRecMask);
    float t[4];
    bool h[4];
    int cc[4];
    if (MT) {
        // per-ray padding (accel_math.h mt_pad / mt_slab; accel_bound.h): each
        // child's static box grown by its pad, the distance limit by lf, then the
        // slab along its cone axis; a child without a finite bound is entered at 0.
        // Record: per child 4 float4 (lo.xyz hi.x | hi.yz axis.xy | axis.z s m0 m1 |
        // m2 m3 m4 m5), then the codes. Results select-written (kMtUnroll < 4 would
        // index them by a loop variable). Pairs of children on packed f32
        // instructions (as wide_pair_q) spilled 40-140 VGPRs in every MT instance (r03).
        const float4 cd = q[16];
        t[0] = t[1] = t[2] = t[3] = 0.0f;
        h[0] = h[1] = h[2] = h[3] = false;
        cc[0] = __float_as_int(cd.x), cc[1] = __float_as_int(cd.y), cc[2] = __float_as_int(cd.z);
        cc[3] = __float_as_int(cd.w);
#pragma unroll kMtUnroll
        for (int s2 = 0; s2 < 4; ++s2) {
            const float4 f0 = q[4 * s2], f1 = q[4 * s2 + 1], f2v = q[4 * s2 + 2], f3 = q[4 * s2 + 3];
            const float k[4] = {f1.z, f1.w, f2v.x, f2v.y};
            const float m[6] = {f2v.z, f2v.w, f3.x, f3.y, f3.z, f3.w};
            float pad, lf, q2, pt, ilf, tt = 0.0f;
            bool hh = true;
            // (r05: a wave-uniform floor case of mt_pad from per-child constants spilled
            // 28 VGPRs in the production MT instance: car MT frame 1.293 -> 1.455 ms in
            // flight, 1.577 without its slab; profiles/r05e_abf_floor*.json. Not kept.)
            const bool ok = rta::mt_pad(c, c.so, k, m, pad, lf, q2, pt, ilf);
            if (ok) {
                float tn, tf;
                hh = rta::box_span(c, f0.x - pad, f0.y - pad, f0.z - pad, f0.w + pad, f1.x + pad, f1.y + pad,
                                   tl * lf, tn, tf);
                if (hh && c.ix != 0.0f && m[5] < 3e38f)
                    hh = rta::mt_slab(c.mox, c.moy, c.moz, c.on, c, k, m, q2, pt, tn, tf);
#if RT_MT_ILF
                tt = tn * ilf;  // the stack's prune compares with tl, not tl * lf (ilf <= 1 / lf)
#else
                tt = tn * rta::rcp(lf) * 0.99999f;  // the stack's prune compares with tl, not tl * lf
#endif
            }
            // select-written (a lane-varying index would put t / h in scratch)
            t[0] = s2 == 0 ? tt : t[0], t[1] = s2 == 1 ? tt : t[1], t[2] = s2 == 2 ? tt : t[2];
            t[3] = s2 == 3 ? tt : t[3];
            h[0] = s2 == 0 ? hh : h[0], h[1] = s2 == 1 ? hh : h[1], h[2] = s2 == 2 ? hh : h[2];
            h[3] = s2 == 3 ? hh : h[3];
        }
    } else {
        const float4 lx = q[0], ly = q[1], lz = q[2], hx = q[3], hy = q[4], hz = q[5];
        const float4 cw = q[6], cd = q[7];
        cc[0] = __float_as_int(cd.x), cc[1] = __float_as_int(cd.y), cc[2] = __float_as_int(cd.z);
        cc[3] = __float_as_int(cd.w);
        wide_pair_q(c, tl, (f2){lx.x, lx.y}, (f2){ly.x, ly.y}, (f2){lz.x, lz.y}, (f2){hx.x, hx.y}, (f2){hy.x, hy.y},
                    (f2){hz.x, hz.y}, __float_as_int(cw.x), __float_as_int(cw.y), t[0], t[1], h[0], h[1]);
        wide_pair_q(c, tl, (f2){lx.z, lx.w}, (f2){ly.z, ly.w}, (f2){lz.z, lz.w}, (f2){hx.z, hx.w}, (f2){hy.z, hy.w},
                    (f2){hz.z, hz.w}, __float_as_int(cw.z), __float_as_int(cw.w), t[2], t[3], h[2], h[3]);
    }
    Kids4 k;
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
        k.t[s2] = (h[s2] & (cc[s2] != kNoChild) & in) ? t[s2] : INFINITY;
        k.code[s2] = cc[s2];
    }
    return k;
}

__device__ __forceinline__ void sort4(Kids4& k) {
    cas(k, 0, 1);
    cas(k, 2, 3);
    cas(k, 0, 2);
    cas(k, 1, 3);
    cas(k, 1, 2);
}

// The second record of a kPair node (its children 4-7), or none: every child a miss.
template <bool MT = false>
__device__ __forceinline__ Kids4 wide_kids_hi(const AccelPtrs& A, unsigned uc, const rta::RayC& c, float tl, bool in) {
    Kids4 k;
    if (!MT && kWide8 && (uc & kPair)) return wide_kids<MT>(A, uc + 1u, c, tl, in);
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
        k.t[s2] = INFINITY;
        k.code[s2] = kNoChild;
    }
    return k;
}

// Both records' children as one list sorted by entry parameter (19-comparator
// network), for the split walk's shared prologue.
struct Kids8 {
    float t[8];
    int code[8];
};
__device__ __forceinline__ Kids8 sort8(const Kids4& a, const Kids4& b) {
    Kids8 k;
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
        k.t[s2] = a.t[s2], k.code[s2] = a.code[s2];
        k.t[4 + s2] = b.t[s2], k.code[4 + s2] = b.code[s2];
    }
    auto cx = [&](int i, int j) {
        const bool sw = k.t[j] < k.t[i];
        const float ti = k.t[i], tj = k.t[j];
        const int ci = k.code[i], cj = k.code[j];
        k.t[i] = sw ? tj : ti, k.t[j] = sw ? ti : tj;
        k.code[i] = sw ? cj : ci, k.code[j] = sw ? ci : cj;
    };
    cx(0, 1), cx(2, 3), cx(4, 5), cx(6, 7), cx(0, 2), cx(1, 3), cx(4, 6), cx(5, 7), cx(1, 2), cx(5, 6);
    cx(0, 4), cx(1, 5), cx(2, 6), cx(3, 7), cx(2, 4), cx(3, 5), cx(1, 2), cx(3, 4), cx(5, 6);
    return k;
}
__device__ __forceinline__ int pick_code8(const Kids8& k, int i) {
    int r = k.code[0];
#pragma unroll
    for (int s2 = 1; s2 < 8; ++s2) r = i == s2 ? k.code[s2] : r;
    return r;
}
__device__ __forceinline__ float pick_t8(const Kids8& k, int i) {
    float r = k.t[0];
#pragma unroll
    for (int s2 = 1; s2 < 8; ++s2) r = i == s2 ? k.t[s2] : r;
    return r;
}

// k.code[i] / k.t[i] for a lane-varying i (selects, no indexed registers)
__device__ __forceinline__ int pick_code(const Kids4& k, int i) {
    return i == 0 ? k.code[0] : i == 1 ? k.code[1] : i == 2 ? k.code[2] : k.code[3];
}
__device__ __forceinline__ float pick_t(const Kids4& k, int i) {
    return i == 0 ? k.t[0] : i == 1 ? k.t[1] : i == 2 ? k.t[2] : k.t[3];
}

// Stacked entry parameters are kept as bf16 rounded toward zero: never above
// the true value (te >= 0), so the pop-time prune only ever drops less.
__device__ __forceinline__ unsigned short f_bf16_down(float t) {
    return static_cast<unsigned short>(__float_as_uint(t) >> 16);
}
__device__ __forceinline__ float bf16_f(unsigned short b) { return __uint_as_float(static_cast<unsigned>(b) << 16); }

#ifndef RT_SPLIT_ALL
#define RT_SPLIT_ALL 0  // split walks (lane_walk_any) in every k_accel instance (experiment builds)
#endif
#ifndef RT_LEAF_PREFETCH
#define RT_LEAF_PREFETCH 0  // lane_walk's leaf loop software-pipelined (experiment builds)
#endif

#ifndef RT_FLAT_LOOP
#define RT_FLAT_LOOP 1  // lane_walk's SPEC descent as a one-exit loop (r03: config 5 -3 %)
#endif

// Per-lane walk ("while-while"): each lane walks its own stack in LDS (code +
// entry parameter per entry). A lane descends until it holds a leaf, keeping
// the nearer child in registers and stacking the farther one; the wave then
// tests all lanes' leaves together. A stacked entry is dropped on pop when a
// nearer hit has been found since it was pushed.
//
// Split walks (sg > 1, lane_walk_any): the sg lanes of an aligned group walk one
// ray. From the root (a prologue before the main loop, so the loop's registers
// are not raised) they share a path (ss lanes, this lane the si-th) and test
// its nodes with a fixed limit (tl0), so every lane of the share sees
// the same children; a node with h hit children hands child p to the lanes
// si * h / ss == p (h < ss) or lane si the children si, si + ss, ... (h >= ss,
// its own from then on). Every child is walked by some lane, leaves of the
// shared part by all of them. The lanes' best distances are pooled after every
// round of leaf tests (and a shadow hit ends the group's walks); the result is
// the (distance, rank) minimum over the group, which does not depend on which
// lane tested which leaf.
// FLAT_SHADOW: a shadow hit sets the lane's flags and ends its leaf loop through the loop
// test, instead of returning from inside the loop (r03: car -1.7 % in flight and serially;
// config 5 +0.5 %, so the big-scene instances, which split walks, keep the return).
template <bool SHADOW, bool COUNT = false, bool WSTAT = false, bool SPEC = true, bool MT = false,
          bool FLAT_SHADOW = false>
__device__ void lane_walk(const AccelPtrs& A, const Ray& r, bool active, float lim_shadow, Best& b, bool& shadow,
                          int* stk, unsigned short* stt, int stride, int cap, WalkCount& wc, int sg = 1,
                          int si = 0) {
    if (A.N <= 0 || !active) return;
    const V inv = inv_dir(r.d);
    const bool fast = A.boxes_finite && aabb_fast_ok(r.o, inv);
    const rta::RayC c = ray_c<MT>(r, A);
    float tl = rta::t_limit(SHADOW ? lim_shadow : b.d, c.rdl);
    // sp: the stack top as an element offset (entries x stride), so a push or pop
    // adds or subtracts stride instead of multiplying (v_mul_lo_u32 is quarter rate)
    int sp = 0, cur = A.troot;
    const int capo = cap * stride;
    bool have = true;
    // The scene tree has no static stack bound: a lane whose push would not fit
    // drops it and marks `ovf`; when its walk ends it walks the reference tree
    // from the root (with the best hit so far), whose bound the builder checked.
    bool ovf = false;
    int pcap = min(cap, A.scene_stack) * stride;  // push bound of the tree being walked (offset)
    unsigned fm = 0;
    if (!use_scene(A, fast, c)) {
        have = enter_root(A, r, inv, c, tl, cur);
        pcap = capo;
    } else if (A.nfew > 0) {
        fm = few_mask(A, r, inv);
    }
    int start = 0, count = 0;  // the leaf range this lane holds (reset after each round's tests)
    if (sg > 1) {
        // Split: the shared top of the tree, out of the main loop (whose registers it
        // does not add to). Shared nodes are tested with a fixed limit (tl0), so every
        // lane of a share (ss lanes, this the si-th) sees the same children.
        const float tl0 = SHADOW ? tl : INFINITY;
        int ss = sg;
        while (have && ss > 1) {
            const unsigned uc = static_cast<unsigned>(cur);
            if (uc & (kLeaf | kItem)) break;  // a leaf: the share tests it (and walks on) together
            if (COUNT) wc.nodes++;
            if (uc & kTopLeaf) {  // plain range + local root: hold the range, enter the root
                if (count > 0) break;
                const int4 lf = A.tleaf[uc & 0x0fffffffu];
                start = lf.x;
                count = lf.y;
                have = lf.z != kNoChild;
                cur = lf.z;
            } else if (uc & kLocal) {
                if constexpr (!MT && kWide8) {
                    // a kPair node: both records' children, sorted as one list of up to 8
                    const Kids8 w = sort8(wide_kids<MT>(A, uc, c, tl0, true), wide_kids_hi<MT>(A, uc, c, tl0, true));
                    int h = 0;
#pragma unroll
                    for (int s2 = 0; s2 < 8; ++s2) h += w.t[s2] < INFINITY;
                    if (h == 0) {
                        have = false;
                    } else if (h >= ss) {  // positions si, si + ss, ... (ss >= 2, h <= 8) are this lane's
                        for (int q = si + ss; q < h; q += ss) {
                            if (sp < pcap) {
                                stk[sp] = pick_code8(w, q);
                                stt[sp] = f_bf16_down(pick_t8(w, q));
                                sp += stride;
                            } else {
                                ovf = true;
                            }
                        }
                        cur = pick_code8(w, si);
                        ss = 1;
                    } else {  // child p, shared by the lanes [lo, hi) of this share
                        const int p = si * h / ss, lo = (p * ss + h - 1) / h, hi = ((p + 1) * ss + h - 1) / h;
                        cur = pick_code8(w, p);
                        si -= lo;
                        ss = hi - lo;
                    }
                } else {
                    Kids4 w = wide_kids<MT>(A, uc, c, tl0, true);
                    sort4(w);
                    const int h = (w.t[0] < INFINITY) + (w.t[1] < INFINITY) + (w.t[2] < INFINITY) + (w.t[3] < INFINITY);
                    if (h == 0) {
                        have = false;
                    } else if (h >= ss) {  // positions si and si + ss (ss >= 2, h <= 4) are this lane's
                        if (si + ss < h) {
                            if (sp < pcap) {
                                stk[sp] = pick_code(w, si + ss);
                                stt[sp] = f_bf16_down(pick_t(w, si + ss));
                                sp += stride;
                            } else {
                                ovf = true;
                            }
                        }
                        cur = pick_code(w, si);
                        ss = 1;
                    } else {  // child p, shared by the lanes [lo, hi) of this share
                        const int p = si * h / ss, lo = (p * ss + h - 1) / h, hi = ((p + 1) * ss + h - 1) / h;
                        cur = pick_code(w, p);
                        si -= lo;
                        ss = hi - lo;
                    }
                }
            } else {
                const Kids k = ref_kids(A, uc, r, inv, c, tl0, true, fast);
                if (k.ha && k.hb) {  // two children over ss >= 2 lanes
                    const bool a_first = !(k.tb < k.ta);
                    const int p = si * 2 / ss, lo = (p * ss + 1) / 2, hi = ((p + 1) * ss + 1) / 2;
                    cur = (p == 0) == a_first ? k.ca : k.cb;
                    si -= lo;
                    ss = hi - lo;
                } else if (k.ha || k.hb) {
                    cur = k.ha ? k.ca : k.cb;
                } else {
                    have = false;
                }
            }
        }
    }
    // From here `cur == kNoChild` means the lane holds no node (no separate flag: one
    // lane mask fewer to merge at every join of the descent)
    if (!have) cur = kNoChild;
    bool ended = false;
    for (;;) {
        // While-while: a lane descends until it holds a leaf. SPEC (speculative):
        // it then keeps walking inner nodes while any other lane is still looking
        // for one; a lane that meets a second leaf parks on it (kept for the next
        // round), and the round ends when every walking lane holds a leaf
        // (measured: config 3 -4 %, config 5 -14 %).
#if RT_FLAT_LOOP
        // SPEC in one-exit form: a lane that finishes, parks or ends its walk sets `stop`
        // instead of leaving the loop, and the round ends on the wave-uniform test alone
        // (the same steps in the same order per lane; fewer lane-mask merges per step).
        bool stop = ended;
        if (SPEC) {  // ended lanes are stopped: no exec test around the loop (config 5: -2 %)
            for (;;) {
                if (__ballot(!stop && count == 0) == 0) break;
                if (!stop && cur == kNoChild) {
                    if (sp == 0) {
                        if (ovf) {  // a scene-tree push was dropped: the reference tree, from its root
                            ovf = false;
                            pcap = capo;
                            if (!enter_root(A, r, inv, c, tl, cur)) cur = kNoChild;
                        }
                        if (cur == kNoChild) {
                            ended = count == 0;  // walk finished (a held leaf is still tested)
                            stop = true;
                        }
                    } else {
                        sp -= stride;
                        const int pc = stk[sp];
                        cur = bf16_f(stt[sp]) > tl ? kNoChild : pc;  // dropped if a nearer hit was found since the push
                    }
                }
                const unsigned uc = static_cast<unsigned>(cur);
                stop = stop || (cur != kNoChild && count > 0 && (uc & (kTopLeaf | kLeaf)));  // park on a leaf
                if (stop || cur == kNoChild) continue;
#else
        if (!ended) {
            for (;;) {
                if (SPEC ? __ballot(!ended && count == 0) == 0 : count > 0) break;
                if (cur == kNoChild) {
                    if (sp == 0) {
                        if (ovf) {  // a scene-tree push was dropped: the reference tree, from its root
                            ovf = false;
                            pcap = capo;
                            if (enter_root(A, r, inv, c, tl, cur)) continue;
                            cur = kNoChild;
                        }
                        if (count == 0) ended = true;  // walk finished (a held leaf is still tested)
                        break;
                    }
                    sp -= stride;
                    if (bf16_f(stt[sp]) > tl) continue;  // a nearer hit was found since the push
                    cur = stk[sp];
                }
                const unsigned uc = static_cast<unsigned>(cur);
                if (count > 0 && (uc & (kTopLeaf | kLeaf))) break;  // park on a leaf
#endif
                if (COUNT) wc.nodes++;
                if (WSTAT && first_active()) wc.wnodes++;
                cur = kNoChild;  // the branches below set the next node, if any
                // kLocal codes (wide nodes and local leaves, including few-leaf items) first,
                // as one region: a round in which no lane holds a reference-tree code skips
                // the rest with one exec test instead of three
                if (uc & kLocal) {
                    if (uc & kLeaf) {
                        start = static_cast<int>((uc >> 6) & 0x3fffffu);
                        count = static_cast<int>(uc & 0x3fu);
                        if (uc & kItem) count = ((fm >> (count >> 3)) & 1u) ? (count & 7) : 0;  // few-leaf item
                    } else {
                        auto push = [&](float t, int code) {
                            if (t < INFINITY) {
                                if (sp < pcap) {
                                    stk[sp] = code;
                                    stt[sp] = f_bf16_down(t);
                                    sp += stride;
                                } else {
                                    ovf = true;  // scene tree only: local trees fit their bound
                                }
                            }
                        };
                        // a node of two records (kPair): the second record's children first,
                        // sorted, its 2nd-4th stacked; then the first record's; the nearer of
                        // the two records' nearest is walked, the other stacked last. One
                        // record's values live at a time (the walk is at the VGPR cap).
                        const bool pair = !MT && kWide8 && (uc & kPair);
                        float vt = INFINITY;
                        int vc = kNoChild;
                        if (pair) {
                            Kids4 v = wide_kids<MT>(A, uc + 1u, c, tl, true);
                            sort4(v);
#pragma unroll
                            for (int s2 = 3; s2 >= 1; --s2) push(v.t[s2], v.code[s2]);
                            vt = v.t[0];
                            vc = v.code[0];
                        }
                        Kids4 w = wide_kids<MT>(A, uc, c, tl, true);
                        sort4(w);
#pragma unroll
                        for (int s2 = 3; s2 >= 1; --s2) push(w.t[s2], w.code[s2]);
                        if (pair) {
                            const bool vf = vt < w.t[0];
                            push(vf ? w.t[0] : vt, vf ? w.code[0] : vc);
                            w.t[0] = vf ? vt : w.t[0];
                            w.code[0] = vf ? vc : w.code[0];
                        }
                        if (w.t[0] < INFINITY) cur = w.code[0];
                    }
                } else if ((uc & (kTopLeaf | kItem)) == (kTopLeaf | kItem)) {
                    int s0, n0;
                    if (enter_item(A, uc, r, inv, s0, n0)) {
                        start = s0;
                        count = n0;
                    }
                } else if (uc & kTopLeaf) {
                    const int4 lf = A.tleaf[uc & 0x0fffffffu];
                    start = lf.x;
                    count = lf.y;
                    cur = lf.z;  // the local root (kNoChild: none) is entered with the leaf
                } else {
                    const Kids k = ref_kids(A, uc, r, inv, c, tl, true, fast);
                    if (k.ha && k.hb) {
                        const bool a_first = !(k.tb < k.ta);  // nearer entry first
                        if (sp < capo) {
                            stk[sp] = a_first ? k.cb : k.ca;
                            stt[sp] = f_bf16_down(a_first ? k.tb : k.ta);
                            sp += stride;
                        }
                        cur = a_first ? k.ca : k.cb;
                    } else if (k.ha || k.hb) {
                        cur = k.ha ? k.ca : k.cb;
                    }
                }
            }
        }
        if (__ballot(count > 0) == 0) return;  // every lane's walk finished
#if RT_LEAF_PREFETCH
        // the leaf's records software-pipelined: record i + 1's loads are in flight while
        // record i is tested (a leaf is a chain of dependent loads otherwise)
        PrimRec gn;
        if (count > 0) gn = load_prim(A.prims, start);
        for (int i = 0; i < count; ++i) {
            const PrimRec g = gn;
            if (i + 1 < count) gn = load_prim(A.prims, start + i + 1);
#else
        for (int i = 0; i < count; ++i) {
            const PrimRec g = load_prim(A.prims, start + i);
#endif
            if (COUNT) wc.tests++;
            if (WSTAT && first_active()) wc.wtests++;
            if (SHADOW && FLAT_SHADOW) {
                // an occluder ends this lane's walk at the next round's test (no exit
                // from inside the loop)
                if (try_shadow<MT>(g, r, lim_shadow)) {
                    shadow = true;
                    ended = true;
                    count = i + 1;
                }
            } else if (SHADOW) {
                if (try_shadow<MT>(g, r, lim_shadow)) {
                    shadow = true;
                    if (sg == 1) return;
                    ended = true;  // split: the group learns it below
                    break;
                }
            } else {
                try_closest<MT>(g, start + i, r, b);
            }
        }
        count = 0;
        if (sg > 1) {  // every lane of the wave's groups is here (the returns above are wave-uniform)
            if (SHADOW) {
                int any = shadow ? 1 : 0;
                for (int o = 1; o < sg; o <<= 1) any |= __shfl_xor(any, o);
                if (any) {
                    shadow = true;
                    ended = true;
                }
            } else {
                float d = b.d;
                for (int o = 1; o < sg; o <<= 1) d = fminf(d, __shfl_xor(d, o));
                tl = rta::t_limit(d, c.rdl);
            }
        } else if (!SHADOW) {
            tl = rta::t_limit(b.d, c.rdl);
        }
    }
}

// lane_walk for a wave's rays. A wave with few rays (at most A.split_max, e.g. the
// reflections of a tile where little is a mirror) gives each ray a group of idle
// lanes that split its walk (lane_walk, sg > 1): the longest walk of the wave gets
// shorter, and the wave issues fewer rounds. The group's result is the lexicographic
// (distance, rank) minimum of its lanes' -- the same hit as one lane's whole walk.
// One lane_walk either way (one copy of the walk in the kernel). b must hold the
// same value in every lane (bounce_step's fresh best); on return it holds each
// active lane's result and r each active lane's own ray (both are rebuilt from the
// group, so neither is live across the walk).
// SPLIT = false compiles the plain walk alone: the split's registers spill in the
// car's production kernel (+8 % per frame there, r02m), so only the kernels of
// big scenes (the compacting k_accel instance and k_accel_tail) carry it.
template <bool SHADOW, bool COUNT = false, bool WSTAT = false, bool SPEC = true, bool MT = false, bool SPLIT = true>
__device__ __forceinline__ void lane_walk_any(const AccelPtrs& A, Ray& r, bool active, float lim_shadow, Best& b,
                                              bool& shadow, int* stk, unsigned short* stt, int stride, int cap,
                                              WalkCount& wc) {
    if (!SPLIT) {  // the plain walk, without the split's registers
        lane_walk<SHADOW, COUNT, WSTAT, SPEC, MT, true>(A, r, active, lim_shadow, b, shadow, stk, stt, stride, cap, wc);
        return;
    }
    const unsigned long long m = __ballot(active);
    const int n = __popcll(m);
    int G = 1;
    while (G < A.split_g && 2 * G * n <= 64) G *= 2;
    if (n == 0 || n > A.split_max) G = 1;  // wave-uniform
    const int lane = lane_id();
    int src = lane;  // the ray this lane walks
    bool walk = active;
    if (G > 1) {
        const int j = lane / G;
        int q = 0;  // the j-th ray of the wave (wave-uniform loop over m's bits)
        for (unsigned long long mm = m; mm; mm &= mm - 1ull, ++q)
            if (q == j) src = __builtin_ctzll(mm);
        walk = j < n;
    }
    Ray rr{mk(__shfl(r.o.x, src), __shfl(r.o.y, src), __shfl(r.o.z, src)),
           mk(__shfl(r.d.x, src), __shfl(r.d.y, src), __shfl(r.d.z, src))};
    const float ls = __shfl(lim_shadow, src);
    bool sh = false;
    lane_walk<SHADOW, COUNT, WSTAT, SPEC, MT>(A, rr, walk, ls, b, sh, stk, stt, stride, cap, wc, G, lane % G);
    // the group lane holding this lane's result (recomputed here: nothing extra live through the walk)
    const int from = G > 1 ? G * __popcll(__ballot(active) & ((1ull << lane) - 1ull)) : lane;
    if (SHADOW) {
        int any = sh ? 1 : 0;
        for (int o = 1; o < G; o <<= 1) any |= __shfl_xor(any, o);
        any = __shfl(any, from);
        if (active && any) shadow = true;
    } else {
        for (int o = 1; o < G; o <<= 1) {
            const float d = __shfl_xor(b.d, o);
            const int sq = __shfl_xor(b.seq, o), sl = __shfl_xor(b.slot, o);
            const float tt = __shfl_xor(b.t, o);
            if (lex_better(d, sq, b)) b = Best{d, sq, tt, sl};
        }
        b = Best{__shfl(b.d, from), __shfl(b.seq, from), __shfl(b.t, from), __shfl(b.slot, from)};
        r = Ray{mk(__shfl(rr.o.x, from), __shfl(rr.o.y, from), __shfl(rr.o.z, from)),
                mk(__shfl(rr.d.x, from), __shfl(rr.d.y, from), __shfl(rr.d.z, from))};
    }
}

// Packet walk: one wave-uniform walk with a 64-bit lane mask per stack entry
// (VGPR-resident stack, scalar node loads). The reference's walk order does
// not depend on the ray, so one walk with masks reproduces every lane's own;
// the order among children follows the first lane that enters both.
template <bool SHADOW, bool COUNT = false, bool WSTAT = false, bool MT = false>
__device__ void packet_walk(const AccelPtrs& A, const Ray& r, bool active, float lim_shadow, Best& b,
                            bool& shadow, WalkCount& wc) {
    unsigned long long m = __ballot(active);
    if (A.N <= 0 || m == 0) return;
    const V inv = inv_dir(r.d);
    const bool fast = A.boxes_finite && aabb_fast_ok(r.o, inv);
    const rta::RayC c = ray_c<MT>(r, A);
    float tl = rta::t_limit(SHADOW ? lim_shadow : b.d, c.rdl);
    WaveStack st{0, 0, 0, 0};
    int cur = 0;
    unsigned long long ovf = 0;  // lanes whose scene-tree pushes were dropped (see lane_walk)
    unsigned fm = 0;             // few-leaf mask (few_mask)
    int pcap = kMaxStack;        // push bound of the tree being walked (uniform)
    {
        int code = 0;
        const bool scene = use_scene(A, fast, c);
        const bool hr = enter_root(A, r, inv, c, tl, code);  // code is the same in every lane
        const unsigned long long mr = __ballot(active && !scene && hr), ms = __ballot(active && scene);
        if (ms && A.nfew > 0) fm = few_mask(A, r, inv);
        cur = uni(code);
        m = mr;
        if (ms) {  // scene-tree lanes first; reference-tree lanes (if any) follow as if overflowed
            ovf = mr;
            cur = A.troot;
            m = ms;
            pcap = min(kMaxStack, A.scene_stack);
        }
    }
    unsigned long long done = 0;
    for (;;) {
        if (m == 0) {
            if (st.sp == 0) {
                if (!ovf) return;
                // scene-tree pushes were dropped for the lanes in ovf: they walk the
                // reference tree from its root (with their best hits so far)
                int code = 0;
                const bool hr = enter_root(A, r, inv, c, tl, code);
                m = __ballot(lane_in(ovf) && hr) & ~done;
                ovf = 0;
                pcap = kMaxStack;
                cur = uni(code);
                continue;
            }
            st.pop(cur, m);
            cur = uni(cur);
            if (SHADOW) m &= ~done;
            continue;
        }
        if (COUNT && lane_in(m)) wc.nodes++;
        if (WSTAT) wc.wnodes += lane_id() == 0 ? 1u : 0u;
        const unsigned uc = static_cast<unsigned>(cur);
        Kids k{0, 0, 0.f, 0.f, false, false};
        int start = 0, count = 0;
        bool item_in = true;
        if ((uc & (kTopLeaf | kItem)) == (kTopLeaf | kItem)) {
            item_in = enter_item(A, uc, r, inv, start, count);
            start = uni(start);
            count = uni(count);
        } else if (uc & kTopLeaf) {
            const int4 lf = A.tleaf[uc & 0x0fffffffu];
            start = uni(lf.x);
            count = uni(lf.y);
            k.ca = uni(lf.z);
            k.ha = (k.ca != kNoChild) && lane_in(m);  // local root: entered with the leaf
        } else if (uc & kLeaf) {
            start = static_cast<int>((uc >> 6) & 0x3fffffu);
            count = static_cast<int>(uc & 0x3fu);
            if (uc & kItem) {  // few-leaf item
                item_in = (fm >> (count >> 3)) & 1u;
                count &= 7;
            }
        } else if (uc & kLocal) {
            // wide node: children ordered by the entry parameters of the first lane
            // that enters any of them; the rest pushed far to near
            // a kPair node (uniform): both records' children, up to 8
            constexpr int NK = !MT && kWide8 ? 8 : 4;
            Kids4 wk[2];
            wk[0] = wide_kids<MT>(A, uc, c, tl, lane_in(m));
            if (NK == 8) wk[1] = wide_kids_hi<MT>(A, uc, c, tl, lane_in(m));
            unsigned long long wm[NK];
            float key[NK];
            int code[NK];
            unsigned long long any = 0;
#pragma unroll
            for (int s2 = 0; s2 < NK; ++s2) {
                wm[s2] = __ballot(wk[s2 >> 2].t[s2 & 3] < INFINITY);
                any |= wm[s2];
            }
            const int rep = any ? __builtin_ctzll(any) : 0;
#pragma unroll
            for (int s2 = 0; s2 < NK; ++s2) {
                const Kids4& w = wk[s2 >> 2];
                key[s2] = wm[s2] ? __int_as_float(__builtin_amdgcn_readlane(__float_as_int(w.t[s2 & 3]), rep)) : INFINITY;
                code[s2] = uni(w.code[s2 & 3]);
                if (wm[s2] && !(key[s2] < INFINITY)) key[s2] = 3.0e38f;  // the representative lane misses it
            }
#define RT_CAS3(i, j)                                                                   \
    if (key[j] < key[i]) {                                                              \
        const float t_ = key[i]; key[i] = key[j]; key[j] = t_;                          \
        const int c_ = code[i]; code[i] = code[j]; code[j] = c_;                        \
        const unsigned long long m_ = wm[i]; wm[i] = wm[j]; wm[j] = m_;                 \
    }
            if (NK == 8) {
                RT_CAS3(0, 1) RT_CAS3(2, 3) RT_CAS3(4, 5) RT_CAS3(6, 7) RT_CAS3(0, 2) RT_CAS3(1, 3) RT_CAS3(4, 6)
                RT_CAS3(5, 7) RT_CAS3(1, 2) RT_CAS3(5, 6) RT_CAS3(0, 4) RT_CAS3(1, 5) RT_CAS3(2, 6) RT_CAS3(3, 7)
                RT_CAS3(2, 4) RT_CAS3(3, 5) RT_CAS3(1, 2) RT_CAS3(3, 4) RT_CAS3(5, 6)
            } else {
                RT_CAS3(0, 1) RT_CAS3(2, 3) RT_CAS3(0, 2) RT_CAS3(1, 3) RT_CAS3(1, 2)
            }
#undef RT_CAS3
#pragma unroll
            for (int s2 = NK - 1; s2 >= 1; --s2)
                if (wm[s2]) {
                    if (st.sp < pcap) st.push(code[s2], wm[s2]);
                    else ovf |= wm[s2];  // scene tree only: local trees fit their bound
                }
            cur = code[0];
            m = wm[0];
            continue;
        } else {
            k = ref_kids(A, uc, r, inv, c, tl, lane_in(m), fast);
            k.ca = uni(k.ca);
            k.cb = uni(k.cb);
        }
        if (count > 0) {
            bool live = lane_in(m) && item_in;
            for (int i = 0; i < count; ++i) {
                const PrimRec g = load_prim(A.prims, start + i);
                if (WSTAT) wc.wtests += lane_id() == 0 ? 1u : 0u;
                if (live) {
                    if (COUNT) wc.tests++;
                    if (SHADOW) {
                        if (try_shadow<MT>(g, r, lim_shadow)) {
                            shadow = true;
                            live = false;
                        }
                    } else {
                        try_closest<MT>(g, start + i, r, b);
                    }
                }
                if (SHADOW && __ballot(live) == 0) break;
            }
            if (SHADOW) {
                done = __ballot(shadow);
                if (k.ha && shadow) k.ha = false;
            } else {
                tl = rta::t_limit(b.d, c.rdl);
            }
        }
        const unsigned long long ma = __ballot(k.ha), mb = __ballot(k.hb);
        if (ma && mb) {
            // near first for the wave: the child the first lane of both masks enters sooner
            const int rep = __builtin_ctzll(ma & mb ? (ma & mb) : ma);
            const float ra = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(k.ta), rep));
            const float rb = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(k.tb), rep));
            const bool a_first = !(rb < ra);
            if (st.sp < kMaxStack) st.push(a_first ? k.cb : k.ca, a_first ? mb : ma);
            cur = a_first ? k.ca : k.cb;
            m = a_first ? ma : mb;
        } else if (ma) {
            cur = k.ca;
            m = ma;
        } else if (mb) {
            cur = k.cb;
            m = mb;
        } else {
            m = 0;
        }
    }
}

// One 8x8 tile per wave (lane l: pixel (l&7, l>>3) of the tile).
__device__ __forceinline__ PixelCoord tile_pixel(const KParams& kp, int tile) {
    const int lane = threadIdx.x & 63;
    PixelCoord pc;
    pc.x = (tile % kp.tiles_x) * 8 + (lane & 7);
    pc.r = (tile / kp.tiles_x) * 8 + (lane >> 3);
    pc.active = pc.x < kp.width && pc.r < kp.out_rows;
    pc.y = pc.active ? image_row(kp, pc.r) : 0;
    pc.active = pc.active && pc.y < kp.height;
    return pc;
}

// Diagnostics (TIMED k_accel): one record of kTileRec u64 per tile:
//   [0] start, [1] end (100 MHz wall clock), [2] node steps and [3] tests
//   summed over the wave's lanes, [4], [5] their per-lane maxima,
//   [6 + s] wave clock ticks and [14 + s] node steps summed over lanes of walk
//   slot s = 2 * bounce + (0 closest, 1 shadow), bounce < 4, [22] leaf-loop and
//   [23] node-step iterations of the wave (all walks).
constexpr int kTileRec = 24;

// Ray compaction (rt_set_tail): queue entries per 64x64-pixel region.
constexpr int kTailRegion = 64 * 64;
constexpr size_t kTailAutoItems = 8192;  // RT_TAIL_AUTO threshold
#ifndef RT_TAIL_ONESHOT
#define RT_TAIL_ONESHOT 1
#endif
// k_accel_tail grid: one wave per possible chunk (64 per region), each taking one, or a
// resident grid striding over the chunks.
constexpr bool kTailOneShot = RT_TAIL_ONESHOT != 0;


// Cost-ordered dispatch (rt_set_schedule, k_tile_order): 32 half-octave
// buckets of a tile's work; the render kernel counts them per group of
// kOrderThreads tiles (one k_tile_order workgroup each).
constexpr int kOrderBuckets = 32, kOrderThreads = 256;
// lane_walk_any defaults (rt_debug_split)
constexpr int kSplitMax = 16, kSplitGroup = 8;
constexpr int kMtWalkFrom = 1 << 16;      // auto walk policy of Moller-Trumbore frames: all packets
constexpr int kMtPacketMaxNodes = 1024;  // ... over reference trees of fewer nodes (walk_from)
// the heaviest tiles of the cost order as several waves (rt_debug_heavy)
constexpr int kHeavyTiles = -1, kHeavyParts = 4, kHeavyAutoSlots = 2;  // -1: auto
// latency mode: frames of at most this many tiles per wave slot (16 per CU). 12: the car's
// 3840x2160 half share (64,800 tiles) waited 0.360 ms with it against 0.318 without, its
// quarter share (32,640) 0.19 against 0.27 (profiles/r05r_share_sweep.json)
constexpr int kLatencyMaxSlots = 12;
constexpr unsigned kXcds = 8;  // MI355X: 8 XCDs, workgroups dealt round-robin

__device__ __forceinline__ int work_bucket(unsigned c) {
    if (c < 2u) return 0;
    const int l = 31 - __builtin_clz(c);  // >= 1
    return min(kOrderBuckets - 1, 2 * l - 1 + static_cast<int>((c >> (l - 1)) & 1u));
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

__device__ __forceinline__ void walk_rec(unsigned long long* rec, int slot, const WalkCount& before,
                                         const WalkCount& after, unsigned long long ticks) {
    if (!rec || slot >= 8) return;
    const unsigned long long n = wave_sum(after.nodes - before.nodes);
    if ((threadIdx.x & 63) == 0) {
        rec[6 + slot] = ticks;
        rec[14 + slot] = n;
    }
}

// One bounce of gpu_shader.comp:450-517 for a wave's rays: closest hit, background
// on a miss, the shadow ray, then Phong and the mirror ray (shade_bounce).
// bg_y() gives the lane's image row (recomputed, not kept live through the walks).
template <bool COUNT, bool SPEC, bool COST, bool MT, bool SPLIT, class BgY>
__device__ __forceinline__ void bounce_step(const AccelPtrs& A, const float4* __restrict__ mat, const KParams& kp,
                                            int depth, Ray& ray, bool& alive, V& acc, V& att, BgY bg_y, int* stk,
                                            unsigned short* stt, int cap, WalkCount& wc, unsigned long long* rec,
                                            int lane_from, int shadow_from) {
    Best best{1e20f, 0x7fffffff, 0.f, -1};
    bool unused = false;
    const bool lane_mode = depth >= lane_from;  // wave-uniform
    WalkCount w0 = wc;
    unsigned long long c0 = COUNT ? clock64() : 0;
    if (lane_mode)
        lane_walk_any<false, COST || COUNT, COUNT, SPEC, MT, SPLIT>(A, ray, alive, 0.f, best, unused, stk, stt,
                                                                    blockDim.x, cap, wc);
    else
        packet_walk<false, COST || COUNT, COUNT, MT>(A, ray, alive, 0.f, best, unused, wc);
    if (COUNT) walk_rec(rec, 2 * depth, w0, wc, clock64() - c0);
    if (alive && best.slot < 0) {
        acc = acc + mulv(att, background(kp, bg_y()));
        alive = false;
    }
    // The shadow ray; the hit's normal and material are fetched again after the
    // shadow walk rather than kept live through it (register pressure).
    Ray sr{mk(0.f, 0.f, 0.f), mk(0.f, 0.f, 1.f)};
    float ld = 0.f;
    if (alive) {
        const V hp = hit_point(ray, best.t);
        const V hn = shape_normal(load_prim(A.prims, best.slot), hp);
        sr = Ray{hp + hn * kp.shadow_off, normalize(kp.light_pos - hp)};
        ld = dist(kp.light_pos, hp);
    }
    bool shadow = false;
    Best dummy{0.f, 0, 0.f, -1};
    w0 = wc;
    c0 = COUNT ? clock64() : 0;
    if (depth >= shadow_from)
        lane_walk_any<true, COST || COUNT, COUNT, SPEC, MT, SPLIT>(A, sr, alive, gmin(ld, 1e20f), dummy, shadow, stk,
                                                                   stt, blockDim.x, cap, wc);
    else
        packet_walk<true, COST || COUNT, COUNT, MT>(A, sr, alive, gmin(ld, 1e20f), dummy, shadow, wc);
    if (COUNT) walk_rec(rec, 2 * depth + 1, w0, wc, clock64() - c0);
    if (alive) {
        const PrimRec g = load_prim(A.prims, best.slot);
        const V hp = hit_point(ray, best.t);
        alive = shade_bounce(kp, ray, hp, shape_normal(g, hp), load_mat(mat, A.prim_shape[best.slot]), shadow, acc,
                             att, 1e-3f);
    }
}

// Walk counts (node steps, tests) are kept when COST: they are the cost that
// orders a later dispatch (rt_set_schedule). COUNT adds the per-walk records.
template <bool COUNT, bool SPEC, bool COST = true, bool TAIL = false, bool MT = false, bool QUEUE = TAIL>
__device__ void accel_tile(const AccelPtrs& A, const float4* __restrict__ mat, const KParams& kp, int tile,
                           int part, int* stk, unsigned short* stt, int cap, WalkCount& wc,
                           unsigned long long* rec, bool heavy) {
    // the heaviest slots (lane_k) may walk their camera rays / shadows per lane (lane_k_mode)
    const int lane_from = heavy && (kp.lane_k_mode & 1) ? 0 : kp.lane_from_depth;
    const int shadow_from = heavy && (kp.lane_k_mode & 2) ? 0 : kp.shadow_lane_from;
    // part > 0: this wave renders band part - 1 of the tile (64 / heavy_parts lanes)
    const bool mine = part == 0 || ((threadIdx.x & 63) * kp.heavy_parts >> 6) == part - 1;
    // Pixel coordinates and the background are recomputed where needed rather than
    // kept live through the walks (register pressure: they would be spilled).
    Ray ray;
    bool alive;
    {
        const PixelCoord pc = tile_pixel(kp, tile);
        ray = primary_ray(kp, pc.x, pc.y);
        alive = pc.active && mine;
    }
    V acc = mk(0.f, 0.f, 0.f), att = mk(1.f, 1.f, 1.f);
    bool deferred = false;  // the lane's remaining bounces run in k_accel_tail
    if (kp.root_ok) {
        // The root's exact test (gpu_shader.comp:386-395) from the kernel arguments: a camera
        // ray that misses it hits nothing in any walk (every leaf box lies inside the root's
        // for the scene tree; the reference walk starts there), so it takes the background
        // without the walk's dependent loads -- the sky tiles of a frame. root_ok 2: the
        // boxes were grown on the device (rt_animate), read the root's from anodes.
        V rlo = mk(kp.root_lo[0], kp.root_lo[1], kp.root_lo[2]), rhi = mk(kp.root_hi[0], kp.root_hi[1], kp.root_hi[2]);
        if (kp.root_ok == 2) {
            const float4 a = A.anodes[4 * static_cast<size_t>(A.N - 1)], b = A.anodes[4 * static_cast<size_t>(A.N - 1) + 1];
            rlo = mk(a.x, a.y, a.z);
            rhi = mk(b.x, b.y, b.z);
        }
        const bool in = ray_aabb(ray.o, inv_dir(ray.d), rlo, rhi);
        if (alive && !in) {
            acc = background(kp, tile_pixel(kp, tile).y);
            alive = false;
        }
    }
    for (int depth = 0; depth < kp.maxBounces; ++depth) {
        if (__ballot(alive) == 0) break;
        bounce_step<COUNT, SPEC, COST, MT, TAIL || RT_SPLIT_ALL>(A, mat, kp, depth, ray, alive, acc, att,
                                       [&]() { return tile_pixel(kp, tile).y; }, stk, stt, cap, wc, rec, lane_from,
                                       shadow_from);
        if (TAIL && QUEUE && depth + 1 == kp.tail_from && __popcll(__ballot(alive)) <= kp.tail_max_lanes) {
            // Compaction: the rays still alive go to the tail queue (one atomic per wave)
            // per 64x64-pixel region (8x8 tiles), so a tail wave's rays come from one area
            const unsigned long long m = __ballot(alive);
            if (m) {
                const int rid = (tile / kp.tiles_x / 8) * kp.tail_rx + (tile % kp.tiles_x) / 8;
                int base = 0;
                if ((threadIdx.x & 63) == 0) base = rid * kTailRegion + atomicAdd(kp.tail_count + rid, __popcll(m));
                base = __shfl(base, 0);
                if (alive) {
                    const int lane = threadIdx.x & 63;
                    const int pos = base + __popcll(m & ((1ull << lane) - 1ull));
                    const PixelCoord pc = tile_pixel(kp, tile);
                    float4* q = kp.tail_queue + 3 * static_cast<size_t>(pos);
                    q[0] = make_float4(ray.o.x, ray.o.y, ray.o.z, acc.x);
                    q[1] = make_float4(ray.d.x, ray.d.y, ray.d.z, acc.y);
                    q[2] = make_float4(att.x, att.y, att.z, acc.z);
                    // unsigned, as k_accel_tail decodes it (launch() keeps width * rows < 2^32)
                    kp.tail_px[pos] = static_cast<int>(static_cast<unsigned>(pc.r) * static_cast<unsigned>(kp.width) +
                                                       static_cast<unsigned>(pc.x));
                }
            }
            deferred = alive;
            break;
        }
    }
    const PixelCoord pc = tile_pixel(kp, tile);
    if (pc.active && mine && !deferred) store_px(kp, pc.r, pc.x, make_float4(acc.x, acc.y, acc.z, 1.0f));
}

// PERSISTENT: each wave pulls tiles from one device counter until none is
// left (every wave reaches the exit); otherwise one tile per wave. TIMED
// writes each tile's start/end wall clock and walk counts (diagnostics only).
// At most 128 VGPRs: four waves per SIMD, which the LDS stacks also fit
// (accel.h, kLaneStack).
#ifndef RT_UNIFORM_TILE
#define RT_UNIFORM_TILE 0  // tile / part / slot forced into SGPRs in every instance: car +-0, config 2 -1 %,
                           // latency instance 4 -> 9 spilled VGPRs (r04zz14); off
#endif
#ifndef RT_ACCEL_ATTR
#define RT_ACCEL_ATTR __attribute__((amdgpu_waves_per_eu(4)))
#endif
// COST = false: no walk counters (their registers: 12 -> 3 spilled VGPRs). REC: the
// dispatch records each tile's cost for the next order (rt_set_schedule); without COST
// it can only record the wall-time cost (kp.cost_time), which needs no counters.
// TAIL: queue the rays alive after bounce tail_from - 1 for k_accel_tail (rt_set_tail).
template <bool PERSISTENT, bool TIMED, bool SPEC, bool COST = true, bool TAIL = false, bool MT = false,
          bool REC = COST, bool QUEUE = TAIL>
__global__ __launch_bounds__(kBlock) RT_ACCEL_ATTR void k_accel(AccelPtrs A, const float4* __restrict__ mat, KParams kp) {
    extern __shared__ int lds_stack[];
    // per-lane stacks, entry j of lane i at [j * blockDim.x + i]: codes, then bf16 entry parameters
    int* stk = lds_stack + threadIdx.x;
    unsigned short* stt =
        reinterpret_cast<unsigned short*>(lds_stack + static_cast<size_t>(kp.lane_stack) * blockDim.x) + threadIdx.x;
    const int lane = threadIdx.x & 63;
    int tile = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (PERSISTENT) {
        int t = 0;
        if (lane == 0) t = atomicAdd(kp.tile_counter, 1);
        tile = __shfl(t, 0);
    }
    // dispatch slots: the heavy_k heaviest tiles (the head of the cost order) as heavy_parts
    // waves each, then the rest of the order one wave per tile
    const int hs = kp.heavy_k * kp.heavy_parts;
    while (tile < kp.tiles + hs - kp.heavy_k) {
        unsigned long long t0 = 0;
        if (TIMED || (REC && kp.cost_time)) t0 = wall_clock64();
        int part = 0;
        const int slot = REC || RT_UNIFORM_TILE ? __builtin_amdgcn_readfirstlane(tile) : tile;
        if (kp.tile_order) {  // dispatch order -> image tile (a permutation)
            if (tile < hs) {
                part = tile % kp.heavy_parts + 1;
                tile = kp.tile_order[tile / kp.heavy_parts];
            } else {
                tile = kp.tile_order[tile - hs + kp.heavy_k];
            }
        }
        if (REC || RT_UNIFORM_TILE) {  // wave-uniform: kept in SGPRs through the walks
            tile = __builtin_amdgcn_readfirstlane(tile);
            part = __builtin_amdgcn_readfirstlane(part);
        }
        WalkCount wc{0u, 0u, 0u, 0u};
        // a split tile's parts stamp records tiles + slot (rt_debug_tile_times with room for them)
        unsigned long long* rec =
            TIMED ? kp.tile_times + kTileRec * static_cast<size_t>(part > 0 ? kp.tiles + slot : tile) : nullptr;
        accel_tile<TIMED, SPEC, COST, TAIL, MT, QUEUE>(A, mat, kp, tile, part, stk, stt, kp.lane_stack, wc, rec,
                                                slot < kp.lane_k);
        if (TIMED) {
            const unsigned long long t1 = wall_clock64();
            unsigned long long sn = wc.nodes, st = wc.tests, mn = wc.nodes, mt = wc.tests;
            for (int off = 32; off > 0; off >>= 1) {
                sn += __shfl_xor(sn, off);
                st += __shfl_xor(st, off);
                mn = max(mn, __shfl_xor(mn, off));
                mt = max(mt, __shfl_xor(mt, off));
            }
            const unsigned long long wn = wave_sum(wc.wnodes), wt = wave_sum(wc.wtests);
            if (lane == 0) {
                unsigned long long* o = rec;
                o[22] = wt;
                o[23] = wn;
                o[0] = t0;
                o[1] = t1;
                o[2] = sn;
                o[3] = st;
                o[4] = mn;
                o[5] = mt;
            }
        }
        if (REC && kp.tile_cost) {
            // the tile's cost: its wave's wall time in 40 ns units (cost_time) -- the length
            // of its dependent chain, which a packet walk's union of nodes stretches beyond
            // what its lanes' own steps count -- or those lanes' node steps + tests. Ranking by
            // time: car waited frame 0.2504 -> 0.2247 ms with the latency mode's split below,
            // in flight -1 % (r04v, profiles/r04v_*)
            const unsigned long long work = !COST || kp.cost_time
                                                ? (wall_clock64() - t0) >> 2
                                                : wave_sum(static_cast<unsigned long long>(wc.nodes) + wc.tests);
            unsigned wk = static_cast<unsigned>(work < 0xffffffffull ? work : 0xffffffffull);
            bool rec = part == 0;
            if (part > 0 && lane == 0) {
                // a split tile's cost is the sum of its parts' (one record per tile, by the
                // part that finishes last). Round 3 took the first band's times the bands: a
                // heavy tile whose first band is sky then ranked low, ran whole and late,
                // ranked high again, and so on (the latency-mode car waited frame 0.25 or
                // 0.287 ms by the phase of that cycle, r04l)
                // One 64-bit atomic carries both the count and the sum, so the last part reads
                // the total from its own return value: no agent-scope fences (each writes back
                // or invalidates the XCD's L2, the cost that sank the in-kernel dilation).
                const int hk = slot / kp.heavy_parts;
                const unsigned long long old =
                    atomicAdd(&kp.heavy_acc[hk], (1ull << 56) | static_cast<unsigned long long>(wk));
                if (static_cast<int>(old >> 56) == kp.heavy_parts - 1) {
                    const unsigned long long sum = (old & ((1ull << 56) - 1)) + wk;
                    wk = static_cast<unsigned>(sum < 0xffffffffull ? sum : 0xffffffffull);
                    rec = true;
                }
            }
            if (lane == 0 && rec) {
                kp.tile_cost[tile] = wk;
                atomicAdd(&kp.sched_hist[(tile / kOrderThreads) * kOrderBuckets + work_bucket(wk)], 1u);
            }
        }
        if (!PERSISTENT) break;
        int t = 0;
        if (lane == 0) t = atomicAdd(kp.tile_counter, 1);
        tile = __shfl(t, 0);
    }
}

// The queued rays' remaining bounces (rt_set_tail): a resident grid, wave w
// taking queue chunks w, w + G, ... of 64 rays. The same bounce arithmetic as
// k_accel; a ray's walk does not depend on the other lanes, so compacting rays
// from different tiles into one wave leaves every pixel's value unchanged.
__device__ __forceinline__ int wave_sum_int(int v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

template <bool SPEC>
__global__ __launch_bounds__(kBlock) RT_ACCEL_ATTR void k_accel_tail(AccelPtrs A, const float4* __restrict__ mat,
                                                                      KParams kp) {
    extern __shared__ int lds_stack[];
    int* stk = lds_stack + threadIdx.x;
    unsigned short* stt =
        reinterpret_cast<unsigned short*>(lds_stack + static_cast<size_t>(kp.lane_stack) * blockDim.x) + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const int waves = gridDim.x * (blockDim.x >> 6);
    // chunks of 64 queued rays, region after region: total chunk count first
    int total = 0;
    for (int b = 0; b < kp.tail_regions; b += 64) {
        const int cnt = b + lane < kp.tail_regions ? kp.tail_count[b + lane] : 0;
        total += wave_sum_int((cnt + 63) >> 6);
    }
    // (r05: the chunks in XCD-contiguous eighths, each XCD's L2 on one band of regions,
    // measured slower on config 5: 2.734 against 2.689 ms in flight, 3.419 against 3.292
    // solo; profiles/r05zs_abf_tail_xcd_negative_*.json)
    for (int chunk = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); chunk < total; chunk += waves) {
        // the region holding chunk: running prefix of the regions' chunk counts
        int rid = 0, first = 0, n = 0, acc0 = 0;
        for (int b = 0; b < kp.tail_regions; b += 64) {
            const int cnt = b + lane < kp.tail_regions ? kp.tail_count[b + lane] : 0;
            const int ch = (cnt + 63) >> 6;
            int incl = ch;  // inclusive prefix over the 64 lanes
            for (int off = 1; off < 64; off <<= 1) {
                const int y = __shfl_up(incl, off);
                if (lane >= off) incl += y;
            }
            const unsigned long long hit = __ballot(acc0 + incl > chunk && acc0 + incl - ch <= chunk && ch > 0);
            if (hit) {
                const int l = __builtin_ctzll(hit);
                rid = b + l;
                first = __shfl(acc0 + incl - ch, l);
                n = __shfl(cnt, l);
                break;
            }
            acc0 += __shfl(incl, 63);
        }
        const int k = (chunk - first) * 64 + lane;  // index within the region
        bool alive = k < n;
        const int i = rid * kTailRegion + k;
        Ray ray{mk(0.f, 0.f, 0.f), mk(0.f, 0.f, 1.f)};
        V acc = mk(0.f, 0.f, 0.f), att = mk(1.f, 1.f, 1.f);
        int r = 0, x = 0;
        if (alive) {
            const float4* q = kp.tail_queue + 3 * static_cast<size_t>(i);
            const float4 q0 = q[0], q1 = q[1], q2 = q[2];
            const unsigned px = static_cast<unsigned>(kp.tail_px[i]);
            ray = Ray{mk(q0.x, q0.y, q0.z), mk(q1.x, q1.y, q1.z)};
            acc = mk(q0.w, q1.w, q2.w);
            att = mk(q2.x, q2.y, q2.z);
            r = static_cast<int>(px / static_cast<unsigned>(kp.width));
            x = static_cast<int>(px - static_cast<unsigned>(r) * static_cast<unsigned>(kp.width));
        }
        const bool have = alive;
        WalkCount wc{0u, 0u, 0u, 0u};
        for (int depth = kp.tail_from; depth < kp.maxBounces; ++depth) {
            if (__ballot(alive) == 0) break;
            bounce_step<false, SPEC, false, false, true>(A, mat, kp, depth, ray, alive, acc, att,
                                            [&]() { return image_row(kp, r); }, stk, stt, kp.lane_stack, wc, nullptr,
                                            kp.lane_from_depth, kp.shadow_lane_from);
        }
        if (have) store_px(kp, r, x, make_float4(acc.x, acc.y, acc.z, 1.0f));
        if (kTailOneShot) break;  // one chunk per wave: no loop-carried state
    }
    if (blockIdx.x == 0)
        for (int b = threadIdx.x; b < kp.tail_counters; b += blockDim.x) kp.tail_count_next[b] = 0;
}

__global__ void k_pack_prims(const float4* __restrict__ geo_lin, const int* __restrict__ prim_shape,
                             const int* __restrict__ prim_seq, int P, float4* __restrict__ prims) {
    int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= P) return;
    store_prim(prims, j, pack_prim(load_rec(geo_lin, prim_shape[j]), prim_seq[j]));
}

// Dispatch order for the next frame (rt_set_schedule): tiles sorted by the
// work their waves did in the last dispatch (node steps + primitive tests over
// the 64 lanes; unlike a duration it does not depend on what ran beside the
// tile), most first, as a counting sort over 32 half-octave buckets. The render
// kernel counts each group of kOrderThreads tiles' buckets (hist rows); group
// j's workgroup here places its tiles after every tile of a heavier bucket and
// after the tiles of the same bucket in groups < j (ranks inside a group by
// LDS atomics: order inside a bucket is arbitrary). Two histogram sets
// alternate by frame; this kernel zeroes the rows the next frame counts into.
__global__ __launch_bounds__(kOrderThreads) void k_tile_order(const unsigned* __restrict__ cost, int n,
                                                              const unsigned* __restrict__ hist,
                                                              unsigned* __restrict__ next, int next_words,
                                                              int* __restrict__ order, int xcd) {
    constexpr int kPart = kOrderThreads / kOrderBuckets;  // threads per bucket for the row sums
    __shared__ unsigned tot[kPart][kOrderBuckets], pre[kPart][kOrderBuckets];
    __shared__ unsigned start[kOrderBuckets], rank[kOrderBuckets], base[kOrderBuckets], count[kOrderBuckets];
    const int t = threadIdx.x, j = blockIdx.x, groups = gridDim.x;
    {
        const int b = t % kOrderBuckets, part = t / kOrderBuckets;
        unsigned a = 0, p = 0;
#pragma unroll 8
        for (int r = part; r < groups; r += kPart) {
            const unsigned h = hist[r * kOrderBuckets + b];
            a += h;
            p += r < j ? h : 0u;
        }
        tot[part][b] = a;
        pre[part][b] = p;
    }
    for (int w = j * kOrderThreads + t; w < next_words; w += groups * kOrderThreads) next[w] = 0u;
    __syncthreads();
    if (t < 64) {  // one wave: bucket sums, then a suffix scan (buckets from the most work down)
        unsigned a = 0, p = 0;
        if (t < kOrderBuckets) {
#pragma unroll
            for (int k = 0; k < kPart; ++k) {
                a += tot[k][t];
                p += pre[k][t];
            }
            rank[t] = 0u;
        }
        unsigned x = a;  // inclusive sum over buckets >= t
        for (int off = 1; off < kOrderBuckets; off <<= 1) {
            const unsigned y = __shfl_down(x, off);
            if (t + off < kOrderBuckets) x += y;
        }
        if (t < kOrderBuckets) {
            start[t] = x - a + p;
            base[t] = x - a;
            count[t] = a;
        }
    }
    __syncthreads();
    const int i = j * kOrderThreads + t;
    if (i < n) {
        const int b = work_bucket(cost[i]);
        const unsigned pos = start[b] + atomicAdd(&rank[b], 1u);
        if (!xcd) {
            order[pos] = i;
        } else {
            // Workgroups go to the 8 XCDs round-robin (slot s on XCD s mod 8), and each
            // XCD has its own L2. Deal the bucket's tiles (in group order, i.e. screen
            // bands) as 8 contiguous chunks, chunk c to the slots base + c, base + 8 + c,
            // ...: each XCD walks one band of the bucket at a time, and every XCD still
            // gets an eighth of every bucket (same longest-first balance).
            const unsigned cnt = count[b], q = cnt / kXcds, rem = cnt % kXcds, pb = pos - base[b];
            unsigned c, k;
            if (pb < rem * (q + 1)) {
                c = pb / (q + 1);
                k = pb % (q + 1);
            } else {
                c = rem + (pb - rem * (q + 1)) / q;
                k = (pb - rem * (q + 1)) % q;
            }
            order[base[b] + kXcds * k + c] = i;
        }
    }
}

// The cost order's input dilated (rt_debug_cost_dilate): each tile's cost replaced by
// the largest within r tiles in x and y, and the per-group bucket rows k_tile_order
// reads recounted from those. A camera that moved since the costs were recorded sees
// its heavy tiles a few tiles away from where they were; ranking their neighbourhood
// high too puts them early anyway. (r05: dilating in the render kernel instead -- each
// tile's cost raised into its 3 x 3 neighbourhood by atomic max, the last recorder of a
// neighbour counting its bucket -- took the moving car frame from 0.296 to 2.77 ms: the
// agent-scope fences between the two phases, per tile, across 8 XCDs; r05zu.)
__global__ __launch_bounds__(kOrderThreads) void k_cost_dilate(const unsigned* __restrict__ cost, int n, int tiles_x,
                                                               int r, unsigned* __restrict__ out,
                                                               unsigned* __restrict__ hist) {
    __shared__ unsigned cnt[kOrderBuckets];
    const int t = threadIdx.x, i = blockIdx.x * kOrderThreads + t;
    if (t < kOrderBuckets) cnt[t] = 0u;
    __syncthreads();
    if (i < n) {
        const int x = i % tiles_x, y = i / tiles_x, rows = (n + tiles_x - 1) / tiles_x;
        unsigned m = 0u;
        for (int yy = max(0, y - r); yy <= min(rows - 1, y + r); ++yy)
            for (int xx = max(0, x - r); xx <= min(tiles_x - 1, x + r); ++xx) {
                const int j = yy * tiles_x + xx;
                if (j < n) m = max(m, cost[j]);
            }
        out[i] = m;
        atomicAdd(&cnt[work_bucket(m)], 1u);
    }
    __syncthreads();
    if (t < kOrderBuckets) hist[blockIdx.x * kOrderBuckets + t] = cnt[t];
}

// ---------------------------------------------------------------------------
// Device animation (rt_animate): updateScene + updateBVH on the device.

// Wall::end (src/shapes/wall.hpp:16-31), host glm operation order.
__host__ __device__ V wall_end(const FlatShape& s) {
    const V n = mk(s.planeNormal.x, s.planeNormal.y, s.planeNormal.z);
    const V t1 = fabsf(n.x) > fabsf(n.y) ? normalize(mk(-n.z, 0.f, n.x)) : normalize(mk(0.f, -n.z, n.y));
    const V t2 = normalize(cross(n, t1));
    return (mk(s.wallStart.x, s.wallStart.y, s.wallStart.z) + t1 * s.wallWidth) + t2 * s.wallHeight;
}

// BoundingBox::growToInclude(shape) (BoundingBox.hpp:50-95) from an empty box:
// the points it adds, as a (lo, hi) pair; a shape that adds nothing leaves
// lo = +inf, hi = -inf.
__host__ __device__ void reference_box(const FlatShape& s, float lo[3], float hi[3]) {
    for (int a = 0; a < 3; ++a) {
        lo[a] = INFINITY;
        hi[a] = -INFINITY;
    }
    auto add = [&](V p) {
        const float v[3] = {p.x, p.y, p.z};
        for (int a = 0; a < 3; ++a) {
            lo[a] = v[a] < lo[a] ? v[a] : lo[a];
            hi[a] = hi[a] < v[a] ? v[a] : hi[a];
        }
    };
    if (s.type == RT_SPHERE) {
        const float r = s.sphereRadius;
        add(mk(s.sphereCenter.x + r, s.sphereCenter.y + r, s.sphereCenter.z + r));
        add(mk(s.sphereCenter.x - r, s.sphereCenter.y - r, s.sphereCenter.z - r));
    } else if (s.type == RT_WALL) {
        add(mk(s.wallStart.x, s.wallStart.y, s.wallStart.z));
        add(wall_end(s));
    } else if (s.type == RT_TRIANGLE) {
        if (isfinite(s.triP1.x) && isfinite(s.triP2.x) && isfinite(s.triP3.x)) {  // :52
            add(mk(s.triP1.x, s.triP1.y, s.triP1.z));
            add(mk(s.triP2.x, s.triP2.y, s.triP2.z));
            add(mk(s.triP3.x, s.triP3.y, s.triP3.z));
        }
    }
}

// CSR lists built by prepare_animation on the host. Per animated shape i:
//   slots  : its geo_leaf slots (bvhIndices positions)
//   prims  : its accelerator prim slots
//   wpos   : wide-record slots (4*w + s) of the local nodes above those prims
// Per reference node j that lists an animated shape (node_ids[j]):
//   node   : the animated shapes it lists (updateBVH's set, leaves + ancestors)
//   wn     : the wnodes child slots (2 * parent + side) that hold its box
//   item   : the scene-tree items (titems records) whose exact box is its box
struct AnimMaps {
    const int *ids, *slot_off, *slot_list, *prim_off, *prim_list, *wpos_off, *wpos_list;
    const int *node_ids, *node_off, *node_list;
    const int *wn_off, *wn_list, *item_off, *item_list;
    const int* ecls;       // per entry: its class when the accelerator was built (accel_bound.h)
    const int* prim_entry; // per accelerator prim: its shape's refit entry, -1 if none
    int count, nodes;
};
// the per-frame flag of a refit entry: the nodes listing it grow to hold it
// (rt_animate: updateBVH on the device; rt_update_shapes leaves the node boxes to
// rt_update_nodes, as a glBufferSubData of the shape records does)
// AF_BOX (with AF_GROW): the growth is the box the host passed for the entry (the union of
// several frames' growToInclude boxes: rtx::animate_deferred), not its current record's
enum { AF_GROW = 4, AF_BOX = 8 };

struct AnimOut {
    FlatShape* shapes;  // staging copy of the full shape array
    FlatNode* nodes;    // staging copy of the node array (authoritative boxes)
    float4 *geo_lin, *geo_leaf, *mat;
    float4* packed;                   // the packed node copies (k_pack_nodes layout)
    float4 *anodes, *lnodes, *prims;  // accelerator (null when off)
    float4 *wnodes, *titems;          // accelerator: per-parent child boxes, scene-tree items' exact boxes
    float4* pbox;                     // conservative box per prim (lo, hi), for the slot refit
    const int* prim_seq;
    float4* sbox;                     // per entry: reference box, conservative box (4 float4)
    float origin_lim;
    int mt;                           // the accelerator's wide nodes: kWideRecMt float cones, else kWideRec
    float mt_z[3];                    // MT accelerators: AccelHost::mt_z (the per-ray padding's centre Z)
    const int* prim_shape;            // accelerator: shape index per prim (AccelPtrs::prim_shape)
    int cone_cull;                    // rt_debug_cone_cull: 0 keeps every cone full
};

// One refit launch (k_refit) of flush_updates: what it reads from the pinned ring
// and how its workgroups split the work.
struct RefitArgs {
    const FlatShape* fresh;    // per entry: its current record (pinned, mapped)
    const int* flags;          // per entry: AF_GROW, AF_BOX (pinned)
    const float4* gbox;        // per entry with AF_BOX: its growth box (lo, hi; pinned), or null
    const FlatNode* nsrc;      // rt_update_nodes: the host's node records (pinned), or null
    int* report;               // pinned: set to 1 when an entry's bound changed kind
    unsigned* ctr;             // [0] workgroup tickets, [1] finished record workgroups, then the flags
    unsigned tbase, abase;     // their values before this launch
    int na, nd, nb;            // workgroups of the record, node-set and node roles
    const int4* dirty;         // slot refit work list (n_dirty entries after the nb node waves, + 1 end)
    int n_big;                 // its first n_big slots take a workgroup each, the rest a wave each
    const float4* dstatic;     // per dirty slot: the box of its prims outside the refit set (lo, hi)
    const int* dlist;          // the refit set's prims of each dirty slot (dirty[j].w ..)
    int n_dirty, rec;          // its length; the wide record size (kWideRec / kWideRecMt)
    const int* titem_ref;      // per scene-tree item: its reference leaf
    int n_items, N;
    int wait;                  // node / slot roles wait for the record role: 1 by tickets, 2 in start order
    int direct;                // node / slot roles derive the entries' boxes from `fresh` themselves
};

// A lane-strided loop over [b, e) in steps of 4 x 64 whose four loads are issued
// before any is used: a long range (a slot near a local root spans thousands of
// prims) then costs a memory latency per step, not per prim.
// nt threads (a wave or a workgroup), this one tid.
template <class Load, class Use>
__device__ __forceinline__ void range4(int b, int e, int tid, int nt, Load load, Use use) {
    for (int p0 = b + tid; p0 < e; p0 += 4 * nt) {
        decltype(load(0)) v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (p0 + nt * u < e) v[u] = load(p0 + nt * u);
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (p0 + nt * u < e) use(v[u]);
    }
}
template <class Load, class Use>
__device__ __forceinline__ void range4(int b, int e, int lane, Load load, Use use) {
    range4(b, e, lane, 64, load, use);
}

struct Box4 {
    float4 a, b;
};

__device__ __forceinline__ void wave_minmax(float lo[3], float hi[3]) {
    for (int off = 32; off > 0; off >>= 1)
        for (int a = 0; a < 3; ++a) {
            lo[a] = fminf(lo[a], __shfl_xor(lo[a], off));
            hi[a] = fmaxf(hi[a], __shfl_xor(hi[a], off));
        }
}

// wave_minmax over the workgroup (up to kRefitWaves waves; every thread gets the
// result); sh: LDS scratch of the workgroup, free again on return.
constexpr int kRefitWaves = 4;
constexpr int kRefitFlag0 = 16, kRefitFlags = 16;  // k_refit's all-done flags: ctr[16 + 16 k]
constexpr long long kDirectReads = 2048;           // rt_ctx::refit_mode auto
constexpr int kBigList = 256;                      // a slot's refit list a wave unions in one step
__device__ __forceinline__ void block_minmax(float lo[3], float hi[3], float (*sh)[6]) {
    wave_minmax(lo, hi);
    const int nw = blockDim.x >> 6;
    if (nw == 1) return;
    if ((threadIdx.x & 63) == 0)
        for (int a = 0; a < 3; ++a) {
            sh[threadIdx.x >> 6][a] = lo[a];
            sh[threadIdx.x >> 6][3 + a] = hi[a];
        }
    __syncthreads();
    for (int k = 0; k < nw; ++k)
        for (int a = 0; a < 3; ++a) {
            lo[a] = fminf(lo[a], sh[k][a]);
            hi[a] = fmaxf(hi[a], sh[k][3 + a]);
        }
    __syncthreads();
}

// Record role, one lane per refit entry: rewrites its records and derives its two
// boxes (the reference's growToInclude box when it grows the nodes, and the
// accelerator's conservative one) for the node and slot roles. The class of the
// bound is decided here, on the device: a shape whose bound changed kind since the
// build (a triangle collapsing to a sliver, a sphere going infinite) gets an
// infinite conservative box, so every box above it is entered and it is tested like
// an always-tested shape -- the frame stays exact -- and `report` asks the host to
// rebuild the accelerator for speed. The cones above the shape are the slot role's.
// The conservative box an entry's current record contributes to the boxes above it
// (b): its classify() box; empty if it was always tested since the build (no box
// above it); infinite if its bound changed kind since (every box above it then
// entered). Returns whether the kind changed.
__device__ bool entry_cbox(const AnimOut& o, const FlatShape& s, int was, rta::Box3& b) {
    const int cls = rta::classify(s, b, o.origin_lim, o.mt != 0);
    const bool changed = cls != was;
    if (was != rta::BOUNDED || cls != rta::BOUNDED)
        for (int a = 0; a < 3; ++a) {
            b.lo[a] = was != rta::BOUNDED ? INFINITY : -INFINITY;
            b.hi[a] = was != rta::BOUNDED ? -INFINITY : INFINITY;
        }
    return changed;
}

__device__ void refit_record(const AnimMaps& m, const AnimOut& o, const RefitArgs& r, int i) {
    if (i >= m.count) return;
    // Every map read first: the stores below may alias them as far as the compiler
    // knows, so a read after one would wait out its own latency, in a chain. The
    // first slot and prim of each list (most entries have one of each) are prefetched
    // with their dependants.
    const int id = m.ids[i], fl = r.flags[i], was = m.ecls[i];
    const int s0 = m.slot_off[i], s1 = m.slot_off[i + 1], p0 = m.prim_off[i], p1 = m.prim_off[i + 1];
    const int slot0 = s0 < s1 ? m.slot_list[s0] : 0;
    const int prim0 = o.anodes && p0 < p1 ? m.prim_list[p0] : 0;
    const int seq0 = o.anodes && p0 < p1 ? o.prim_seq[prim0] : 0;
    const FlatShape s = r.fresh[i];
    o.shapes[id] = s;
    const GeoRec g = pack_geo(s, id);
    store_geo(o.geo_lin + 5 * static_cast<size_t>(id), g);
    store_mat(o.mat, id, s.material);
    if (s0 < s1) store_geo(o.geo_leaf + 5 * static_cast<size_t>(slot0), g);
    for (int q = s0 + 1; q < s1; ++q) store_geo(o.geo_leaf + 5 * static_cast<size_t>(m.slot_list[q]), g);
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    if (fl & AF_BOX) {  // several frames' boxes, unioned on the host
        const float4 a = r.gbox[2 * static_cast<size_t>(i)], b = r.gbox[2 * static_cast<size_t>(i) + 1];
        lo[0] = a.x, lo[1] = a.y, lo[2] = a.z, hi[0] = b.x, hi[1] = b.y, hi[2] = b.z;
    } else if (fl & AF_GROW) {
        reference_box(s, lo, hi);  // else the nodes keep their boxes
    }
    float4* sb = o.sbox + 4 * static_cast<size_t>(i);
    sb[0] = make_float4(lo[0], lo[1], lo[2], 0.f);
    sb[1] = make_float4(hi[0], hi[1], hi[2], 0.f);
    if (!o.anodes) {
        sb[2] = make_float4(INFINITY, INFINITY, INFINITY, 0.f);
        sb[3] = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.f);
        return;
    }
    // rank in the reference walk (k_pack_prims)
    if (p0 < p1) store_prim(o.prims, prim0, pack_prim(g, seq0));
    for (int q = p0 + 1; q < p1; ++q) {
        const int p = m.prim_list[q];
        store_prim(o.prims, p, pack_prim(g, o.prim_seq[p]));
    }
    rta::Box3 b;
    if (entry_cbox(o, s, was, b)) *r.report = 1;  // the host rebuilds at its next flush
    const float4 c0 = make_float4(b.lo[0], b.lo[1], b.lo[2], 0.f), c1 = make_float4(b.hi[0], b.hi[1], b.hi[2], 0.f);
    sb[2] = c0;
    sb[3] = c1;
    if (was != rta::BOUNDED) return;  // always tested since the build: no box above it
    for (int q = p0; q < p1; ++q) {    // the prim's box for the slot refit
        float4* pb = o.pbox + 2 * static_cast<size_t>(q == p0 ? prim0 : m.prim_list[q]);
        pb[0] = c0;
        pb[1] = c1;
    }
}

// Node role, one wave per reference node listing a refit entry: the union of the
// entries' boxes (lanes stride the list, then a wave reduction), then one grow of
// the node's box - updateBVH's growToInclude of each listed shape, entries with
// AF_GROW only - and of its content box. A single writer per node: no atomics,
// and the min/max result is the same in any order (no stored value is NaN; a NaN
// coordinate adds nothing). The same lane writes the grown box through to every
// copy the kernels read: the packed node, the accelerator's exact box, its
// parent's child copy (wnodes: exact + content box) and the scene-tree items gated
// by it. Nodes listing no entry never change, so no other copy needs refreshing.
__device__ void grow_node(const AnimMaps& m, const AnimOut& o, const RefitArgs& r, int j, float (*sh)[6]) {
    const int tid = threadIdx.x;
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
    struct Two {
        Box4 ref, con;
    };
    range4(m.node_off[j], m.node_off[j + 1], tid, blockDim.x,
        [&](int q) {
            const int i = m.node_list[q];
            Two v;
            if (r.direct) {  // from the record itself (no wait for the record role)
                const FlatShape s = r.fresh[i];
                float rl[3] = {INFINITY, INFINITY, INFINITY}, rh[3] = {-INFINITY, -INFINITY, -INFINITY};
                if (r.flags[i] & AF_BOX) {
                    const float4 a = r.gbox[2 * static_cast<size_t>(i)], b = r.gbox[2 * static_cast<size_t>(i) + 1];
                    rl[0] = a.x, rl[1] = a.y, rl[2] = a.z, rh[0] = b.x, rh[1] = b.y, rh[2] = b.z;
                } else if (r.flags[i] & AF_GROW) {
                    reference_box(s, rl, rh);
                }
                rta::Box3 cb;
                if (o.anodes) entry_cbox(o, s, m.ecls[i], cb);
                else cb = rta::Box3{{INFINITY, INFINITY, INFINITY}, {-INFINITY, -INFINITY, -INFINITY}};
                v.ref = Box4{make_float4(rl[0], rl[1], rl[2], 0.f), make_float4(rh[0], rh[1], rh[2], 0.f)};
                v.con = Box4{make_float4(cb.lo[0], cb.lo[1], cb.lo[2], 0.f), make_float4(cb.hi[0], cb.hi[1], cb.hi[2], 0.f)};
            } else {
                const float4* sb = o.sbox + 4 * static_cast<size_t>(i);
                v.ref = Box4{sb[0], sb[1]};
                v.con = Box4{sb[2], sb[3]};
            }
            return v;
        },
        [&](const Two& v) {
            const float4 a = v.ref.a, b = v.ref.b, c = v.con.a, d = v.con.b;
            lo[0] = fminf(lo[0], a.x), lo[1] = fminf(lo[1], a.y), lo[2] = fminf(lo[2], a.z);
            hi[0] = fmaxf(hi[0], b.x), hi[1] = fmaxf(hi[1], b.y), hi[2] = fmaxf(hi[2], b.z);
            clo[0] = fminf(clo[0], c.x), clo[1] = fminf(clo[1], c.y), clo[2] = fminf(clo[2], c.z);
            chi[0] = fmaxf(chi[0], d.x), chi[1] = fmaxf(chi[1], d.y), chi[2] = fmaxf(chi[2], d.z);
        });
    block_minmax(lo, hi, sh);
    block_minmax(clo, chi, sh);
    if (tid != 0) return;
    const int k = m.node_ids[j];
    FlatNode& nd = o.nodes[k];
    float mn[3] = {nd.boundsMin.x, nd.boundsMin.y, nd.boundsMin.z};
    float mx[3] = {nd.boundsMax.x, nd.boundsMax.y, nd.boundsMax.z};
    bool grew = false;
    for (int a = 0; a < 3; ++a) {  // glm::min(Min, p) = (p < Min) ? p : Min (BoundingBox.hpp:46)
        grew = grew || lo[a] < mn[a] || mx[a] < hi[a];
        mn[a] = lo[a] < mn[a] ? lo[a] : mn[a];
        mx[a] = mx[a] < hi[a] ? hi[a] : mx[a];
    }
    if (grew) {  // only then: the node-set role may be writing this record in the same launch
        nd.boundsMin = rt_vec3{mn[0], mn[1], mn[2]};
        nd.boundsMax = rt_vec3{mx[0], mx[1], mx[2]};
        const bool leaf = nd.leftChild == -1;
        const int ca = leaf ? -(nd.startShapeIdx + 1) : nd.leftChild, cb = leaf ? nd.numShapes : nd.rightChild;
        o.packed[2 * static_cast<size_t>(k)] = make_float4(mn[0], mn[1], mn[2], __int_as_float(ca));
        o.packed[2 * static_cast<size_t>(k) + 1] = make_float4(mx[0], mx[1], mx[2], __int_as_float(cb));
    }
    if (!o.anodes) return;
    float4* an = o.anodes + 4 * static_cast<size_t>(k);
    if (grew) {
        an[0] = make_float4(mn[0], mn[1], mn[2], an[0].w);
        an[1] = make_float4(mx[0], mx[1], mx[2], an[1].w);
    }
    float4 c0 = an[2], c1 = an[3];  // content box (accel.h)
    c0 = make_float4(fminf(c0.x, clo[0]), fminf(c0.y, clo[1]), fminf(c0.z, clo[2]), c0.w);
    c1 = make_float4(fmaxf(c1.x, chi[0]), fmaxf(c1.y, chi[1]), fmaxf(c1.z, chi[2]), c1.w);
    an[2] = c0;
    an[3] = c1;
    for (int qq = m.wn_off[j]; qq < m.wn_off[j + 1]; ++qq) {
        const int ws = m.wn_list[qq];
        float4* q = o.wnodes + 8 * static_cast<size_t>(ws >> 1) + 4 * (ws & 1);
        if (grew) {
            q[0] = make_float4(mn[0], mn[1], mn[2], q[0].w);
            q[1] = make_float4(mx[0], mx[1], mx[2], q[1].w);
        }
        q[2] = make_float4(c0.x, c0.y, c0.z, q[2].w);
        q[3] = make_float4(c1.x, c1.y, c1.z, q[3].w);
    }
    if (!grew) return;
    for (int q = m.item_off[j]; q < m.item_off[j + 1]; ++q) {
        float4* t = o.titems + 2 * static_cast<size_t>(m.item_list[q]);
        t[0] = make_float4(mn[0], mn[1], mn[2], t[0].w);
        t[1] = make_float4(mx[0], mx[1], mx[2], t[1].w);
    }
}

// Node-set role (rt_update_nodes), one lane per node or scene-tree item: the host's
// node records (same topology) to every copy the kernels read. k < N: node k's
// record, packed copy and accelerator exact box, and for an inner node its
// children's exact boxes in its wnodes record; k >= N: item k - N's gating box (its
// reference leaf's). Content boxes, cones and codes are the shapes' and stay.
__device__ void set_node(const AnimOut& o, const RefitArgs& r, int k) {
    const FlatNode* __restrict__ src = r.nsrc;
    if (k < r.N) {
        const FlatNode n = src[k];
        o.nodes[k] = n;
        const bool leaf = n.leftChild == -1;
        const int ca = leaf ? -(n.startShapeIdx + 1) : n.leftChild, cb = leaf ? n.numShapes : n.rightChild;
        o.packed[2 * static_cast<size_t>(k)] =
            make_float4(n.boundsMin.x, n.boundsMin.y, n.boundsMin.z, __int_as_float(ca));
        o.packed[2 * static_cast<size_t>(k) + 1] =
            make_float4(n.boundsMax.x, n.boundsMax.y, n.boundsMax.z, __int_as_float(cb));
        if (!o.anodes) return;
        float* a = reinterpret_cast<float*>(o.anodes + 4 * static_cast<size_t>(k));
        a[0] = n.boundsMin.x, a[1] = n.boundsMin.y, a[2] = n.boundsMin.z;
        a[4] = n.boundsMax.x, a[5] = n.boundsMax.y, a[6] = n.boundsMax.z;
        if (leaf) return;
        const int ch[2] = {n.leftChild, n.rightChild};
        for (int s = 0; s < 2; ++s) {
            const FlatNode& cn = src[ch[s]];
            float* q = reinterpret_cast<float*>(o.wnodes + 8 * static_cast<size_t>(k) + 4 * s);
            q[0] = cn.boundsMin.x, q[1] = cn.boundsMin.y, q[2] = cn.boundsMin.z;
            q[4] = cn.boundsMax.x, q[5] = cn.boundsMax.y, q[6] = cn.boundsMax.z;
        }
    } else if (k - r.N < r.n_items && o.titems) {
        const int i = k - r.N;
        const FlatNode& ln = src[r.titem_ref[i]];
        float* t = reinterpret_cast<float*>(o.titems + 2 * static_cast<size_t>(i));
        t[0] = ln.boundsMin.x, t[1] = ln.boundsMin.y, t[2] = ln.boundsMin.z;
        t[4] = ln.boundsMax.x, t[5] = ln.boundsMax.y, t[6] = ln.boundsMax.z;
    }
}

// The current record of the shape of accelerator prim p, for the slot role: the
// staging copy (which the record role has brought up to date), or with `direct` a
// moved shape's record itself.
__device__ __forceinline__ const FlatShape& slot_shape(const AnimMaps& m, const AnimOut& o, const RefitArgs& r,
                                                       int p) {
    const int e = r.direct ? m.prim_entry[p] : -1;
    return e >= 0 ? r.fresh[e] : o.shapes[o.prim_shape[p]];
}

// The slot role's back-face cone (barycentric accelerators, accel.cpp build_cones
// and shape_cone): moved walls and triangles turn their stored normals (a wheel's),
// so the child's cone is recomputed from the current records below: axis = the unit
// normals' sum, half angle = the largest angle to the stored (float) axis, plus
// kConeMargin; any other shape or a normal sum near 0 makes it full. A child whose
// cone is full already (kConeNever: the build found it so, or culling is off) keeps
// it -- a word that never culls always holds -- which spares the large subtrees
// near the roots a pass over their prims.
__device__ void refit_slot_cone(const AnimMaps& m, const AnimOut& o, const RefitArgs& r, int4 d, int w, int sl,
                                int lane) {
    int* cw = reinterpret_cast<int*>(o.lnodes + kWideRec * static_cast<size_t>(w) + 6) + sl;
    if (*cw == rta::kConeNever) return;  // the same word for the whole wave
    auto load = [&](int p) {  // the stored normal (w: 0 for a shape without a cone)
        const FlatShape& s = slot_shape(m, o, r, p);
        const bool cone = s.type == RT_WALL || s.type == RT_TRIANGLE;
        return make_float4(s.planeNormal.x, s.planeNormal.y, s.planeNormal.z, cone ? 1.f : 0.f);
    };
    auto unit_normal = [](const float4& v, double n[3]) {  // accel.cpp shape_cone
        n[0] = v.x, n[1] = v.y, n[2] = v.z;
        const double l = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
        if (v.w == 0.f || !(l > 1e-20) || !isfinite(l)) return false;
        for (int a = 0; a < 3; ++a) n[a] /= l;
        return true;
    };
    double sn[3] = {0, 0, 0};
    int full = 0;
    range4(d.y, d.z, lane, load, [&](const float4& v) {
        double n[3];
        if (!unit_normal(v, n)) {
            full = 1;
            return;
        }
        for (int a = 0; a < 3; ++a) sn[a] += n[a];
    });
    for (int off = 32; off > 0; off >>= 1) {
        for (int a = 0; a < 3; ++a) sn[a] += __shfl_xor(sn[a], off);
        full |= __shfl_xor(full, off);
    }
    const double l = sqrt(sn[0] * sn[0] + sn[1] * sn[1] + sn[2] * sn[2]);
    if (full || !(l > 1e-6) || d.y >= d.z) {
        if (lane == 0) *cw = rta::kConeNever;
        return;
    }
    float af[3];  // the axis as lane 0 rounds it (the butterfly's sums may differ in the last bits)
    for (int a = 0; a < 3; ++a) af[a] = __shfl(static_cast<float>(sn[a] / l), 0);
    const double al = sqrt(static_cast<double>(af[0]) * af[0] + static_cast<double>(af[1]) * af[1] +
                           static_cast<double>(af[2]) * af[2]);
    double cmin = 1.0;  // the smallest cosine to the axis
    range4(d.y, d.z, lane, load, [&](const float4& v) {
        double n[3];
        unit_normal(v, n);
        cmin = fmin(cmin, (n[0] * af[0] + n[1] * af[1] + n[2] * af[2]) / al);
    });
    for (int off = 32; off > 0; off >>= 1) cmin = fmin(cmin, __shfl_xor(cmin, off));
    if (lane != 0) return;
    const double t = acos(fmax(-1.0, fmin(1.0, cmin))) + rta::kConeMargin;
    *cw = t >= 1.5707 ? rta::kConeNever : rta::cone_word(af[0], af[1], af[2], static_cast<float>(-sin(t)));
}

// The slot role's Moller-Trumbore part (MT accelerators have local trees only):
// the child's grazing cone, per-ray padding constants and slab (accel.cpp
// build_cones_mt), recomputed from the current records of every triangle below,
// since a refit moves and turns them (a wheel's). Two passes over the slot's prims:
// the normals' sum (each flipped towards the old axis) gives the new axis, stored as
// float; then s = the largest min(|n - a|, |n + a|) against that stored axis (for
// any a, |d.n| >= |d.a| - |n -+ a|: what mt_pad's cone term needs) and the slab of
// a . vertex. The constants take the worst triangle as the build's do, without its
// grow-only margin. A shape other than a bounded triangle below: no slab, as built.
__device__ void refit_slot_mt(const AnimMaps& m, const AnimOut& o, const RefitArgs& r, int4 d, int w, int sl,
                              int lane) {
    float* k = wide_box_f(o.lnodes, kWideRecMt, w, sl, 0) + 6;  // axis xyz, s, {cr, u X, M, 18 M + 10.5 Esum, w, h0}
    const double a0[3] = {k[0], k[1], k[2]};                      // every lane reads before lane 0 writes
    struct Tri {
        int type;
        rt_vec3 p1, p2, p3;
    };
    auto load = [&](int p) {
        const FlatShape& s = slot_shape(m, o, r, p);
        return Tri{s.type, s.triP1, s.triP2, s.triP3};
    };
    auto as_shape = [](const Tri& v) {  // what classify_mt_tight reads
        FlatShape s{};
        s.type = v.type, s.triP1 = v.p1, s.triP2 = v.p2, s.triP3 = v.p3;
        return s;
    };
    auto tri_normal = [](const FlatShape& s, double n[3]) {  // accel.cpp mt_normal, with |e1 x e2|
        const float e1[3] = {s.triP2.x - s.triP1.x, s.triP2.y - s.triP1.y, s.triP2.z - s.triP1.z};
        const float e2[3] = {s.triP3.x - s.triP1.x, s.triP3.y - s.triP1.y, s.triP3.z - s.triP1.z};
        n[0] = static_cast<double>(e1[1]) * e2[2] - static_cast<double>(e1[2]) * e2[1];
        n[1] = static_cast<double>(e1[2]) * e2[0] - static_cast<double>(e1[0]) * e2[2];
        n[2] = static_cast<double>(e1[0]) * e2[1] - static_cast<double>(e1[1]) * e2[0];
        const double l = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
        for (int a = 0; a < 3; ++a) n[a] /= l;
    };
    double sn[3] = {0, 0, 0}, cr = INFINITY, X = 0, es = 0, mm = 0;
    int other = 0;
    range4(d.y, d.z, lane, load, [&](const Tri& v) {
        const FlatShape s = as_shape(v);
        rta::MtTri t;
        rta::Box3 tb;
        if (s.type != RT_TRIANGLE || rta::classify_mt_tight(s, tb, 0.0, t) != rta::BOUNDED) {
            other = 1;
            return;
        }
        double n[3];
        tri_normal(s, n);
        const double sg = n[0] * a0[0] + n[1] * a0[1] + n[2] * a0[2] < 0 ? -1.0 : 1.0;
        for (int a = 0; a < 3; ++a) sn[a] += sg * n[a];
        const double dz[3] = {t.p1[0] - o.mt_z[0], t.p1[1] - o.mt_z[1], t.p1[2] - o.mt_z[2]};
        cr = fmin(cr, t.cr);
        X = fmax(X, t.X);
        es = fmax(es, t.esum);
        mm = fmax(mm, sqrt(dz[0] * dz[0] + dz[1] * dz[1] + dz[2] * dz[2]));
    });
    for (int off = 32; off > 0; off >>= 1) {
        for (int a = 0; a < 3; ++a) sn[a] += __shfl_xor(sn[a], off);
        cr = fmin(cr, __shfl_xor(cr, off));
        X = fmax(X, __shfl_xor(X, off));
        es = fmax(es, __shfl_xor(es, off));
        mm = fmax(mm, __shfl_xor(mm, off));
        other |= __shfl_xor(other, off);
    }
    // the axis as lane 0 rounds it (the butterfly's sums may differ in the last bits)
    const double l = sqrt(sn[0] * sn[0] + sn[1] * sn[1] + sn[2] * sn[2]);
    const bool full = !(l > 1e-6) || !(X > 0);  // no triangle, or normals cancelling: a full cone
    float af[3];
    for (int a = 0; a < 3; ++a) af[a] = __shfl(full ? static_cast<float>(a0[a]) : static_cast<float>(sn[a] / l), 0);
    double sm = 0, lo = INFINITY, hi = -INFINITY;
    range4(d.y, full ? d.y : d.z, lane, load, [&](const Tri& v) {
        const FlatShape s = as_shape(v);
        rta::MtTri t;
        rta::Box3 tb;
        if (s.type != RT_TRIANGLE || rta::classify_mt_tight(s, tb, 0.0, t) != rta::BOUNDED) return;
        double n[3], dm = 0, dp = 0;
        tri_normal(s, n);
        for (int a = 0; a < 3; ++a) {
            dm += (n[a] - af[a]) * (n[a] - af[a]);
            dp += (n[a] + af[a]) * (n[a] + af[a]);
        }
        sm = fmax(sm, sqrt(fmin(dm, dp)));
        for (const rt_vec3& v : {s.triP1, s.triP2, s.triP3}) {
            const double x = static_cast<double>(af[0]) * v.x + static_cast<double>(af[1]) * v.y +
                             static_cast<double>(af[2]) * v.z;
            lo = fmin(lo, x);
            hi = fmax(hi, x);
        }
    });
    for (int off = 32; off > 0; off >>= 1) {
        sm = fmax(sm, __shfl_xor(sm, off));
        lo = fmin(lo, __shfl_xor(lo, off));
        hi = fmax(hi, __shfl_xor(hi, off));
    }
    if (lane != 0) return;
    const double up = 1.0 + 1e-5, sv = sm * (1.0 + 1e-6) + 2e-5;
    k[0] = af[0], k[1] = af[1], k[2] = af[2];
    // build_cones_mt: theta >= 1.5 is a full cone; so is every cone with culling off (the build's)
    k[3] = full || sv >= 1.3633 || !o.cone_cull ? 2.f : static_cast<float>(sv);
    if (!(X > 0)) {  // no triangle below: pad 0, no slab
        for (int a = 4; a < 9; ++a) k[a] = 0.f;
        k[9] = INFINITY;
        return;
    }
    k[4] = static_cast<float>(cr * (1.0 - 1e-5));
    k[5] = static_cast<float>(rta::kU * X * up);
    k[6] = static_cast<float>(mm * up + 1e-5);
    k[7] = static_cast<float>((18.0 * mm + 10.5 * es) * up + 1e-5);
    const bool slab = !full && !other && lo <= hi;
    const double wc = slab ? 0.5 * (lo + hi) : 0.0;
    k[8] = static_cast<float>(wc);
    k[9] = slab ? static_cast<float>(0.5 * (hi - lo) * up + 1e-5 * (fabs(wc) + 1.0)) : INFINITY;
}

// Slot role: exact refit of the local / scene-tree boxes above moved prims (they
// are the accelerator's own, so unlike the reference nodes they may shrink): one
// workgroup per dirty wide-record slot, the union of the box of the slot's prims
// that are not in the refit set (fixed: prepare_animation, dstatic) and of pbox over
// those that are (dlist) -- a subtree's prims are contiguous (accel.cpp
// LocalBuilder), the scene tree's top slots span every prim (the car: 4,020, against
// 640 refit prims). dirty[j] = (4*w + s, first prim, end prim, first of its dlist
// entries); dirty[j + 1].w ends them.
__device__ void refit_slot(const AnimMaps& m, const AnimOut& o, const RefitArgs& r, int j, float (*sh)[6],
                           bool block) {
    const int tid = block ? threadIdx.x : threadIdx.x & 63, lane = tid & 63;
    const int4 d = r.dirty[j];
    const float4* __restrict__ pbox = o.pbox;
    const float4 s0 = r.dstatic[2 * j], s1 = r.dstatic[2 * j + 1];
    float lo[3] = {s0.x, s0.y, s0.z}, hi[3] = {s1.x, s1.y, s1.z};
    range4(d.w, r.dirty[j + 1].w, tid, block ? static_cast<int>(blockDim.x) : 64,
        [&](int q) {
            const int p = r.dlist[q];
            const int e = r.direct ? m.prim_entry[p] : -1;
            if (e >= 0 && m.ecls[e] == rta::BOUNDED) {  // a moved prim, from its record itself
                rta::Box3 cb;
                entry_cbox(o, r.fresh[e], rta::BOUNDED, cb);
                return Box4{make_float4(cb.lo[0], cb.lo[1], cb.lo[2], 0.f), make_float4(cb.hi[0], cb.hi[1], cb.hi[2], 0.f)};
            }
            return Box4{pbox[2 * static_cast<size_t>(p)], pbox[2 * static_cast<size_t>(p) + 1]};
        },
        [&](const Box4& v) {
            const float4 a = v.a, b = v.b;
            lo[0] = fminf(lo[0], a.x), lo[1] = fminf(lo[1], a.y), lo[2] = fminf(lo[2], a.z);
            hi[0] = fmaxf(hi[0], b.x), hi[1] = fmaxf(hi[1], b.y), hi[2] = fmaxf(hi[2], b.z);
        });
    if (block)
        block_minmax(lo, hi, sh);
    else
        wave_minmax(lo, hi);
    if (tid >= 64) return;  // the cones: one wave
    const int w = d.x >> 2, sl = d.x & 3;
    if (lane < 6) {  // rows 0-5 of the wide record: lo.xyz, hi.xyz
        const float v = lane == 0 ? lo[0] : lane == 1 ? lo[1] : lane == 2 ? lo[2] : lane == 3 ? hi[0] : lane == 4 ? hi[1] : hi[2];
        *wide_box_f(o.lnodes, r.rec, w, sl, lane) = v;
    }
    if (o.mt)
        refit_slot_mt(m, o, r, d, w, sl, lane);
    else
        refit_slot_cone(m, o, r, d, w, sl, lane);
}

// The per-frame refit of flush_updates, in workgroups of four roles:
//   [0, na)             record role (refit_record), a lane per entry;
//   [na, na + nd)       node-set role (set_node), a lane per node or item;
//   [na + nd, ...)      a workgroup each: node role (grow_node) for the first nb, then
//                       slot role (refit_slot); both read what the record role wrote.
// Modes (rt_debug_refit), on the car's wheels (640 entries, 650 dirty slots):
//   1 default: two launches, records and node sets in one-wave workgroups, then nodes
//     and slots in kRefitWaves-wave ones: the kernel boundary orders them (11.4 + 8.4
//     us, no gap between them; r05n);
//   3 ONE launch of kRefitWaves-wave workgroups whose node / slot workgroups wait (wait
//     2) until every record workgroup has released its writes. Workgroups start in
//     index order, record workgroups first, and every one of them runs to its end
//     without waiting, so the waits end. Measured 42 us polling the done counter, 52
//     us polling kRefitFlags copies of a flag (r05o, r05p), 29 us with one agent-scope
//     fence per workgroup instead of one per thread (each writes back or invalidates the
//     XCD's L2; r05zv): slower than two launches;
//   0 as 3 with the start order made explicit by a ticket per workgroup (wait 1): the
//     ticket counter serialises the launch (35 us when measured with one-wave slots);
//   2 one launch whose node / slot roles derive each entry's boxes from its record over
//     the host link themselves (direct; 72 us).
// Copying the records to the device before the launches instead of reading them over
// the host link measured no faster (r05k: waited car frame 0.259 against 0.252 ms). The
// record role's 11 us are not its stores: with every store skipped in turn (timing builds,
// r05x) it took 10.0-12.2 us, and moved beside the slot roles (its boxes alone in the first
// launch, r05y) the first launch still took 10.3 us while the second grew to 23.
// The node-set role never runs with AF_GROW entries in the same flush (flush_updates
// applies host node records first), so no two roles write the same box.
__global__ __launch_bounds__(64 * kRefitWaves) void k_refit(AnimMaps m, AnimOut o, RefitArgs r) {
    __shared__ float sh[kRefitWaves][6];
    const int tid = threadIdx.x, nt = blockDim.x;
    unsigned t = blockIdx.x;  // without waits the start order does not matter
    if (r.wait == 1) {
        __shared__ unsigned ticket;
        if (tid == 0) ticket = __hip_atomic_fetch_add(r.ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - r.tbase;
        __syncthreads();
        t = ticket;
    }
    if (t < static_cast<unsigned>(r.na)) {
        refit_record(m, o, r, static_cast<int>(t) * nt + tid);
        if (r.wait) {
            // the workgroup's writes complete (barrier), then ONE agent-scope release: each
            // fence writes the XCD's L2 back, and one per thread cost the launch ~30 us
            __syncthreads();
            if (tid == 0) {
                __threadfence();
                const unsigned done = __hip_atomic_fetch_add(r.ctr + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
                if (done - r.abase == static_cast<unsigned>(r.na) - 1u)  // the last one: raise the flags
                    for (int k = 0; k < kRefitFlags; ++k)
                        __hip_atomic_store(r.ctr + kRefitFlag0 + 16 * k, r.abase + r.na, __ATOMIC_RELEASE,
                                           __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        return;
    }
    t -= r.na;
    if (t < static_cast<unsigned>(r.nd)) {
        set_node(o, r, static_cast<int>(t) * nt + tid);
        return;
    }
    t -= r.nd;
    if (r.wait) {
        // one of kRefitFlags copies of the all-done flag, a cache line each: ~650 waiting
        // workgroups polling the counter itself held its increments back (car: 42 us)
        const unsigned* flag = r.ctr + kRefitFlag0 + 16 * (blockIdx.x % kRefitFlags);
        if (tid == 0) {
            // Bounded (diagnostic modes only): these waits rely on the record
            // workgroups having started, which HIP does not promise. Past ~1 s of the
            // constant-rate clock (100 MHz) the wait gives up and reports, so a scheduling
            // change shows up as a rebuild (check_reports), not as a GPU hang.
            const unsigned long long t0 = wall_clock64();
            while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - r.abase <
                   static_cast<unsigned>(r.na)) {
                __builtin_amdgcn_s_sleep(2);
                if (wall_clock64() - t0 > 100000000ull) {
                    __hip_atomic_store(r.report, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // one invalidation per workgroup
        }
        __syncthreads();
    }
    const int w = static_cast<int>(t) - r.nb;
    if (w < 0) {
        grow_node(m, o, r, w + r.nb, sh);
        return;
    }
    const int nbig = min(r.n_big, r.n_dirty);
    if (w < nbig) {
        refit_slot(m, o, r, w, sh, true);  // a long list: the whole workgroup
        return;
    }
    const int j = nbig + (w - nbig) * (nt >> 6) + (tid >> 6);  // a wave per slot
    if (j < r.n_dirty) refit_slot(m, o, r, j, sh, false);
}

// Scene-tree wide slots of the unbounded subtree (kNoPrune): their boxes are the
// reference leaves' padded boxes, which animation grows; while a set is animated
// they are infinite (entered by every ray; the items' exact boxes still gate).
__global__ void k_inf_slots(const int* __restrict__ slots, int n, float4* __restrict__ lnodes, int rec) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int w = slots[i] >> 2, sl = slots[i] & 3;
    for (int r = 0; r < 6; ++r) *wide_box_f(lnodes, rec, w, sl, r) = r < 3 ? -INFINITY : INFINITY;
}

}  // namespace

// ===========================================================================
// C ABI

struct rt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;      // used once the ring is full
    hipEvent_t sync_ev = nullptr;                  // rt_sync's poll target
    // The cost order's kernels (k_cost_dilate, k_tile_order) on a second stream behind the
    // render's end event (rt_debug_order_stream; 0: on this stream, 1: latency-mode
    // dispatches, 2: all), so that a waited frame ends with its render; the next accelerated
    // dispatch waits for order_done (join_order), anything that frees or reads the order's
    // buffers on the host synchronizes order_stream first (sync_order).
    hipStream_t order_stream = nullptr;
    hipEvent_t order_ready = nullptr, order_done = nullptr;
    bool order_pending = false;  // order_done not yet waited for on `stream`
    int order_mode = 0;
    // rt_sync_frame: a latency-mode cost frame records frame_ev between its render and the
    // order's kernels (same stream), and the waited frame ends there (rt_debug_frame_event)
    int frame_event = 1;
    hipEvent_t frame_ev = nullptr;
    bool frame_ev_set = false;         // this context's last launch recorded frame_ev
    rt_ctx* frame_from = nullptr;      // the context whose launch rendered the last dispatch
    unsigned long long refit_launches = 0;  // k_refit launches so far
    unsigned long long frame_refits = 0;    // those of this context + sub-contexts at that dispatch
    hipEvent_t last0 = nullptr, last1 = nullptr;  // events of the latest dispatch
    bool timed = false;
    // per-dispatch event pairs since the last rt_kernel_times call
    std::vector<hipEvent_t> ring0, ring1;
    int ring_used = 0;
    bool timing = true;  // rt_set_kernel_timing: record the ring's events around each render
    // scene
    float4 *geo_lin = nullptr, *geo_leaf = nullptr, *mat = nullptr, *nodes = nullptr;
    int S = 0, N = 0, I = 0, max_stack = 1;
    bool have_scene = false, have_cam = false, have_light = false;
    std::vector<FlatNode> host_nodes;  // topology check for rt_update_nodes
    FlatShape* staging_shapes = nullptr;
    size_t staging_shapes_cap = 0;
    FlatNode* staging_nodes = nullptr;
    size_t staging_nodes_cap = 0;
    int* staging_idx = nullptr;
    size_t staging_idx_cap = 0;
    std::vector<int> host_idx;
    std::vector<FlatShape> host_shapes;
    // exact-result accelerator (accel.h); device copies in the layouts of AccelPtrs
    float4 *anodes = nullptr, *lnodes = nullptr, *wnodes = nullptr, *prims = nullptr;
    int4* tleaf = nullptr;
    float4* titems = nullptr;  // scene-tree items (AccelPtrs::titems)
    int* titem_ref = nullptr;  // per titems record: its reference leaf (device copy)
    std::vector<int> host_titem_ref;  // the same on the host (prepare_animation: items of a grown leaf)
    int n_titems = 0;
    int* anim_inf_slots = nullptr;  // wide slots whose boxes go infinite while animating (kNoPrune)
    int n_inf_slots = 0;
    bool inf_open = false;          // open_inf_slots ran since the accelerator was built
    int st_root = 0x7fffffff;  // scene-tree root code, kNoChild if none
    int tree_mode = 1;         // rt_set_tree
    int scene_stack = 0;       // rt_debug_scene_stack (0: the walk's own cap)
    int nfew = 0;              // few-leaf mode (AccelPtrs::nfew)
    int* prim_idx_dev = nullptr;
    bool accel_ok = false;
    size_t record_bytes = 0;   // device records k_accel reads (rt_accel_info::record_bytes)
    int boxes_finite = 0;
    rta::AccelHost accel;
    // frame constants
    FlatCamera cam{};
    FlatLight light{};
    rt_params params{0.f, 0.f, 0, 0, 0, 0};  // the reference's first frame sees zeros
    int kernel = RT_KERNEL_AUTO;
    int last_kind = 0;
    // own surface
    float* img = nullptr;
    size_t img_pitch = 0;
    int img_w = 0, img_h = 0;
    unsigned long long* stats_dev = nullptr;
    // launch shape of k_accel (rt_set_launch)
    int waves_per_block = 1, persistent = 0, cu_count = 256;
    int lane_from_depth = -1;  // bounces >= this use the per-lane walk (0: all, large: none;
                               // -1: auto, see walk_from)
    int cone_cull = 1;
    int spec_mode = 1;  // speculative while-while in lane_walk (rt_debug_spec): 1 on, 0 off
    int split_max = kSplitMax, split_g = kSplitGroup;  // split per-lane walks (rt_debug_split)
    int heavy_k = kHeavyTiles, heavy_parts = kHeavyParts;  // heaviest tiles as several waves (rt_debug_heavy)
    int lane_k = -1, lane_k_mode = 2;  // heaviest slots' walk modes (rt_debug_lane_k; -1: auto)
    int cost_time = -1;                // tile cost: 0 lane work, else wave wall time (rt_debug_cost_time)
    int latency_mode = 0;              // rt_set_latency_mode
    int* tile_order = nullptr;  // diagnostics (rt_debug_tile_order): fixed dispatch order of the 8x8 tiles
    int tile_order_n = 0;
    // rt_set_schedule: per-tile durations of the last dispatch and the order derived from them
    int schedule = RT_SCHED_COST;
    unsigned* sched_cost = nullptr;
    unsigned long long* heavy_acc = nullptr;  // split heavy tiles' part counts + sums (cost-recording dispatches)
    size_t heavy_acc_cap = 0;
    int* sched_order = nullptr;
    unsigned* sched_sets = nullptr;      // 2 sets of per-group bucket histograms, alternating by frame
    int sched_parity = 0;
    int sched_cap = 0, sched_valid = 0;  // buffer capacity; tile count the order is for (0: none)
    // The order is re-derived on every sched_period-th dispatch (and whenever the tile
    // count changes); the dispatches between reuse it and record no work counts. 16:
    // car in flight -1.0 % against 8 (32: -0.9 %, 4: +1.5 %; profiles/r04z2_*)
    int sched_period = 16, sched_frame = 0;
    int cost_dilate = 0;                 // rt_debug_cost_dilate: radius in tiles (0: off)
    // The cost order of a dispatch whose camera differs from the last accelerated
    // dispatch's (rt_debug_moving; period 0: as any other): re-derived after every such
    // dispatch from whole-tile wall times dilated by one tile. The car's waited frame
    // along the orbit / dolly paths of bench.py --camera-path, against the same cameras
    // held still (median ratio over 8 cameras, tools/camera_probe.py, r05h / r05i):
    // the still policy (every 16th frame, undilated) 1.53 / 1.46; every frame undilated
    // 1.26; every 4th dilated by 2 1.16; every frame dilated by 1 1.09 / 1.06, with split
    // tiles on those frames 1.15 / 1.14 (a split tile ranked by its parts' sum), 1.15-1.19 by
    // half or a quarter of it, 1.18 / 1.13 by its longest part (r05z, r05z2).
    int moving_period = 1, moving_dilate = 1, moving_split = 0;
    FlatCamera sched_cam{};
    bool have_sched_cam = false;
    bool moving = false;  // this dispatch's camera moved
    unsigned* dil_cost = nullptr;        // its dilated costs (sched_cap) + bucket rows
    size_t dil_cap = 0;
    // compaction (rt_set_tail): bounces >= tail_from run in k_accel_tail (0: off)
    int tail_from = RT_TAIL_AUTO;
    float4* tail_queue = nullptr;
    size_t tail_cap = 0;     // queue entries
    int* tail_counts = nullptr;  // two sets of per-region counters, alternating by dispatch
    int tail_regions_cap = 0;
    int tail_max_lanes = 64;  // rt_debug_tail_lanes
    int shadow_walk_override = -1;  // rt_debug_shadow_walk (-1: policy)
    int tail_parity = 0;
    int lane_stack_override = 0;  // diagnostics only (rt_debug_lane_stack): breaks exactness if too small
    int* tile_counter = nullptr;
    unsigned long long* tile_times = nullptr;  // diagnostics (rt_debug_tile_times)
    size_t tile_times_cap = 0;
    // animation (rt_set_animated / rt_animate) and the reference's own uploads
    // (rt_update_shapes / rt_update_nodes), both applied by the device refit
    std::vector<int> anim_ids;          // rt_set_animated's set, in rt_animate's record order
    // The refit set: every shape moved since the accelerator was built (the animated
    // set plus the shapes rt_update_shapes rewrote). One entry each; AnimMaps lists them.
    std::vector<int> refit_ids;
    std::vector<int> refit_of;          // per shape: its refit entry, -1 if none
    std::vector<int> anim_cls;          // per refit entry: accelerator class at the last build (accel_bound.h)
    std::vector<FlatShape> anim_base;   // per refit entry: the record the accelerator's cones were built from
    // rt_update_shapes / rt_update_nodes only write the host copies; the next device
    // operation (flush_updates) applies them in one refit, like glBufferSubData
    // calls that take effect at the next dispatch.
    std::vector<int> upd_ids;           // shapes written since the last flush
    std::vector<char> upd_mark;         // per shape: listed in upd_ids
    std::vector<std::pair<int, FlatShape>> upd_base;  // their build-time records (shapes new to the refit set)
    bool nodes_dirty = false;           // host_nodes newer than every device copy
    bool nodes_rebuild = false;         // host_nodes break a condition the accelerator was built on
    bool bounds_rebuild = false;        // a refit reported a shape whose bound changed kind
    int updates_flushed = 0;            // flushes that refit instead of rebuilding (diagnostics)
    // rt_debug_refit: 0 one launch (box roles wait on tickets), 1 two launches (default:
    // the car's waited animated frame 0.262 ms against 0.268 and 0.299, r05d), 2 one
    // launch (box roles read the records over the host link themselves)
    // rt_debug_refit; -1 auto: one direct launch (mode 2) while the records its readers
    // fetch over the host link are few (direct_reads <= kDirectReads), else two launches
    // (mode 1). Waited animated frames, mode 1 against 2: config 2's three spheres (~50
    // reads) 0.1062 against 0.1024 ms; the car's wheels (~7,500 reads) 0.2449 against
    // 0.2777 (r05q)
    int refit_mode = -1;
    long long direct_reads = 0, n_direct_slot_reads = 0;
    char* refit_dev = nullptr;  // refit mode 4: the pinned slot's records copied to the device
    size_t refit_dev_cap = 0;
    long long dirty_sum = 0;  // rt_debug_refit_stats: the slot refit's prim ranges (largest, total)
    long long last_flush_bytes = 0;  // rt_debug_refit_stats: the pinned records of the last flush
    int refit_compactions = 0;       // rt_debug_refit_stats: stale entries dropped (compact_refit_set)
    int dirty_max = 0;
    int* anim_maps = nullptr;           // AnimMaps lists, one allocation
    size_t anim_maps_cap = 0;
    AnimMaps anim{};
    // Per-frame records, FlatShape[count] then int flags[count]: a ring of pinned, mapped
    // host buffers that k_refit reads directly, so a flush waits only for the
    // k_refit kAnimRing flushes back (not for the previous frame's render). Each slot
    // ends in a report word k_refit sets when a shape's bound changed kind.
    static constexpr int kAnimRing = 3;
    void* anim_pinned[kAnimRing] = {nullptr, nullptr, nullptr};
    void* anim_pinned_dev[kAnimRing] = {nullptr, nullptr, nullptr};  // the same buffers as the device sees them
    size_t anim_pinned_cap[kAnimRing] = {0, 0, 0};
    hipEvent_t anim_copied[kAnimRing] = {nullptr, nullptr, nullptr};  // that slot's k_refit has run
    size_t report_at[kAnimRing] = {0, 0, 0};       // offset of the slot's report word
    bool report_pending[kAnimRing] = {false, false, false};  // its k_refit not yet checked
    bool slot_busy[kAnimRing] = {false, false, false};       // a k_refit reads it (anim_copied ends that)
    // The slot of the last k_refit whose anim_copied is not recorded yet. An event
    // costs the stream ~6 us wherever it sits (the car's animated frame: between k_refit
    // and the render kernel it held the render kernel back, behind the render kernel
    // it delayed rt_sync's own event; rocprofv3 --hip-trace, r05h / r05i), so it is
    // recorded only when needed: before the next k_refit (frames in flight), or when
    // the slot is wanted back. A wait that drains the stream (rt_sync) retires it
    // unrecorded (stream_drained).
    int mark_slot = -1;
    unsigned* refit_ctr = nullptr;      // k_refit's ticket and done counters (never reset)
    unsigned ctr_tickets = 0, ctr_done = 0;  // their values after the last launch
    int anim_slot = 0;
    float4* anim_sbox = nullptr;        // per animated shape boxes (AnimOut::sbox)
    size_t anim_sbox_cap = 0;
    float4* pbox = nullptr;             // per prim conservative box (AnimOut::pbox)
    int4* refit_dirty = nullptr;        // k_refit's slot work list (RefitArgs::dirty)
    int n_big = 0;                      // its first n_big slots have long refit lists (RefitArgs::n_big)
    float4* refit_static = nullptr;     // RefitArgs::dstatic
    int* refit_list = nullptr;          // RefitArgs::dlist
    int n_dirty = 0;
    int anim_rebuilds = 0;              // host rebuilds rt_animate fell back to (diagnostics)
    // A refit that asks for a rebuild (a bound changed kind, or the node boxes stopped
    // nesting) starts it on a host thread over a snapshot of the records (AsyncBuild) and
    // the frames go on meanwhile, exact: a changed-kind shape is entered through every box
    // above it (k_refit), and while the boxes do not nest the rays walk the reference tree
    // (st_suspended). The first device operation after the build finishes swaps the new
    // accelerator in and refits it to the records written since the snapshot. rt_debug_
    // async_rebuild(0): the rebuild runs in the flush that asked for it, as before round 6.
    struct AsyncBuild {
        std::thread th;
        std::atomic<bool> done{false};
        bool ok = false;
        rta::AccelHost A;
        std::vector<FlatShape> shapes;  // the snapshot the accelerator is built from
        std::vector<FlatNode> nodes;
    };
    std::unique_ptr<AsyncBuild> rebuild;
    // The last swapped-in build's object, kept for the next rebuild: its snapshot buffers
    // are refilled in place, and its A (the replaced accelerator's host arrays) is
    // released by the next build on its thread -- freeing ~30-100 MB at the swap took
    // 5-11 ms of the frame on config 5 (munmap).
    std::unique_ptr<AsyncBuild> spare;
    int async_rebuild = 1;
    bool st_suspended = false;          // the scene tree is off until the rebuild lands
    int async_swaps = 0;                // rebuilt accelerators swapped in (diagnostics)
    bool nodes_on_device_newer = false; // staging_nodes grew past host_nodes
    // The root node's box as the next render sees it, kept on the host without a
    // readback: set from the records by rt_upload_scene / rt_update_nodes, grown by
    // rt_animate as k_refit grows it (reference_box of every animated shape the root
    // lists). rt_group computes its sky-row band from it (rtx::view_root).
    float root_lo[3] = {0.f, 0.f, 0.f}, root_hi[3] = {0.f, 0.f, 0.f};
    std::vector<char> entry_root;       // per refit entry: node N-1 lists it (k_refit grows the root by it)
    // rtx::animate_deferred (rt_group's frame slots): per animated shape (anim_ids order)
    // the union of the growToInclude boxes of every frame given since the last flush
    // (lo xyz, hi xyz), applied by the next flush as that shape's growth (AF_BOX)
    std::vector<float> grow_box;
    bool grow_pending = false;
    // per shape: its host record may differ from the one AccelHost::shape_cls / shape_box
    // were classified from (the build's, or prepare_animation's since): prepare_animation
    // then classifies it again and caches the result there
    std::vector<char> shape_moved;
    // The brute-force branch (useBVH = 0, gpu_shader.comp:523-620) tests every shape in
    // index order, keeps the strict-< first minimum and stops shadows at the first
    // occluder: exactly the BVH branch walking a tree of ONE leaf that lists shapes
    // 0..S-1 in order under an infinite box (which every ray with a non-NaN slab passes,
    // and for which a NaN ray gets no hit in either branch), except for the shadow
    // offset, 1e-5 instead of 1e-3 (:565 vs :469). `brute` is that second context: the
    // same shapes over the one-leaf tree, with its own accelerator, on this stream.
    rt_ctx* brute = nullptr;
    bool brute_stale = true;            // shapes changed since brute's upload
    int brute_accel = 1;                // rt_set_brute_accel
    // Moller-Trumbore frames (useMollerTrumbore = 1) render through `mtc`: the same
    // scene with its accelerator built for the MT test (accel.h AccelHost::mt).
    rt_ctx* mtc = nullptr;
    bool mtc_stale = true;              // shapes or nodes changed since mtc's upload
    bool build_mt = false;              // this context's accelerator is built for MT
};

namespace {

hipError_t sync_stream(rt_ctx* c);  // hipStreamSynchronize + the refit slots retired (below)

#pragma clang diagnostic ignored "-Wunused-result"
#define HIP_TRY(x)                                  \
    do {                                            \
        hipError_t e__ = (x);                       \
        if (e__ != hipSuccess) return RT_ERR_DEVICE; \
    } while (0)

int set_dev(rt_ctx* c) {
    HIP_TRY(hipSetDevice(c->device));
    return RT_OK;
}

template <class T>
int ensure_staging(T*& p, size_t& cap, size_t n) {
    if (n <= cap && p) return RT_OK;
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(&p, n * sizeof(T) > 0 ? n * sizeof(T) : sizeof(T)) != hipSuccess) return RT_ERR_NO_MEMORY;
    cap = n;
    return RT_OK;
}

void free_accel(rt_ctx* c) {
    hipFree(c->anodes);
    hipFree(c->lnodes);
    hipFree(c->wnodes);
    hipFree(c->tleaf);
    hipFree(c->titems);
    c->titems = nullptr;
    hipFree(c->titem_ref);
    c->titem_ref = nullptr;
    c->n_titems = 0;
    c->host_titem_ref.clear();
    hipFree(c->anim_inf_slots);
    c->anim_inf_slots = nullptr;
    c->n_inf_slots = 0;
    c->inf_open = false;
    c->st_root = kNoChild;
    hipFree(c->prims);
    hipFree(c->prim_idx_dev);
    hipFree(c->pbox);
    hipFree(c->refit_dirty);
    hipFree(c->refit_static);
    hipFree(c->refit_list);
    c->pbox = nullptr;
    c->refit_dirty = nullptr;
    c->refit_static = nullptr;
    c->refit_list = nullptr;
    c->n_dirty = 0;
    c->anodes = c->lnodes = c->wnodes = c->prims = nullptr;
    c->tleaf = nullptr;
    c->prim_idx_dev = nullptr;
    c->accel_ok = false;
}

void discard_rebuild(rt_ctx* c);
void free_scene(rt_ctx* c) {
    discard_rebuild(c);
    hipFree(c->geo_lin);
    hipFree(c->geo_leaf);
    hipFree(c->mat);
    hipFree(c->nodes);
    c->geo_lin = c->geo_leaf = c->mat = c->nodes = nullptr;
    free_accel(c);
    c->have_scene = false;
}

// Checks the arrays the way the reference shader would dereference them and
// measures the reference walk's worst-case stack need (every box hit).
int check_tree(const FlatNode* nodes, int N, const int* idx, int I, int S, int* max_stack) {
    for (int i = 0; i < I; ++i)
        if (idx[i] < 0 || idx[i] >= S) return RT_ERR_BVH;
    for (int k = 0; k < N; ++k) {
        const FlatNode& n = nodes[k];
        if (n.leftChild == -1) {
            if (n.numShapes > 0 && (n.startShapeIdx < 0 || n.startShapeIdx > I - n.numShapes)) return RT_ERR_BVH;
        } else if (n.leftChild < 0 || n.leftChild >= N || n.rightChild < 0 || n.rightChild >= N) {
            return RT_ERR_BVH;
        }
    }
    int ms = N > 0 ? 1 : 0;
    if (N > 0) {
        std::vector<int> st;
        st.push_back(N - 1);
        long long visits = 0;
        while (!st.empty()) {
            int k = st.back();
            st.pop_back();
            if (++visits > 4ll * N + 8) return RT_ERR_BVH;  // cycle or exploding DAG
            if (nodes[k].leftChild != -1) {
                st.push_back(nodes[k].leftChild);
                st.push_back(nodes[k].rightChild);
                ms = static_cast<int>(st.size()) > ms ? static_cast<int>(st.size()) : ms;
            }
        }
    }
    if (ms > kMaxStack) return RT_ERR_BVH;
    *max_stack = ms;
    return RT_OK;
}

inline float bits_f(int v) {
    float f;
    std::memcpy(&f, &v, sizeof f);
    return f;
}

// Builds the accelerator from the host copies of the scene and uploads it;
// expects geo_lin to be packed (k_pack_prims copies from it). On failure the
// context keeps rendering with k_packet.
// Diagnostics (RT_REBUILD_PROFILE set): wall time of the phases of a host step on
// stderr, each lap since the previous one.
struct PhaseLaps {
    const char* step;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    explicit PhaseLaps(const char* s) : step(s) {}
    void operator()(const char* what) {
        static const bool on = std::getenv("RT_REBUILD_PROFILE") != nullptr;
        if (!on || !step) return;  // (a null step: this instance reports nothing)
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "%s %-24s %8.3f ms\n", step, what, std::chrono::duration<double, std::milli>(t - t0).count());
        t0 = t;
    }
};

// A host array left uninitialised: no serial zeroing pass, its pages are first touched
// by the threads that fill it (config 5's 24 MB of wnodes: 5.4 ms of page faults on one
// thread). Every element is written before the array is read.
template <class T>
struct RawArray {
    std::unique_ptr<T[]> p;
    size_t n;
    explicit RawArray(size_t count) : p(new T[count]), n(count) {}
    T* data() { return p.get(); }
    size_t size() const { return n; }
    T& operator[](size_t i) { return p[i]; }
};

int upload_built_accel(rt_ctx* c);
// built: the host build already ran (rt_upload_scene overlaps it with the records'
// device upload) and returned *built; null: build here.
int build_upload_accel(rt_ctx* c, const bool* built = nullptr) {
    PhaseLaps lap("build_upload_accel");
    free_accel(c);
    const int N = c->N;
    if (N == 0) return RT_OK;
    lap("free");
    if (built ? !*built
              : !rta::build_accel(c->host_shapes.data(), c->S, c->host_nodes.data(), N, c->host_idx.data(), c->I,
                                  kLeafScan, kMaxStack, c->accel, c->build_mt))
        return RT_OK;
    lap("host build");
    return upload_built_accel(c);
}

// The device half of build_upload_accel: c->accel (built) to the device, with the
// current host node records' exact boxes and the device's current shape records.
int upload_built_accel(rt_ctx* c) {
    PhaseLaps lap("  upload");
    const int N = c->N;
    rta::AccelHost& A = c->accel;
    if (N >= (1 << 28)) return RT_OK;  // codes carry the node index in 28 bits
    // The arrays below are packed on the build threads (rta::parallel_for): each entry is
    // written by one thread from read-only inputs.
    constexpr int kPackChunk = 8192;
    // anodes: every reference node's exact box and content box (the root's entry test).
    RawArray<float4> an(4 * static_cast<size_t>(N));
    std::atomic<int> nan_box{0};
    rta::parallel_for(N, kPackChunk, [&](int k0, int k1) {
        int nan = 0;
        for (int k = k0; k < k1; ++k) {
            const FlatNode& n = c->host_nodes[k];
            for (float v : {n.boundsMin.x, n.boundsMin.y, n.boundsMin.z, n.boundsMax.x, n.boundsMax.y, n.boundsMax.z})
                nan |= std::isnan(v) ? 1 : 0;
            const rta::Box3& cb = A.content[k];
            an[4 * k + 0] = make_float4(n.boundsMin.x, n.boundsMin.y, n.boundsMin.z, bits_f(n.leftChild));
            an[4 * k + 1] = make_float4(n.boundsMax.x, n.boundsMax.y, n.boundsMax.z, bits_f(n.rightChild));
            an[4 * k + 2] = make_float4(cb.lo[0], cb.lo[1], cb.lo[2], bits_f(A.flags[k]));
            an[4 * k + 3] = make_float4(cb.hi[0], cb.hi[1], cb.hi[2], 0.f);
        }
        if (nan) nan_box.store(1);
    });
    c->boxes_finite = nan_box.load() ? 0 : 1;
    lap("anodes");
    // lnodes: the wide local nodes (accel.h, build_wide), kWideRec float4 each with
    // quantized cones (kWideRecMt with the MT accelerator's float grazing cones; wide_kids).
    const size_t P = A.prim_shape.size();
    const int rec = A.mt ? kWideRecMt : kWideRec;
    std::atomic<bool> codes_ok{true};
    auto leaf_code = [&](size_t j) -> int {
        const unsigned st = static_cast<unsigned>(-A.la[j] - 1), cnt = static_cast<unsigned>(A.lb[j]);
        if (st >= (1u << 22) || cnt > 63u) codes_ok.store(false);
        return static_cast<int>(kLocal | kLeaf | (st << 6) | cnt);
    };
    // The scene tree's wide nodes (accel.h, SceneTree) follow the local ones;
    // its leaves are item codes (kTopLeaf | kItem | item).
    const rta::SceneTree& T = A.st;
    const bool use_st = T.wroot >= 0;
    const size_t nw = A.wchild.size() / rta::kWide;
    const size_t nws = use_st ? T.wchild.size() / rta::kWide : 0;
    if (nw + nws >= (1u << 27) || T.item_ref.size() >= (1u << 28)) return RT_OK;  // kRecMask, kItem
    // the code of the node whose first record is r (+ base): kPair when it spans two
    auto wide_code = [](const std::vector<char>& pair, int r, size_t base) {
        return static_cast<int>(kLocal | static_cast<unsigned>(base + r) |
                                (r < static_cast<int>(pair.size()) && pair[r] ? kPair : 0u));
    };
    std::vector<float4> ln(rec * (nw + nws ? nw + nws : 1));
    auto emit_wide = [&](size_t w, size_t at, const std::vector<int>& wchild, const std::vector<int>& wsub,
                         const std::vector<char>& wpair, const std::vector<rta::Box3>& boxes,
                         const std::vector<float>& cones, const std::function<int(int)>& leaf_of, size_t sub_base) {
        float v[kWideRecMt][4];
        for (int s2 = 0; s2 < 4; ++s2) {
            const int j = wchild[rta::kWide * w + s2];
            int code = kNoChild;
            float box[6] = {0, 0, 0, 0, 0, 0}, cone[4] = {0, 0, 0, -4.f}, mtc[rta::kMtPadF] = {0, 0, 0, 0, 0, 0};
            if (j >= 0) {
                const rta::Box3& bx = boxes[j];
                for (int a = 0; a < 3; ++a) {
                    box[a] = bx.lo[a];
                    box[3 + a] = bx.hi[a];
                }
                for (int a = 0; a < 4; ++a) cone[a] = cones[4 * j + a];
                if (!c->cone_cull && cone[3] > rta::kNoPrune) cone[3] = A.mt ? 2.f : -4.f;
                if (A.mt && boxes.data() == A.lbox.data())
                    for (int a = 0; a < rta::kMtPadF; ++a) mtc[a] = A.lmt[rta::kMtPadF * j + a];
                const int sub = wsub[rta::kWide * w + s2];
                code = sub < 0 ? leaf_of(j) : wide_code(wpair, sub, sub_base);
            }
            if (A.mt) {  // per child 16 floats: box, cone, the per-ray padding constants
                float* blk = &v[0][0] + 16 * s2;
                for (int a = 0; a < 6; ++a) blk[a] = box[a];
                for (int a = 0; a < 4; ++a) blk[6 + a] = cone[a];
                for (int a = 0; a < rta::kMtPadF; ++a) blk[10 + a] = mtc[a];
            } else {
                for (int a = 0; a < 6; ++a) v[a][s2] = box[a];
                v[6][s2] = bits_f(j < 0 ? rta::kConeNever : rta::cone_word(cone[0], cone[1], cone[2], cone[3]));
            }
            v[rec - 1][s2] = bits_f(code);
        }
        for (int r = 0; r < rec; ++r) ln[rec * at + r] = make_float4(v[r][0], v[r][1], v[r][2], v[r][3]);
    };
    {
        const std::function<int(int)> leaf_of = [&](int j) { return leaf_code(static_cast<size_t>(j)); };
        rta::parallel_for(static_cast<int>(nw), kPackChunk, [&](int w0, int w1) {
            for (size_t w = static_cast<size_t>(w0); w < static_cast<size_t>(w1); ++w)
                emit_wide(w, w, A.wchild, A.wsub, A.wpair, A.lbox, A.lcone, leaf_of, 0);
        });
    }
    lap("local wide nodes");
    // Items: with <= 8 distinct reference leaves (few-leaf mode, few_mask) a
    // local-leaf code kLocal|kLeaf|kItem|start<<6|leaf<<3|count and titems =
    // the leaves' exact boxes; otherwise kTopLeaf|kItem|item and titems = per
    // item its leaf's exact box + prim range.
    std::vector<int> few;
    if (use_st) {
        for (int k : T.item_ref)
            if (std::find(few.begin(), few.end(), k) == few.end()) {
                few.push_back(k);
                if (few.size() > 8) break;
            }
        if (few.size() > 8) few.clear();
        for (size_t i = 0; i < T.item_ref.size() && !few.empty(); ++i)
            if (T.item_count[i] > 7 || T.item_start[i] >= (1 << 22)) few.clear();
    }
    c->nfew = static_cast<int>(few.size());
    auto item_code = [&](int j) {
        const int i = T.item_of[j];
        if (few.empty()) return static_cast<int>(kTopLeaf | kItem | static_cast<unsigned>(i));
        const unsigned f = static_cast<unsigned>(std::find(few.begin(), few.end(), T.item_ref[i]) - few.begin());
        return static_cast<int>(kLocal | kLeaf | kItem | (static_cast<unsigned>(T.item_start[i]) << 6) | (f << 3) |
                                static_cast<unsigned>(T.item_count[i]));
    };
    std::vector<float4> ti(2 * (use_st ? std::max<size_t>(T.item_ref.size(), 1) : 1));
    if (use_st) {
        const std::function<int(int)> item_of = item_code;
        rta::parallel_for(static_cast<int>(nws), kPackChunk, [&](int w0, int w1) {
            for (size_t w = static_cast<size_t>(w0); w < static_cast<size_t>(w1); ++w)
                emit_wide(w, nw + w, T.wchild, T.wsub, T.wpair, T.box, A.st_cone, item_of, nw);
        });
        auto put = [&](size_t i, int ref, int start, int count) {
            const FlatNode& n = c->host_nodes[ref];
            ti[2 * i] = make_float4(n.boundsMin.x, n.boundsMin.y, n.boundsMin.z, bits_f(start));
            ti[2 * i + 1] = make_float4(n.boundsMax.x, n.boundsMax.y, n.boundsMax.z, bits_f(count));
        };
        if (!few.empty())
            for (size_t i = 0; i < few.size(); ++i) put(i, few[i], 0, 0);
        else
            for (size_t i = 0; i < T.item_ref.size(); ++i) put(i, T.item_ref[i], T.item_start[i], T.item_count[i]);
        const std::vector<int>& refs = few.empty() ? T.item_ref : few;
        if (hipMalloc(&c->titem_ref, refs.size() * sizeof(int)) != hipSuccess) return RT_ERR_NO_MEMORY;
        HIP_TRY(hipMemcpyAsync(c->titem_ref, refs.data(), refs.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
        c->n_titems = static_cast<int>(refs.size());
        c->host_titem_ref = refs;
    }
    lap("scene tree nodes, items");
    // wnodes: per reference inner node both children's exact + content boxes;
    // tleaf: per reference leaf its plain range and local root code.
    RawArray<float4> wn(8 * static_cast<size_t>(N));
    RawArray<int4> tl(static_cast<size_t>(N));
    auto top_code_of = [&](int k) {
        return c->host_nodes[k].leftChild == -1 ? static_cast<int>(kTopLeaf | static_cast<unsigned>(k)) : k;
    };
    rta::parallel_for(N, kPackChunk, [&](int k0, int k1) {
        for (int k = k0; k < k1; ++k) {
            const FlatNode& n = c->host_nodes[k];
            if (n.leftChild == -1) {
                const int r = A.local_root[k];
                const int lr = A.wroot[k] >= 0 ? wide_code(A.wpair, A.wroot[k], 0)
                                               : (r >= 0 ? leaf_code(static_cast<size_t>(r)) : kNoChild);
                tl[k] = make_int4(A.plain_start[k], A.plain_count[k], lr, 0);
                for (int q = 0; q < 8; ++q) wn[8 * static_cast<size_t>(k) + q] = make_float4(0.f, 0.f, 0.f, 0.f);
                continue;
            }
            tl[k] = make_int4(0, 0, kNoChild, 0);
            const int ch[2] = {n.leftChild, n.rightChild};
            for (int s2 = 0; s2 < 2; ++s2) {
                const FlatNode& cn = c->host_nodes[ch[s2]];
                const rta::Box3& cb = A.content[ch[s2]];
                float4* q = &wn[8 * static_cast<size_t>(k) + 4 * s2];
                q[0] = make_float4(cn.boundsMin.x, cn.boundsMin.y, cn.boundsMin.z, s2 == 0 ? bits_f(top_code_of(ch[0])) : 0.f);
                q[1] = make_float4(cn.boundsMax.x, cn.boundsMax.y, cn.boundsMax.z, s2 == 0 ? bits_f(top_code_of(ch[1])) : 0.f);
                q[2] = make_float4(cb.lo[0], cb.lo[1], cb.lo[2], bits_f(A.flags[ch[s2]] & 8));
                q[3] = make_float4(cb.hi[0], cb.hi[1], cb.hi[2], 0.f);
            }
        }
    });
    lap("wnodes, tleaf");
    if (!codes_ok.load()) return RT_OK;
    for (size_t i = 0; i < P; ++i)  // PrimRec::st = seq << 2 | type
        if (A.prim_seq[i] < 0 || A.prim_seq[i] >= (1 << 29)) return RT_OK;
    std::vector<int> ps(2 * (P ? P : 1));
    for (size_t i = 0; i < P; ++i) {
        ps[i] = A.prim_shape[i];
        ps[P + i] = A.prim_seq[i];
    }
    lap("prim lists");
    if (hipMalloc(&c->anodes, an.size() * sizeof(float4)) != hipSuccess ||
        hipMalloc(&c->lnodes, ln.size() * sizeof(float4)) != hipSuccess ||
        hipMalloc(&c->wnodes, wn.size() * sizeof(float4)) != hipSuccess ||
        hipMalloc(&c->tleaf, tl.size() * sizeof(int4)) != hipSuccess ||
        hipMalloc(&c->titems, ti.size() * sizeof(float4)) != hipSuccess ||
        hipMalloc(&c->prims, 4 * (P ? P : 1) * sizeof(float4)) != hipSuccess ||
        hipMalloc(&c->prim_idx_dev, ps.size() * sizeof(int)) != hipSuccess)
        return RT_ERR_NO_MEMORY;
    lap("hipMalloc");
    HIP_TRY(hipMemcpyAsync(c->anodes, an.data(), an.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->lnodes, ln.data(), ln.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->wnodes, wn.data(), wn.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->tleaf, tl.data(), tl.size() * sizeof(int4), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->titems, ti.data(), ti.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->prim_idx_dev, ps.data(), ps.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
    if (P > 0)
        hipLaunchKernelGGL(k_pack_prims, dim3((P + 255) / 256), dim3(256), 0, c->stream, c->geo_lin, c->prim_idx_dev,
                           c->prim_idx_dev + P, static_cast<int>(P), c->prims);
    HIP_TRY(hipGetLastError());
    lap("copies issued");
    HIP_TRY(sync_stream(c));  // the host vectors die here
    lap("copies + pack done");
    c->st_root = use_st ? wide_code(T.wpair, T.wroot, nw) : kNoChild;
    c->accel_ok = true;
    c->record_bytes = (an.size() + ln.size() + wn.size() + tl.size() + ti.size() + 4 * P + 2 * static_cast<size_t>(c->S)) *
                      sizeof(float4);
    return RT_OK;
}

// Brings host_nodes up to the boxes rt_animate grew on the device.
int sync_host_nodes(rt_ctx* c) {
    if (!c->nodes_on_device_newer) return RT_OK;
    HIP_TRY(hipMemcpyAsync(c->host_nodes.data(), c->staging_nodes, c->N * sizeof(FlatNode), hipMemcpyDeviceToHost,
                           c->stream));
    HIP_TRY(sync_stream(c));
    c->nodes_on_device_newer = false;
    return RT_OK;
}

// The scene tree's unbounded part (kNoPrune) has boxes padded from the reference
// leaves' exact boxes, which animation and rt_update_nodes change: once they may
// differ from the build's, those wide slots go infinite (entered by every ray; the
// items' exact boxes still gate). Idempotent; reset by every accelerator build.
int open_inf_slots(rt_ctx* c) {
    if (c->inf_open || !c->accel_ok) return RT_OK;
    const rta::AccelHost& A = c->accel;
    const rta::SceneTree& T = A.st;
    c->inf_open = true;
    if (T.wroot < 0) return RT_OK;
    const size_t nw = A.wchild.size() / rta::kWide;
    std::vector<int> slots;
    for (size_t q = 0; q < T.wchild.size(); ++q) {
        const int j = T.wchild[q];
        if (j >= 0 && A.st_cone[4 * static_cast<size_t>(j) + 3] <= rta::kNoPrune)
            slots.push_back(static_cast<int>(4 * nw + q));
    }
    hipFree(c->anim_inf_slots);
    c->anim_inf_slots = nullptr;
    c->n_inf_slots = static_cast<int>(slots.size());
    if (slots.empty()) return RT_OK;
    if (hipMalloc(&c->anim_inf_slots, slots.size() * sizeof(int)) != hipSuccess) return RT_ERR_NO_MEMORY;
    HIP_TRY(hipMemcpyAsync(c->anim_inf_slots, slots.data(), slots.size() * sizeof(int), hipMemcpyHostToDevice,
                           c->stream));
    hipLaunchKernelGGL(k_inf_slots, dim3((c->n_inf_slots + 255) / 256), dim3(256), 0, c->stream, c->anim_inf_slots,
                       c->n_inf_slots, c->lnodes, c->accel.mt ? kWideRecMt : kWideRec);
    HIP_TRY(hipGetLastError());
    return RT_OK;
}

// The device lists of the refit (AnimMaps) for the current scene, accelerator and
// refit set (refit_ids: the animated shapes and those rt_update_shapes rewrote).
// anim_base holds, per entry, the record the accelerator's bounds and cones were
// built from.
int prepare_animation(rt_ctx* c) {
    PhaseLaps lap("  prepare");
    const int n = static_cast<int>(c->refit_ids.size());
    c->anim = AnimMaps{};
    c->n_direct_slot_reads = 0;
    c->refit_of.assign(c->S, -1);
    for (int i = 0; i < n; ++i) c->refit_of[c->refit_ids[i]] = i;
    c->entry_root.clear();
    if (n == 0) return RT_OK;
    const int N = c->N;
    const std::vector<int>& which = c->refit_of;  // shape -> refit entry
    const rta::AccelHost& A = c->accel;
    c->anim_cls.assign(n, rta::UNBOUNDED);
    for (int i = 0; i < n; ++i) {
        rta::Box3 b;
        c->anim_cls[i] = rta::classify(c->anim_base[i], b, A.origin_lim, A.mt);
    }
    // reference nodes listing each shape: the leaves that list it and every node above
    // (CSR: a vector per node took ~6 ms of a config-5 setup)
    std::vector<int> poff(static_cast<size_t>(N) + 1, 0), plist;
    for (int k = 0; k < N; ++k) {
        const FlatNode& nd = c->host_nodes[k];
        if (nd.leftChild != -1) {
            ++poff[nd.leftChild + 1];
            if (nd.rightChild != nd.leftChild) ++poff[nd.rightChild + 1];
        }
    }
    for (int k = 0; k < N; ++k) poff[k + 1] += poff[k];
    plist.resize(poff[N]);
    {
        std::vector<int> fill(poff.begin(), poff.end() - 1);
        for (int k = 0; k < N; ++k) {
            const FlatNode& nd = c->host_nodes[k];
            if (nd.leftChild != -1) {
                plist[fill[nd.leftChild]++] = k;
                if (nd.rightChild != nd.leftChild) plist[fill[nd.rightChild]++] = k;
            }
        }
    }
    std::vector<std::vector<int>> nodes_of(n), slots_of(n), prims_of(n), wpos_of(n);
    std::vector<int> stamp(N, -1);
    for (int k = 0; k < N; ++k) {
        const FlatNode& nd = c->host_nodes[k];
        if (nd.leftChild != -1) continue;
        for (int j = nd.startShapeIdx; j < nd.startShapeIdx + nd.numShapes; ++j) {
            const int i = which[c->host_idx[j]];
            if (i < 0) continue;
            slots_of[i].push_back(j);
            nodes_of[i].push_back(k);
        }
    }
    for (int i = 0; i < n; ++i) {
        std::vector<int>& L = nodes_of[i];
        std::vector<int> todo;
        for (int k : L)
            if (stamp[k] != i) {
                stamp[k] = i;
                todo.push_back(k);
            }
        L.clear();
        while (!todo.empty()) {
            const int k = todo.back();
            todo.pop_back();
            L.push_back(k);
            for (int q = poff[k]; q < poff[k + 1]; ++q)
                if (const int p = plist[q]; stamp[p] != i) {
                    stamp[p] = i;
                    todo.push_back(p);
                }
        }
        std::sort(L.begin(), L.end());
    }
    lap("nodes_of");
    c->entry_root.assign(n, 0);
    for (int i = 0; i < n; ++i) c->entry_root[i] = std::binary_search(nodes_of[i].begin(), nodes_of[i].end(), N - 1);
    if (c->accel_ok) {
        const size_t P = A.prim_shape.size(), M = A.lbox.size();
        std::vector<int> lleaf(P, -1), lparent(M, -1), wpos(M, -1);
        for (size_t j = 0; j < M; ++j) {
            if (A.la[j] < 0) {
                const int st = -A.la[j] - 1;
                for (int q = 0; q < A.lb[j]; ++q) lleaf[st + q] = static_cast<int>(j);
            } else {
                lparent[A.la[j]] = static_cast<int>(j);
                lparent[A.lb[j] & 0x3fffffff] = static_cast<int>(j);
            }
        }
        for (size_t q = 0; q < A.wchild.size(); ++q)
            if (A.wchild[q] >= 0) wpos[A.wchild[q]] = static_cast<int>(q);
        std::vector<int> wstamp(M, -1);
        std::vector<char> dirty(M, 0);
        for (size_t p = 0; p < P; ++p) {
            const int i = which[A.prim_shape[p]];
            if (i < 0) continue;
            prims_of[i].push_back(static_cast<int>(p));
            for (int j = lleaf[p]; j >= 0; j = lparent[j])
                if (wpos[j] >= 0 && wstamp[j] != i) {
                    wstamp[j] = i;
                    wpos_of[i].push_back(wpos[j]);
                    dirty[j] = 1;
                }
        }
    lap("local maps");
        // prim range of every local subtree (contiguous: LocalBuilder emits a subtree's prims together)
        std::vector<int> first(M, 0), end(M, 0);
        for (size_t j = M; j-- > 0;) {  // children have larger indices than their parent
            if (A.la[j] < 0) {
                first[j] = -A.la[j] - 1;
                end[j] = first[j] + A.lb[j];
            } else {
                const int l = A.la[j], r = A.lb[j] & 0x3fffffff;
                if (end[l] != first[r]) return RT_ERR_BVH;  // not contiguous: cannot happen
                first[j] = first[l];
                end[j] = end[r];
            }
        }
        std::vector<int4> work;
        for (size_t j = 0; j < M; ++j)
            if (dirty[j]) work.push_back(make_int4(wpos[j], first[j], end[j], 0));
        // The scene tree (accel.h SceneTree), refit like the local trees: its wide
        // nodes follow the local ones in lnodes (global slot 4*nw + q), a subtree's
        // prims are contiguous. Its unbounded part (kNoPrune: boxes are the padded
        // reference-leaf boxes, which grow) goes infinite while the set is animated;
        // the items' exact boxes follow the grown leaves (k_refit).
    lap("local ranges");
        const rta::SceneTree& T = A.st;
        if (T.wroot >= 0) {
            const size_t nw = A.wchild.size() / rta::kWide, Ms = T.box.size();
            std::vector<int> sparent(Ms, -1), swpos(Ms, -1), sfirst(Ms, -1), send(Ms, -1), sleaf(P, -1);
            for (size_t j = 0; j < Ms; ++j) {
                if (T.a[j] < 0) {
                    const int st = -T.a[j] - 1;
                    sfirst[j] = st;
                    send[j] = st + T.b[j];
                    for (int q = 0; q < T.b[j]; ++q) sleaf[st + q] = static_cast<int>(j);
                } else {
                    sparent[T.a[j]] = static_cast<int>(j);
                    sparent[T.b[j] & 0x3fffffff] = static_cast<int>(j);
                }
            }
            std::function<void(int)> range = [&](int j) {
                if (sfirst[j] >= 0) return;
                const int l = T.a[j], r = T.b[j] & 0x3fffffff;
                range(l);
                range(r);
                sfirst[j] = sfirst[l];
                send[j] = send[r];
            };
            for (size_t j = 0; j < Ms; ++j) range(static_cast<int>(j));
            for (size_t q = 0; q < T.wchild.size(); ++q)
                if (T.wchild[q] >= 0) swpos[T.wchild[q]] = static_cast<int>(4 * nw + q);
            auto noprune = [&](int j) { return A.st_cone[4 * static_cast<size_t>(j) + 3] <= rta::kNoPrune; };
            std::vector<int> sstamp(Ms, -1);
            std::vector<char> sdirty(Ms, 0);
            for (size_t p = 0; p < P; ++p) {
                const int i = which[A.prim_shape[p]];
                if (i < 0 || sleaf[p] < 0) continue;
                for (int j = sleaf[p]; j >= 0; j = sparent[j])
                    if (swpos[j] >= 0 && !noprune(j) && sstamp[j] != i) {
                        sstamp[j] = i;
                        wpos_of[i].push_back(swpos[j]);
                        sdirty[j] = 1;
                    }
            }
            for (size_t j = 0; j < Ms; ++j)
                if (sdirty[j]) work.push_back(make_int4(swpos[j], sfirst[j], send[j], 0));
        }
    lap("scene tree maps");
        std::vector<float4> pb(2 * (P ? P : 1), make_float4(INFINITY, INFINITY, INFINITY, 0.f));
        // per shape its class and box as last classified (the build's, or here for shapes
        // written since: a host rewriting a different 1 % of config 5 every frame had
        // every shape it ever wrote classified again at each change of the set, 11 ms)
        const bool cached = A.shape_cls.size() == static_cast<size_t>(c->S) && c->shape_moved.size() == A.shape_cls.size();
        for (size_t p = 0; p < P; ++p) {
            rta::Box3 b;
            const int sh = A.prim_shape[p];
            int cls;
            if (cached && !c->shape_moved[sh]) {
                cls = A.shape_cls[sh];
                b = A.shape_box[sh];
            } else {
                cls = rta::classify(c->host_shapes[sh], b, A.origin_lim, A.mt);
                if (cached) {
                    c->accel.shape_cls[sh] = cls;
                    c->accel.shape_box[sh] = b;
                    c->shape_moved[sh] = 0;
                }
            }
            if (cls != rta::BOUNDED) {
                pb[2 * p + 1] = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.f);
                continue;
            }
            pb[2 * p] = make_float4(b.lo[0], b.lo[1], b.lo[2], 0.f);
            pb[2 * p + 1] = make_float4(b.hi[0], b.hi[1], b.hi[2], 0.f);
        }
    lap("prim boxes (classify)");
        // per dirty slot: the box of its prims outside the refit set (they never move
        // while this set stands) and the list of those in it, which k_refit unions per frame
        c->dirty_max = c->dirty_sum = 0;
        // slots whose refit list takes a wave more than one step (kBigList) first, one
        // workgroup each; the rest kRefitWaves to a workgroup, one wave each (k_refit)
        {
            std::vector<char> big(work.size(), 0);
            for (size_t q = 0; q < work.size(); ++q) {
                int n_ref = 0;
                for (int p = work[q].y; p < work[q].z; ++p) n_ref += which[A.prim_shape[p]] >= 0;
                big[q] = n_ref > kBigList;
            }
            std::vector<int4> ord;
            for (int pass = 1; pass >= 0; --pass)
                for (size_t q = 0; q < work.size(); ++q)
                    if (big[q] == pass) ord.push_back(work[q]);
            c->n_big = static_cast<int>(std::count(big.begin(), big.end(), 1));
            work.swap(ord);
        }
        std::vector<float4> st(2 * (work.empty() ? 1 : work.size()));
        std::vector<int> dl;
        for (size_t q = 0; q < work.size(); ++q) {
            int4& w4 = work[q];
            c->dirty_max = std::max(c->dirty_max, w4.z - w4.y);
            c->dirty_sum += w4.z - w4.y;
            w4.w = static_cast<int>(dl.size());
            float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
            for (int p = w4.y; p < w4.z; ++p) {
                if (which[A.prim_shape[p]] >= 0) {
                    dl.push_back(p);
                    continue;
                }
                const float4 a = pb[2 * static_cast<size_t>(p)], b = pb[2 * static_cast<size_t>(p) + 1];
                lo[0] = std::min(lo[0], a.x), lo[1] = std::min(lo[1], a.y), lo[2] = std::min(lo[2], a.z);
                hi[0] = std::max(hi[0], b.x), hi[1] = std::max(hi[1], b.y), hi[2] = std::max(hi[2], b.z);
            }
            st[2 * q] = make_float4(lo[0], lo[1], lo[2], 0.f);
            st[2 * q + 1] = make_float4(hi[0], hi[1], hi[2], 0.f);
        }
    lap("slot static boxes");
        const int nw = static_cast<int>(work.size());
        work.push_back(make_int4(0, 0, 0, static_cast<int>(dl.size())));  // the end of the last list
        if (dl.empty()) dl.push_back(0);
        hipFree(c->pbox);
        hipFree(c->refit_dirty);
        hipFree(c->refit_static);
        hipFree(c->refit_list);
        c->pbox = nullptr;
        c->refit_dirty = nullptr;
        c->refit_static = nullptr;
        c->refit_list = nullptr;
        c->n_dirty = 0;
        if (hipMalloc(&c->pbox, pb.size() * sizeof(float4)) != hipSuccess ||
            hipMalloc(&c->refit_dirty, work.size() * sizeof(int4)) != hipSuccess ||
            hipMalloc(&c->refit_static, st.size() * sizeof(float4)) != hipSuccess ||
            hipMalloc(&c->refit_list, dl.size() * sizeof(int)) != hipSuccess)
            return RT_ERR_NO_MEMORY;
        HIP_TRY(hipMemcpyAsync(c->pbox, pb.data(), pb.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipMemcpyAsync(c->refit_dirty, work.data(), work.size() * sizeof(int4), hipMemcpyHostToDevice,
                               c->stream));
        HIP_TRY(hipMemcpyAsync(c->refit_static, st.data(), st.size() * sizeof(float4), hipMemcpyHostToDevice,
                               c->stream));
        HIP_TRY(hipMemcpyAsync(c->refit_list, dl.data(), dl.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
        c->n_dirty = nw;
        c->n_direct_slot_reads = static_cast<long long>(work.back().w);  // the slots' refit prims
        const int rc = open_inf_slots(c);
        if (rc != RT_OK) return rc;
    }
    lap("slot uploads");
    // one int allocation: ids, then (offsets, list) x 4
    std::vector<int> buf(c->refit_ids);
    auto append = [&](const std::vector<std::vector<int>>& lists, size_t& off_at, size_t& list_at) {
        off_at = buf.size();
        int run = 0;
        buf.push_back(0);
        for (const auto& l : lists) buf.push_back(run += static_cast<int>(l.size()));
        list_at = buf.size();
        for (const auto& l : lists) buf.insert(buf.end(), l.begin(), l.end());
    };
    // per reference node, the animated shapes it lists (k_refit's node role)
    std::vector<int> node_ids;
    std::vector<std::vector<int>> lists_of;
    {
        std::vector<int> slot(N, -1);
        for (int i = 0; i < n; ++i)
            for (int k : nodes_of[i]) {
                if (slot[k] < 0) {
                    slot[k] = static_cast<int>(node_ids.size());
                    node_ids.push_back(k);
                    lists_of.emplace_back();
                }
                lists_of[slot[k]].push_back(i);
            }
    }
    // per grown node, where its box is copied (k_refit writes them through): the
    // wnodes child slots of its parent(s) and the scene-tree items it gates
    std::vector<std::vector<int>> wn_of(node_ids.size()), items_of(node_ids.size());
    {
        std::vector<int> slot(N, -1);
        for (size_t j = 0; j < node_ids.size(); ++j) slot[node_ids[j]] = static_cast<int>(j);
        for (int p = 0; p < N; ++p) {
            const FlatNode& nd = c->host_nodes[p];
            if (nd.leftChild == -1) continue;
            if (slot[nd.leftChild] >= 0) wn_of[slot[nd.leftChild]].push_back(2 * p);
            if (slot[nd.rightChild] >= 0) wn_of[slot[nd.rightChild]].push_back(2 * p + 1);
        }
        if (c->accel_ok && c->titems)
            for (size_t i = 0; i < c->host_titem_ref.size(); ++i) {
                const int k = c->host_titem_ref[i];
                if (k >= 0 && k < N && slot[k] >= 0) items_of[slot[k]].push_back(static_cast<int>(i));
            }
    }
    size_t o[12];
    append(slots_of, o[0], o[1]);
    append(prims_of, o[2], o[3]);
    append(wpos_of, o[4], o[5]);
    append(lists_of, o[6], o[7]);
    c->direct_reads = n + c->n_direct_slot_reads;
    for (const auto& l : lists_of) c->direct_reads += static_cast<long long>(l.size());
    append(wn_of, o[8], o[9]);
    append(items_of, o[10], o[11]);
    const size_t o_ids = buf.size();
    buf.insert(buf.end(), node_ids.begin(), node_ids.end());
    const size_t o_cls = buf.size();  // per entry: the class the accelerator was built with
    buf.insert(buf.end(), c->anim_cls.begin(), c->anim_cls.end());
    const size_t o_pe = buf.size();   // per accelerator prim: its shape's refit entry (-1: none)
    for (size_t p = 0; p < (c->accel_ok ? A.prim_shape.size() : 0); ++p) buf.push_back(which[A.prim_shape[p]]);
    lap("node lists");
    int rc = ensure_staging(c->anim_maps, c->anim_maps_cap, buf.size());
    if (rc != RT_OK) return rc;
    HIP_TRY(hipMemcpyAsync(c->anim_maps, buf.data(), buf.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(sync_stream(c));
    lap("maps upload + sync");
    const int* d = c->anim_maps;
    c->anim = AnimMaps{d,        d + o[0], d + o[1],  d + o[2],  d + o[3], d + o[4], d + o[5], d + o_ids,
                       d + o[6], d + o[7], d + o[8], d + o[9], d + o[10], d + o[11], d + o_cls, d + o_pe,
                       n,
                       static_cast<int>(node_ids.size())};
    return ensure_staging(c->anim_sbox, c->anim_sbox_cap, 4 * static_cast<size_t>(n));
}

// The root's box from the host's node records (rt_upload_scene, rt_update_nodes).
void set_root(rt_ctx* c) {
    if (c->N <= 0 || static_cast<int>(c->host_nodes.size()) != c->N) return;
    const FlatNode& r = c->host_nodes[c->N - 1];
    const float lo[3] = {r.boundsMin.x, r.boundsMin.y, r.boundsMin.z}, hi[3] = {r.boundsMax.x, r.boundsMax.y, r.boundsMax.z};
    std::memcpy(c->root_lo, lo, sizeof lo);
    std::memcpy(c->root_hi, hi, sizeof hi);
}

// (Re)builds the accelerator after the host copies changed, then the animation lists.
int upload_accel(rt_ctx* c, const bool* built = nullptr) {
    discard_rebuild(c);
    c->st_suspended = false;
    int rc = sync_host_nodes(c);
    if (rc != RT_OK) return rc;
    rc = build_upload_accel(c, built);
    c->shape_moved.assign(c->S, 0);  // built from the current host records
    // the degraded-bound reports of earlier refits concern the accelerator this replaced
    // (prepare_animation alone, when the refit set changes, keeps them: same accelerator)
    for (bool& pend : c->report_pending) pend = false;
    // the refit set stays (its shapes tend to move again), with the records just built from
    c->anim_base.resize(c->refit_ids.size());
    for (size_t i = 0; i < c->refit_ids.size(); ++i) c->anim_base[i] = c->host_shapes[c->refit_ids[i]];
    c->nodes_rebuild = c->bounds_rebuild = false;
    const int rc2 = prepare_animation(c);
    return rc != RT_OK ? rc : rc2;
}

// Whether every reachable inner node's children lie inside its box (accel.cpp
// boxes_nest), the condition the scene tree was built on.
bool host_nodes_nest(const rt_ctx* c) {
    const int N = c->N;
    if (N <= 0) return true;
    auto in = [](const FlatNode& p, const FlatNode& q) {
        const float* plo = &p.boundsMin.x;
        const float* phi = &p.boundsMax.x;
        const float* qlo = &q.boundsMin.x;
        const float* qhi = &q.boundsMax.x;
        for (int a = 0; a < 3; ++a)
            if (!(plo[a] <= qlo[a] && qlo[a] <= phi[a] && plo[a] <= qhi[a] && qhi[a] <= phi[a])) return false;
        return true;
    };
    std::vector<char> seen(N, 0);
    std::vector<int> st{N - 1};
    while (!st.empty()) {
        const int k = st.back();
        st.pop_back();
        if (seen[k]) continue;
        seen[k] = 1;
        const FlatNode& nd = c->host_nodes[k];
        if (nd.leftChild == -1) continue;
        if (!in(nd, c->host_nodes[nd.leftChild]) || !in(nd, c->host_nodes[nd.rightChild])) return false;
        st.push_back(nd.leftChild);
        st.push_back(nd.rightChild);
    }
    return true;
}

// Asynchronous rebuild (rt_ctx::AsyncBuild). A running build is joined and dropped
// by anything that replaces the scene or rebuilds synchronously.
void discard_rebuild(rt_ctx* c) {
    if (!c->rebuild) return;
    if (c->rebuild->th.joinable()) c->rebuild->th.join();
    c->rebuild.reset();
}

// Starts the rebuild over a snapshot of the host records (device-grown node boxes
// fetched first). A rebuild already running is left to finish: the refit that lands it
// checks the kinds of bound and the nesting again.
int start_rebuild(rt_ctx* c) {
    if (c->rebuild) return RT_OK;
    ++c->anim_rebuilds;
    const int rc = sync_host_nodes(c);
    if (rc != RT_OK) return rc;
    if (c->nodes_rebuild) c->st_suspended = true;  // exact meanwhile: the reference tree only
    c->nodes_rebuild = false;
    std::unique_ptr<rt_ctx::AsyncBuild> b = c->spare ? std::move(c->spare) : std::make_unique<rt_ctx::AsyncBuild>();
    b->done.store(false);
    b->ok = false;
    b->shapes.assign(c->host_shapes.begin(), c->host_shapes.end());  // into the spare's capacity
    b->nodes.assign(c->host_nodes.begin(), c->host_nodes.end());
    rt_ctx::AsyncBuild* raw = b.get();
    const std::vector<int>* idx = &c->host_idx;  // fixed while the build runs: an upload joins it first
    const int S = c->S, N = c->N, I = c->I;
    const bool mt = c->build_mt;
    raw->th = std::thread([raw, idx, S, N, I, mt] {
        try {  // (bad_alloc: swapped in as a failed build, no accelerator; never past the thread)
            raw->ok = rta::build_accel(raw->shapes.data(), S, raw->nodes.data(), N, idx->data(), I, kLeafScan,
                                       kMaxStack, raw->A, mt);
        } catch (...) {
            raw->A = rta::AccelHost();
            raw->ok = false;
        }
        raw->done.store(true, std::memory_order_release);
    });
    c->rebuild = std::move(b);
    return RT_OK;
}

// Swaps a finished rebuild in: its accelerator to the device (the frames in flight end
// first), then every shape whose record differs from the snapshot, and the animated
// ones, form the refit set with their snapshot records as the build-time base, so the
// next refit brings the new accelerator to the current records (the caller's flush).
int finish_rebuild(rt_ctx* c, bool* refit) {
    if (!c->rebuild || !c->rebuild->done.load(std::memory_order_acquire)) return RT_OK;
    PhaseLaps lap("finish_rebuild");
    std::unique_ptr<rt_ctx::AsyncBuild> b = std::move(c->rebuild);
    b->th.join();
    lap("join");
    int rc = sync_host_nodes(c);
    if (rc != RT_OK) return rc;
    HIP_TRY(sync_stream(c));
    lap("sync");
    free_accel(c);
    c->st_suspended = false;
    for (bool& pend : c->report_pending) pend = false;  // reports about the accelerator replaced
    ++c->async_swaps;
    // the replaced accelerator's host arrays go to b->A, freed by the next build's thread
    std::swap(c->accel, b->A);
    if (!b->ok) {  // as a failed synchronous build: no accelerator (k_packet)
        c->accel = rta::AccelHost();
        c->refit_ids.clear();
        c->anim_base.clear();
        c->spare = std::move(b);
        return prepare_animation(c);
    }
    lap("free");
    if ((rc = upload_built_accel(c)) != RT_OK) return rc;
    lap("upload");
    std::vector<char> in(c->S, 0);
    std::vector<int> ids;
    std::vector<FlatShape> base;
    auto add = [&](int id) {
        if (in[id]) return;
        in[id] = 1;
        ids.push_back(id);
        base.push_back(b->shapes[id]);
    };
    for (int id : c->anim_ids) add(id);
    c->shape_moved.assign(c->S, 0);
    for (int id = 0; id < c->S; ++id)
        if (std::memcmp(&c->host_shapes[id], &b->shapes[id], sizeof(FlatShape)) != 0) {
            add(id);
            c->shape_moved[id] = 1;
        }
    c->refit_ids.swap(ids);
    c->anim_base.swap(base);
    // pending writes stay pending (upd_ids): their shapes are in the set with the snapshot base
    for (auto& ub : c->upd_base) ub.second = b->shapes[ub.first];
    // the node records since the snapshot are in every copy already (upload_built_accel read
    // host_nodes; pending ones stay nodes_dirty); boxes that do not nest (any more) rebuild
    // again, exact meanwhile
    c->nodes_rebuild = c->accel_ok && c->accel.st.wroot >= 0 && !host_nodes_nest(c);
    *refit = !c->refit_ids.empty();
    lap("refit set");
    rc = prepare_animation(c);
    lap("prepare_animation");
    c->spare = std::move(b);  // reused by the next rebuild (not freed here)
    return rc;
}

// Reads the report words of earlier refits whose k_refit has run (block: wait for
// them): a shape whose bound changed kind leaves the accelerator exact but slower
// (k_refit enters every box above it) until the host rebuilds it.
// Every refit slot is free once the stream has drained: no event needed.
void stream_drained(rt_ctx* c) {
    c->mark_slot = -1;
    for (bool& b : c->slot_busy) b = false;
}

// hipStreamSynchronize of the context's stream, which also retires its refit slots
// (and its sub-contexts', which run on the same stream).
hipError_t sync_stream(rt_ctx* c) {
    hipError_t e = hipStreamSynchronize(c->stream);
    for (rt_ctx* x : {c, c->brute, c->mtc})
        if (e == hipSuccess && x && x->order_stream) {
            e = hipStreamSynchronize(x->order_stream);
            if (e == hipSuccess) x->order_pending = false;
        }
    if (e == hipSuccess)
        for (rt_ctx* x : {c, c->brute, c->mtc})
            if (x) stream_drained(x);
    return e;
}

// The host is about to free or reuse the cost order's buffers: the order stream's kernels end first.
hipError_t sync_order(rt_ctx* c) {
    if (!c->order_stream) return hipSuccess;
    const hipError_t e = hipStreamSynchronize(c->order_stream);
    if (e == hipSuccess) c->order_pending = false;
    return e;
}

// The next accelerated dispatch reads the order the order stream wrote: the context's
// stream waits for it (a device-side wait, the host does not block).
hipError_t join_order(rt_ctx* c) {
    if (!c->order_pending) return hipSuccess;
    c->order_pending = false;
    return hipStreamWaitEvent(c->stream, c->order_done, 0);
}

// Records the anim_copied event of the last k_refit's slot if it is still pending.
int record_mark(rt_ctx* c) {
    if (c->mark_slot < 0) return RT_OK;
    const int s = c->mark_slot;
    c->mark_slot = -1;
    HIP_TRY(hipEventRecord(c->anim_copied[s], c->stream));
    return RT_OK;
}

int check_reports(rt_ctx* c, bool block = false) {
    for (int s = 0; s < rt_ctx::kAnimRing; ++s) {
        if (!c->report_pending[s]) continue;
        if (s == c->mark_slot) {  // its event is not recorded yet: not done unless waited for
            if (!block) continue;
            if (const int rc = record_mark(c)) return rc;
        }
        if (block) {
            HIP_TRY(hipEventSynchronize(c->anim_copied[s]));
        } else {
            const hipError_t e = hipEventQuery(c->anim_copied[s]);
            if (e == hipErrorNotReady) continue;
            if (e != hipSuccess) return RT_ERR_DEVICE;
        }
        c->report_pending[s] = false;
        const int* rep = reinterpret_cast<const int*>(static_cast<const char*>(c->anim_pinned[s]) + c->report_at[s]);
        if (*rep) c->bounds_rebuild = true;
    }
    return RT_OK;
}

// A slot of the pinned ring k_refit reads from, `bytes` large plus its report word;
// waits for that slot's previous k_refit (kAnimRing flushes back).
int pinned_slot(rt_ctx* c, size_t bytes, char** host, const char** dev) {
    const int slot = c->anim_slot;
    c->anim_slot = (slot + 1) % rt_ctx::kAnimRing;
    if (!c->anim_copied[slot]) {
        HIP_TRY(hipEventCreateWithFlags(&c->anim_copied[slot], hipEventDisableTiming));
    } else if (c->slot_busy[slot]) {
        if (slot == c->mark_slot && record_mark(c) != RT_OK) return RT_ERR_DEVICE;
        HIP_TRY(hipEventSynchronize(c->anim_copied[slot]));  // this slot's last k_refit has run
        c->slot_busy[slot] = false;
        if (const int rc = check_reports(c)) return rc;
    }
    bytes = (bytes + 15) / 16 * 16;
    if (c->anim_pinned_cap[slot] < bytes + 16) {
        if (c->anim_pinned[slot]) hipHostFree(c->anim_pinned[slot]);
        c->anim_pinned[slot] = nullptr;
        c->anim_pinned_dev[slot] = nullptr;
        c->anim_pinned_cap[slot] = 0;
        // mapped and coherent: the kernel reads it over the host link, never a stale cached copy
        if (hipHostMalloc(&c->anim_pinned[slot], bytes + 16, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
            return RT_ERR_NO_MEMORY;
        if (hipHostGetDevicePointer(&c->anim_pinned_dev[slot], c->anim_pinned[slot], 0) != hipSuccess)
            return RT_ERR_DEVICE;
        c->anim_pinned_cap[slot] = bytes + 16;
    }
    c->report_at[slot] = bytes;
    *host = static_cast<char*>(c->anim_pinned[slot]);
    *dev = static_cast<const char*>(c->anim_pinned_dev[slot]);
    *reinterpret_cast<int*>(*host + bytes) = 0;
    return slot;
}

// The refit set only grows while shapes join it (rt_update_shapes of a shape not in
// it), and every flush copies and refits all of it. A host that writes a different
// few shapes each frame would make that every shape it ever touched. So once the
// entries that are neither animated nor written since the last flush ("stale")
// outnumber kRefitSlack, S / 16 and the live ones, they leave the set: their device
// records are current (the last flush that listed them wrote them), and
// prepare_animation folds their current boxes into the slots' fixed parts, which it
// recomputes from the host records. An entry whose bound changed kind since the build
// stays (the fixed part has no box for it; its report rebuilds the accelerator).
// Per-flush entries stay below about 2 x live + max(kRefitSlack, S / 16).
constexpr size_t kRefitSlack = 4096;
void compact_refit_set(rt_ctx* c) {
    const size_t n = c->refit_ids.size(), live = c->anim_ids.size() + c->upd_ids.size();
    if (n <= live || n - live <= std::max({kRefitSlack, static_cast<size_t>(c->S) / 16, live})) return;
    std::vector<char> keep_shape(c->S, 0);
    for (int id : c->anim_ids) keep_shape[id] = 1;
    for (int id : c->upd_ids) keep_shape[id] = 1;
    std::vector<int> ids;
    std::vector<FlatShape> base;
    for (size_t i = 0; i < n; ++i) {
        const int id = c->refit_ids[i];
        bool keep = keep_shape[id] != 0;
        if (!keep && i < c->anim_cls.size()) {
            rta::Box3 b;
            keep = rta::classify(c->host_shapes[id], b, c->accel.origin_lim, c->accel.mt) != c->anim_cls[i];
        }
        if (keep) {
            ids.push_back(id);
            base.push_back(c->anim_base[i]);
        }
    }
    c->refit_ids.swap(ids);
    c->anim_base.swap(base);
    ++c->refit_compactions;
}

// Applies what rt_update_shapes / rt_update_nodes left on the host, and an
// rt_animate frame (grow: the animated entries grow the nodes listing them, as
// updateBVH does), to every device copy with one launch of k_refit on the stream:
// every refit entry's records (read from the pinned ring), the nodes listing an
// entry (their content boxes; with grow their exact boxes), the local and
// scene-tree boxes above its prims, and the host's node records (rt_update_nodes).
// The host does no per-shape work beyond copying the records: whether a bound
// changed kind is decided by k_refit, which keeps such a frame exact and reports it.
// The host rebuilds the accelerator (for speed) once a report comes in, and (for
// exactness of the scene tree) when new node boxes stop nesting. Called by every
// operation that reads the device scene.
int flush_updates(rt_ctx* c, bool grow = false) {
    if (!c->have_scene) return RT_OK;
    bool swapped = false;  // a rebuilt accelerator landed: its refit set is refit now
    int rc = finish_rebuild(c, &swapped);
    if (rc != RT_OK) return rc;
    PhaseLaps lap(swapped ? "flush after swap" : nullptr);
    rc = check_reports(c);
    if (rc != RT_OK) return rc;
    lap("check_reports");
    const bool gbox = c->grow_pending && !c->anim_ids.empty();
    const bool work = !c->upd_ids.empty() || c->nodes_dirty || grow || gbox || swapped;
    if (!work && !c->bounds_rebuild) return RT_OK;
    if (work) {
        // shapes new to the refit set join it with their build-time records
        bool added = false;
        for (const auto& ub : c->upd_base)
            if (c->refit_of[ub.first] < 0) {
                c->refit_of[ub.first] = static_cast<int>(c->refit_ids.size());
                c->refit_ids.push_back(ub.first);
                c->anim_base.push_back(ub.second);
                added = true;
            }
        if (added) compact_refit_set(c);
        if (added && (rc = prepare_animation(c)) != RT_OK) return rc;
        lap("refit set joined");
        const int n = static_cast<int>(c->refit_ids.size());
        const bool nodes = c->nodes_dirty && c->N > 0;
        const size_t rec_bytes = static_cast<size_t>(n) * (sizeof(FlatShape) + sizeof(int));
        const size_t node_bytes = nodes ? static_cast<size_t>(c->N) * sizeof(FlatNode) : 0;
        const size_t box_at = (rec_bytes + node_bytes + 15) / 16 * 16;  // growth boxes (AF_BOX), 2 float4 per entry
        const size_t bytes = gbox ? box_at + static_cast<size_t>(n) * 2 * sizeof(float4) : rec_bytes + node_bytes;
        c->last_flush_bytes = static_cast<long long>(bytes);
        if (bytes > 0) {
            char* pin = nullptr;
            const char* pin_dev = nullptr;
            const int slot = pinned_slot(c, bytes, &pin, &pin_dev);
            if (slot < 0) return slot;
            lap("pinned slot");
            for (int i = 0; i < n; ++i)
                std::memcpy(pin + i * sizeof(FlatShape), &c->host_shapes[c->refit_ids[i]], sizeof(FlatShape));
            int* flags = reinterpret_cast<int*>(pin + n * sizeof(FlatShape));
            std::memset(flags, 0, n * sizeof(int));
            if (grow)
                for (int id : c->anim_ids) flags[c->refit_of[id]] = AF_GROW;
            if (gbox) {
                float4* gb = reinterpret_cast<float4*>(pin + box_at);
                for (size_t k = 0; k < c->anim_ids.size(); ++k) {
                    const int e = c->refit_of[c->anim_ids[k]];
                    const float* b = &c->grow_box[6 * k];
                    flags[e] = AF_GROW | AF_BOX;
                    gb[2 * e] = make_float4(b[0], b[1], b[2], 0.f);
                    gb[2 * e + 1] = make_float4(b[3], b[4], b[5], 0.f);
                }
            }
            if (nodes) std::memcpy(pin + rec_bytes, c->host_nodes.data(), c->N * sizeof(FlatNode));
            const bool acc = c->accel_ok;
            const size_t P = c->accel.prim_shape.size();
            const AnimOut out{c->staging_shapes, c->staging_nodes, c->geo_lin, c->geo_leaf, c->mat, c->nodes,
                              acc ? c->anodes : nullptr, acc ? c->lnodes : nullptr, acc ? c->prims : nullptr,
                              acc ? c->wnodes : nullptr, acc ? c->titems : nullptr,
                              acc ? c->pbox : nullptr, acc ? c->prim_idx_dev + P : nullptr, c->anim_sbox,
                              c->accel.origin_lim, c->accel.mt ? 1 : 0,
                              {c->accel.mt_z[0], c->accel.mt_z[1], c->accel.mt_z[2]},
                              acc ? c->prim_idx_dev : nullptr, c->cone_cull};
            if (!c->refit_ctr) {
                const size_t words = kRefitFlag0 + 16 * kRefitFlags;  // tickets, done, then the flags
                if (hipMalloc(&c->refit_ctr, words * sizeof(unsigned)) != hipSuccess) return RT_ERR_NO_MEMORY;
                HIP_TRY(hipMemsetAsync(c->refit_ctr, 0, words * sizeof(unsigned), c->stream));
                c->ctr_tickets = c->ctr_done = 0;
            }
            // mode 4: the records copied to the device first, then read there by every role
            // (direct, one launch): one crossing of the host link instead of one per reader
            const char* src = pin_dev;
            const int mode = c->refit_mode >= 0 ? c->refit_mode : c->direct_reads <= kDirectReads ? 2 : 1;
            if (mode == 4) {
                if (c->refit_dev_cap < bytes) {
                    hipFree(c->refit_dev);
                    c->refit_dev = nullptr;
                    c->refit_dev_cap = 0;
                    if (hipMalloc(&c->refit_dev, bytes) != hipSuccess) return RT_ERR_NO_MEMORY;
                    c->refit_dev_cap = bytes;
                }
                HIP_TRY(hipMemcpyAsync(c->refit_dev, pin, bytes, hipMemcpyHostToDevice, c->stream));
                src = c->refit_dev;
            }
            const int waves = mode == 2 ? 1 : kRefitWaves;  // per workgroup of a single launch
            RefitArgs r{};
            r.fresh = reinterpret_cast<const FlatShape*>(src);
            r.flags = reinterpret_cast<const int*>(src + n * sizeof(FlatShape));
            r.gbox = gbox ? reinterpret_cast<const float4*>(src + box_at) : nullptr;
            r.nsrc = nodes ? reinterpret_cast<const FlatNode*>(src + rec_bytes) : nullptr;
            r.report = reinterpret_cast<int*>(const_cast<char*>(pin_dev) + c->report_at[slot]);
            r.ctr = c->refit_ctr;
            r.tbase = c->ctr_tickets;
            r.abase = c->ctr_done;
            const int per = 64 * (mode == 1 ? 1 : waves);  // record / node-set lanes per workgroup
            r.na = (n + per - 1) / per;
            r.N = c->N;
            r.n_items = nodes && acc ? c->n_titems : 0;
            r.titem_ref = c->titem_ref;
            r.nd = nodes ? (c->N + r.n_items + per - 1) / per : 0;
            r.nb = n > 0 ? c->anim.nodes : 0;
            r.dirty = c->refit_dirty;
            r.n_big = c->n_big;
            r.dstatic = c->refit_static;
            r.dlist = c->refit_list;
            r.n_dirty = n > 0 && acc ? c->n_dirty : 0;
            r.rec = c->accel.mt ? kWideRecMt : kWideRec;
            r.wait = mode == 0 ? 1 : mode == 3 ? 2 : 0;
            r.direct = mode == 2 || mode == 4;
            // waves per workgroup: the node and slot roles' own launch takes kRefitWaves (a
            // slot's or node's list in one step), a launch with the one-wave roles one
            auto go = [&](const RefitArgs& ra, int waves) -> int {
                const int small = std::max(0, ra.n_dirty - ra.n_big);
                const int grid = ra.na + ra.nd + ra.nb + std::min(ra.n_big, ra.n_dirty) + (small + waves - 1) / waves;
                if (grid == 0) return RT_OK;
                hipLaunchKernelGGL(k_refit, dim3(grid), dim3(64 * waves), 0, c->stream, c->anim, out, ra);
                HIP_TRY(hipGetLastError());
                if (ra.wait == 1) c->ctr_tickets += static_cast<unsigned>(grid);
                if (ra.wait) c->ctr_done += static_cast<unsigned>(ra.na);
                return RT_OK;
            };
            if (mode == 1) {  // records and node sets, then (a kernel boundary later) the boxes
                RefitArgs r1 = r, r2 = r;
                r1.nb = r1.n_dirty = 0;
                r2.na = r2.nd = 0;
                if ((rc = go(r1, 1)) != RT_OK || (rc = go(r2, kRefitWaves)) != RT_OK) return rc;
            } else if ((rc = go(r, waves)) != RT_OK) {
                return rc;
            }
            lap("records staged, k_refit launched");
            // the slot may be refilled once its event (recorded behind the next dispatch) is done
            if ((rc = record_mark(c)) != RT_OK) return rc;
            c->mark_slot = slot;
            c->slot_busy[slot] = true;
            ++c->refit_launches;  // rt_sync_frame: a slot taken since the frame's dispatch
            c->report_pending[slot] = n > 0 && acc;
            if (nodes && (rc = open_inf_slots(c)) != RT_OK) return rc;
        }
        if (grow || gbox) c->nodes_on_device_newer = true;  // the device grew the nodes past host_nodes
        if (gbox) {
            c->grow_pending = false;
            for (size_t k = 0; k < c->anim_ids.size(); ++k)
                for (int a = 0; a < 3; ++a) {
                    c->grow_box[6 * k + a] = INFINITY;
                    c->grow_box[6 * k + 3 + a] = -INFINITY;
                }
        }
        c->nodes_dirty = false;
        for (int id : c->upd_ids) c->upd_mark[id] = 0;
        c->upd_ids.clear();
        c->upd_base.clear();
        lap("flush end");
    }
    if (!c->nodes_rebuild && !c->bounds_rebuild) {
        ++c->updates_flushed;
        return RT_OK;
    }
    // a bound changed kind (reported by an earlier k_refit), or the node boxes stopped
    // nesting: rebuild from the host copies (which the refit above brought to the device),
    // on a host thread while the frames go on (rt_ctx::AsyncBuild), or here
    c->bounds_rebuild = false;
    if (c->async_rebuild) return start_rebuild(c);
    ++c->anim_rebuilds;
    return upload_accel(c);
}

size_t sched_set_words(int tiles) {
    return static_cast<size_t>((tiles + kOrderThreads - 1) / kOrderThreads) * kOrderBuckets;
}

int fill_kparams(rt_ctx* c, int width, int height, int y0, int stripe, int period, int out_rows, float* dst,
                 size_t pitch, KParams& kp, int format = RT_FORMAT_RGBA32F) {
    if (!c->have_scene || !c->have_cam || !c->have_light) return RT_ERR_NO_SCENE;
    const size_t px = format == RT_FORMAT_RGB32F ? 12 : 16, align = format == RT_FORMAT_RGB32F ? 4 : 16;
    if (width <= 0 || height <= 0 || stripe <= 0 || period < stripe || out_rows < 0 || y0 < 0 || !dst ||
        (format != RT_FORMAT_RGBA32F && format != RT_FORMAT_RGB32F && format != RT_FORMAT_RGBA32F_IMAGE) ||
        pitch < static_cast<size_t>(width) * px ||
        (pitch % align) != 0 || (reinterpret_cast<uintptr_t>(dst) % align) != 0)
        return RT_ERR_INVALID;
    std::memset(&kp, 0, sizeof kp);
    kp.geo_leaf = c->geo_leaf;
    kp.geo_lin = c->geo_lin;
    kp.mat = c->mat;
    kp.nodes = c->nodes;
    kp.S = c->S;
    kp.N = c->N;
    kp.I = c->I;
    kp.max_stack = c->max_stack < 1 ? 1 : c->max_stack;
    const FlatCamera& cam = c->cam;
    kp.cam_pos = V{cam.Position.x, cam.Position.y, cam.Position.z};
    kp.cam_front = V{cam.Front.x, cam.Front.y, cam.Front.z};
    kp.cam_right = V{cam.Right.x, cam.Right.y, cam.Right.z};
    kp.cam_up = V{cam.Up.x, cam.Up.y, cam.Up.z};
    // gpu_shader.comp:156-157 (radians = deg * 0.0174532925..., glm/GLSL).
    const float h = 2.0f * std::tan((cam.fov / 2.0f) * 0.01745329251994329576923690768489f);
    kp.plane_h = h;
    kp.plane_w = h * cam.aspectRatio;
    kp.light_pos = V{c->light.position.x, c->light.position.y, c->light.position.z};
    kp.light_color = V{c->light.color.x, c->light.color.y, c->light.color.z};
    kp.resX = c->params.resX;
    kp.resY = c->params.resY;
    kp.maxBounces = c->params.maxBounces;
    kp.useBVH = c->params.useBVH;
    kp.useFresnel = c->params.useFresnel;
    kp.useMT = c->params.useMollerTrumbore;
    kp.width = width;
    kp.height = height;
    kp.y0 = y0;
    kp.stripe = stripe;
    kp.period = period;
    kp.out_rows = out_rows;
    kp.dst = reinterpret_cast<char*>(dst);
    kp.pitch = pitch;
    kp.shadow_off = 1e-3f;
    kp.rgb = format;  // RT_FORMAT_*: 0 RGBA32F, 1 RGB32F, 2 RGBA32F at the image row
    kp.heavy_k = 0;
    kp.heavy_parts = 1;
    kp.lane_k = 0;
    kp.lane_k_mode = 0;
    kp.cost_time = 0;
    return RT_OK;
}

bool accel_usable(const rt_ctx* c, const KParams& kp) {
    const float cmag = std::max({std::fabs(kp.cam_pos.x), std::fabs(kp.cam_pos.y), std::fabs(kp.cam_pos.z)});
    return c->accel_ok && kp.useBVH && (kp.useMT != 0) == c->accel.mt && cmag <= c->accel.origin_lim;
}

int launch(rt_ctx* c, const KParams& kp, bool stats);

// A sub-context on this context's stream (brute / mtc), created on first use.
rt_ctx* sub_ctx(rt_ctx* c, rt_ctx*& sub, bool& stale) {
    if (!sub) {
        if (rtx::create_ctx(&sub, c->device, c->stream) != RT_OK) return nullptr;
        stale = true;
    }
    return sub;
}

// The frame constants and walk settings of `c`, for a sub-context rendering its frame.
void inherit(rt_ctx* b, const rt_ctx* c) {
    b->cam = c->cam;
    b->light = c->light;
    b->have_cam = b->have_light = true;
    b->params = c->params;
    b->kernel = RT_KERNEL_ACCEL;
    b->waves_per_block = c->waves_per_block;
    b->persistent = c->persistent;
    b->lane_from_depth = c->lane_from_depth;
    b->cone_cull = c->cone_cull;
    b->spec_mode = c->spec_mode;
    b->split_max = c->split_max;
    b->split_g = c->split_g;
    b->heavy_k = c->heavy_k;
    b->heavy_parts = c->heavy_parts;
    b->lane_k = c->lane_k;
    b->lane_k_mode = c->lane_k_mode;
    b->cost_time = c->cost_time;
    b->latency_mode = c->latency_mode;
    b->schedule = c->schedule;
    b->sched_period = c->sched_period;
    b->cost_dilate = c->cost_dilate;
    b->moving_period = c->moving_period;
    b->moving_dilate = c->moving_dilate;
    b->moving_split = c->moving_split;
    b->order_mode = c->order_mode;
    b->frame_event = c->frame_event;
    b->refit_mode = c->refit_mode;
    b->tail_from = c->tail_from;
    b->tail_max_lanes = c->tail_max_lanes;
    b->shadow_walk_override = c->shadow_walk_override;
    b->tree_mode = c->tree_mode;
    b->scene_stack = c->scene_stack;
    b->lane_stack_override = c->lane_stack_override;
}

// The walk policy in force (rt_set_walk, or auto): barycentric frames walk camera
// rays and their shadows as packets and reflections per lane (1, measured fastest on
// configs 2, 3 and 5). Moller-Trumbore frames over a shallow reference tree with
// big leaves (the car's 3 nodes, whose local BVHs carry the grazing cones) walk every
// bounce as packets, since the cones force entries that neighbouring rays share: car
// MT frame 8.99 ms at 1, 7.73 at 2, 7.00 at 3 (= all packets at depth 3), 12.2 per
// lane for every bounce. Over a deep tree of small leaves (config 5: 6.86 ms at 1,
// 11.39 all packets) they keep 1; the monkey is equal either way
// (profiles/r02zz5_abf_mt_walk*.jsonl).
int walk_from(const rt_ctx* c) {
    if (c->lane_from_depth >= 0) return c->lane_from_depth;
    return c->accel.mt && c->N < kMtPacketMaxNodes ? kMtWalkFrom : 1;
}

bool sub_usable(const rt_ctx* b, const KParams& kp) {
    const float cmag = std::max({std::fabs(kp.cam_pos.x), std::fabs(kp.cam_pos.y), std::fabs(kp.cam_pos.z)});
    return b->accel_ok && cmag <= b->accel.origin_lim;
}

// The brute branch through `brute` (rt_ctx::brute): the same shapes under one
// leaf listing 0..S-1 with an infinite box, built on first use after the
// shapes change. nullptr: render the branch literally (k_packet).
rt_ctx* brute_ctx(rt_ctx* c, const KParams& kp) {
    if (!c->brute_accel || kp.useBVH || c->S <= 0 ||
        (c->kernel != RT_KERNEL_AUTO && c->kernel != RT_KERNEL_ACCEL))
        return nullptr;
    rt_ctx* b = sub_ctx(c, c->brute, c->brute_stale);
    if (!b) return nullptr;
    if (c->brute_stale) {
        FlatNode leaf;
        std::memset(&leaf, 0, sizeof leaf);
        const float inf = std::numeric_limits<float>::infinity();
        leaf.boundsMin = rt_vec3{-inf, -inf, -inf};
        leaf.boundsMax = rt_vec3{inf, inf, inf};
        leaf.leftChild = leaf.rightChild = -1;
        leaf.startShapeIdx = 0;
        leaf.numShapes = c->S;
        std::vector<int> order(c->S);
        for (int i = 0; i < c->S; ++i) order[i] = i;
        if (rt_upload_scene(b, c->host_shapes.data(), c->S, &leaf, 1, order.data(), c->S) != RT_OK) return nullptr;
        c->brute_stale = false;
    }
    inherit(b, c);
    b->params.useBVH = 1;
    return b;  // its own MT forwarding (mt_ctx) applies on the next hop
}

// Moller-Trumbore frames through `mtc` (rt_ctx::mtc): the same shapes and tree,
// the accelerator built for the MT test.
rt_ctx* mt_ctx(rt_ctx* c, const KParams& kp) {
    if (!kp.useBVH || !kp.useMT || c->build_mt || c->S <= 0 || c->N <= 0 ||
        (c->kernel != RT_KERNEL_AUTO && c->kernel != RT_KERNEL_ACCEL))
        return nullptr;
    rt_ctx* b = sub_ctx(c, c->mtc, c->mtc_stale);
    if (!b) return nullptr;
    if (c->mtc_stale) {
        b->build_mt = true;
        if (sync_host_nodes(c) != RT_OK ||
            rt_upload_scene(b, c->host_shapes.data(), c->S, c->host_nodes.data(), c->N, c->host_idx.data(),
                            c->I) != RT_OK ||
            (!c->anim_ids.empty() &&  // rt_animate frames forward to it from now on
             rt_set_animated(b, c->anim_ids.data(), static_cast<int>(c->anim_ids.size())) != RT_OK))
            return nullptr;
        c->mtc_stale = false;
    }
    inherit(b, c);
    return b;
}

// rt_dispatch_rows' render: through `brute` (useBVH = 0) and / or `mtc`
// (Moller-Trumbore) when they apply and their accelerator can take the frame,
// timed by this context's events (rt_kernel_times) like any other dispatch.
unsigned long long refit_launches(const rt_ctx* c, int depth = 0) {
    if (!c) return 0;
    unsigned long long n = c->refit_launches;
    if (depth < 2) n += refit_launches(c->brute, depth + 1) + refit_launches(c->mtc, depth + 1);
    return n;
}

int render_frame(rt_ctx* c, const KParams& kp, rt_ctx** from);

// rt_dispatch_rows' render (render_frame), remembering for rt_sync_frame which context's
// launch drew it and the refit launches so far
int render(rt_ctx* c, const KParams& kp) {
    rt_ctx* from = nullptr;
    const int rc = render_frame(c, kp, &from);
    c->frame_from = rc == RT_OK ? from : nullptr;
    c->frame_refits = refit_launches(c);
    return rc;
}

int render_frame(rt_ctx* c, const KParams& kp, rt_ctx** from) {
    // this context's own pending writes first, also when a sub-context renders the frame
    if (const int rc = flush_updates(c)) return rc;
    rt_ctx* t = c;
    KParams kt = kp;
    for (int hop = 0; hop < 2; ++hop) {
        float off = kt.shadow_off;
        rt_ctx* nxt = brute_ctx(t, kt);
        if (nxt) off = 1e-5f;  // gpu_shader.comp:565
        else nxt = mt_ctx(t, kt);
        if (!nxt) break;
        KParams kn;
        const int rc = fill_kparams(nxt, kt.width, kt.height, kt.y0, kt.stripe, kt.period, kt.out_rows,
                                    reinterpret_cast<float*>(kt.dst), kt.pitch, kn,
                                    kt.rgb);
        if (rc != RT_OK) return rc;
        kn.shadow_off = off;
        t = nxt;
        kt = kn;
    }
    if (t == c || !accel_usable(t, kt)) {
        *from = c;
        return launch(c, kp, false);
    }
    *from = t;
    t->timing = false;  // the sub-context's own events would not be read: this context's time it
    if (!c->timing) {
        const int rc = launch(t, kt, false);
        c->last_kind = t->last_kind;
        c->timed = false;  // no events recorded for this dispatch
        return rc;
    }
    hipEvent_t e0 = c->ev0, e1 = c->ev1;
    if (c->ring_used < static_cast<int>(c->ring0.size())) {
        e0 = c->ring0[c->ring_used];
        e1 = c->ring1[c->ring_used];
    }
    HIP_TRY(hipEventRecord(e0, c->stream));
    const int rc = launch(t, kt, false);
    if (rc != RT_OK) return rc;
    HIP_TRY(hipEventRecord(e1, c->stream));
    c->last0 = e0;
    c->last1 = e1;
    if (c->ring_used < static_cast<int>(c->ring0.size())) ++c->ring_used;
    c->timed = true;
    c->last_kind = t->last_kind;
    t->ring_used = 0;  // its own records are not read
    return RT_OK;
}

int launch(rt_ctx* c, const KParams& kp, bool stats) {
    c->frame_ev_set = false;
    if (const int rc = flush_updates(c)) return rc;  // rt_update_shapes / rt_update_nodes since the last dispatch
    if (kp.out_rows == 0) return RT_OK;
    dim3 grid((kp.width + kTileW - 1) / kTileW, (kp.out_rows + kTileH - 1) / kTileH);
    if (grid.y > 65535u) return RT_ERR_INVALID;
    int kind = c->kernel;
    const bool usable = accel_usable(c, kp);
    if (kind == RT_KERNEL_AUTO) kind = usable ? RT_KERNEL_ACCEL : RT_KERNEL_PACKET;
    if (kind == RT_KERNEL_ACCEL && !usable) kind = RT_KERNEL_PACKET;  // same image either way
    const size_t lds = static_cast<size_t>(kp.max_stack) * kBlock * sizeof(int);
    const bool rec = !stats && c->timing;  // rt_set_kernel_timing
    hipEvent_t e0 = c->ev0, e1 = c->ev1;
    if (rec && c->ring_used < static_cast<int>(c->ring0.size())) {
        e0 = c->ring0[c->ring_used];
        e1 = c->ring1[c->ring_used];
    }
    if (rec) HIP_TRY(hipEventRecord(e0, c->stream));
    bool order_after = false;  // e1 already recorded between the render and the order kernel
    if (stats) {
        hipLaunchKernelGGL(k_lane<true>, grid, dim3(kBlock), lds, c->stream, c->geo_leaf, c->geo_lin, c->mat,
                           c->nodes, kp);
    } else if (kind == RT_KERNEL_LANE) {
        hipLaunchKernelGGL(k_lane<false>, grid, dim3(kBlock), lds, c->stream, c->geo_leaf, c->geo_lin, c->mat,
                           c->nodes, kp);
    } else if (kind == RT_KERNEL_ACCEL) {
        HIP_TRY(join_order(c));  // the previous cost frame's order, if it ran on the order stream
        KParams k2 = kp;
        k2.tiles_x = (kp.width + 7) / 8;
        k2.tiles = k2.tiles_x * ((kp.out_rows + 7) / 8);
        // rt_set_latency_mode applies to frames of at most kLatencyMaxSlots tiles per wave
        // slot: a bigger frame keeps the chip busy on its own, and the split-walk instance's
        // throughput cost then outweighs the shorter chains (waited frame, latency mode on
        // against off: car 1080p 0.216 against 0.262 ms; car 3840x2160 0.706 against 0.626;
        // config 5 3.364 against 3.332; profiles/r04zz2_latency_sweep_*.json)
        const bool latency = c->latency_mode && k2.tiles <= kLatencyMaxSlots * c->cu_count * 16;
        // a moved camera's cost order (moving_period): waited frames only -- with frames in
        // flight a cost frame after every move cost the car's orbit 0.194 -> 0.238 ms per
        // frame (r05j), and the order matters less there
        c->moving = latency && c->have_sched_cam && std::memcmp(&c->sched_cam, &c->cam, sizeof c->cam) != 0 &&
                    c->moving_period > 0;
        c->sched_cam = c->cam;
        c->have_sched_cam = true;
        const int period = c->moving ? c->moving_period : c->sched_period;
        const int dilate = c->moving ? c->moving_dilate : c->cost_dilate;
        k2.tile_counter = c->tile_counter;
        k2.tile_times = c->tile_times;
        if (c->tile_times)
            HIP_TRY(hipMemsetAsync(c->tile_times, 0, kTileRec * c->tile_times_cap * sizeof(unsigned long long),
                                   c->stream));
        const int wpb = c->waves_per_block;
        int blocks = (k2.tiles + wpb - 1) / wpb;
        if (c->persistent) {
            HIP_TRY(hipMemsetAsync(c->tile_counter, 0, 16, c->stream));
            blocks = std::min(blocks, c->cu_count * 20 / wpb);  // resident at 5 waves/SIMD
        }
        const bool spec = c->spec_mode != 0;  // speculative while-while (lane_walk)
        auto kfn = spec ? (c->persistent ? (c->tile_times ? k_accel<true, true, true> : k_accel<true, false, true>)
                                         : (c->tile_times ? k_accel<false, true, true> : k_accel<false, false, true>))
                        : (c->persistent ? (c->tile_times ? k_accel<true, true, false> : k_accel<true, false, false>)
                                         : (c->tile_times ? k_accel<false, true, false> : k_accel<false, false, false>));
        k2.tile_order = nullptr;
        k2.tile_cost = nullptr;
        k2.heavy_k = 0;
        k2.heavy_parts = 1;
        if (c->tile_order && c->tile_order_n == k2.tiles) {
            k2.tile_order = c->tile_order;
        } else if (c->schedule != RT_SCHED_ROWS) {
            if (c->sched_cap < k2.tiles) {
                HIP_TRY(sync_order(c));
                hipFree(c->sched_cost);
                hipFree(c->sched_order);
                hipFree(c->sched_sets);
                c->sched_cost = nullptr;
                c->sched_order = nullptr;
                c->sched_sets = nullptr;
                c->sched_cap = c->sched_valid = 0;
                if (hipMalloc(&c->sched_cost, k2.tiles * sizeof(unsigned)) != hipSuccess ||
                    hipMalloc(&c->sched_order, k2.tiles * sizeof(int)) != hipSuccess ||
                    hipMalloc(&c->sched_sets, 2 * sched_set_words(k2.tiles) * sizeof(unsigned)) != hipSuccess)
                    return RT_ERR_NO_MEMORY;
                HIP_TRY(hipMemsetAsync(c->sched_sets, 0, 2 * sched_set_words(k2.tiles) * sizeof(unsigned), c->stream));
                c->sched_parity = 0;
                c->sched_cap = k2.tiles;
            }
            k2.sched_hist = c->sched_sets + c->sched_parity * sched_set_words(c->sched_cap);
            const bool have = c->sched_valid == k2.tiles;
            if (have) k2.tile_order = c->sched_order;
            if (!have || c->sched_frame % period == 0) {
                k2.tile_cost = c->sched_cost;
                c->sched_frame = 0;
            }
            ++c->sched_frame;
        }
        k2.lane_from_depth = walk_from(c);
        // the root's bounds as kernel arguments while the host copy is current; once
        // rt_animate grew the boxes on the device, from the accelerator's copy of the
        // root record (which the refit keeps current)
        k2.root_ok = 0;
        if (kp.N > 0 && kp.useBVH && c->nodes_on_device_newer) k2.root_ok = 2;
        if (kp.N > 0 && kp.useBVH && !c->nodes_on_device_newer && static_cast<int>(c->host_nodes.size()) == kp.N) {
            const FlatNode& rn = c->host_nodes[kp.N - 1];
            k2.root_ok = 1;
            k2.root_lo[0] = rn.boundsMin.x;
            k2.root_lo[1] = rn.boundsMin.y;
            k2.root_lo[2] = rn.boundsMin.z;
            k2.root_hi[0] = rn.boundsMax.x;
            k2.root_hi[1] = rn.boundsMax.y;
            k2.root_hi[2] = rn.boundsMax.z;
        }
        // big scenes (the RT_TAIL_AUTO criterion): camera rays' shadow walks per lane too
        // (measured on config 5: -3.7 %; on the car the packet walk is faster)
        const bool big = c->accel.st.item_ref.size() >= kTailAutoItems;
        k2.shadow_lane_from = c->shadow_walk_override >= 0 ? c->shadow_walk_override
                              : (big && k2.lane_from_depth <= 1 ? 0 : k2.lane_from_depth);
        k2.lane_stack = c->lane_stack_override > 0 ? c->lane_stack_override : c->accel.max_stack;
        if (k2.tile_order && k2.tile_order == c->sched_order) {
            // the first lane_k dispatch slots (the heaviest tiles): explicit (rt_debug_lane_k)
            // or auto -- in frames that walk per lane anyway (LDS stacks allocated), the
            // heaviest 1/128 of the tiles walk their camera rays' shadows per lane: shorter
            // chains on the slowest tiles (car: serial -5.5 %, 2 in flight equal, r02q)
            int lk = c->lane_k, lm = c->lane_k_mode;
            if (lk < 0) {
                const bool lanes = std::min(k2.lane_from_depth, k2.shadow_lane_from) < k2.maxBounces;
                lk = lanes ? std::max(64, k2.tiles / 128) : 0;
                lm = 2;
            }
            if (lk > 0 && lm > 0) {
                k2.lane_k = lk;
                k2.lane_k_mode = lm;
            }
        }
        // LDS stacks for the per-lane walks (also those of the lane_k slots)
        const size_t lds = std::min(k2.lane_from_depth, k2.shadow_lane_from) < k2.maxBounces || k2.lane_k > 0
                               ? static_cast<size_t>(k2.lane_stack) * 64 * wpb * 6
                               : 0;
        if (k2.tile_order && k2.tile_order == c->sched_order) {
            // heavy tiles: explicit (rt_debug_heavy) or auto. A frame of at most
            // kHeavyAutoSlots waves per wave slot whose walks are all packets (config 2:
            // 800x600, primary + shadow) is bound by its slowest tiles even with frames
            // in flight, and a packet walks the union of its rays' nodes: the heaviest
            // 1/256 of its tiles run as 8 waves of 8 rays (measured -20 %, r02n). Where
            // per-lane walks dominate the slow tiles (the car's reflections) it loses.
            int hk = c->heavy_k, hp = c->heavy_parts;
            if (hk < 0) {
                const bool small = k2.tiles <= kHeavyAutoSlots * c->cu_count * 16 &&
                                   std::min(k2.lane_from_depth, k2.shadow_lane_from) >= k2.maxBounces;
                hk = small ? std::max(16, k2.tiles / 256) : 0;
                hp = small ? 8 : 1;
                if (small && latency) {
                    // Waited, such a frame ends on its heaviest packet chains: split into 32
                    // waves of 2 rays, a tile's parts walk little more than their own rays'
                    // nodes. Config 2 waited (Python loop, tools/latency_sweep.py, r06k-r06m):
                    // 29 x 8 (the in-flight rule) 0.0957 ms, 40 x 16 0.0907, 40 x 32 0.0793,
                    // 60 / 120 x 32 0.0798, 20 x 32 0.0819, 40 x 64 0.0855. In flight the
                    // in-flight rule stays best (4 frames: 0.0314 against 0.0416 with 40 x 32).
                    hk = std::max(16, k2.tiles / 128);
                    hp = 32;
                }
                if (!small && latency) {
                    // rt_set_latency_mode: the heaviest 1/200 as 4 waves. Car waited frame with the
                    // wall-time cost order and whole-tile cost frames (Python loop,
                    // profiles/r04z7_latency_sweep.json, r04z8_latency_sweep.json), heaviest k as
                    // 4 waves: k = 95 0.2362 ms, 126 0.2161, 159 0.2184, 191 0.2203, 255 0.2260;
                    // as 2 waves: 63 0.2371, 127-511 0.224, 1023 0.229; 126 as 8: 0.2275. Some
                    // tiles ranked ~96-126 by whole time gain most from the split, so k sits
                    // well above that edge (162 of the car's 32,400 tiles).
                    // A frame of few tiles per CU (a rank's stripe share of a strong frame) has
                    // idle CUs to spread its heaviest chains over: the car's 1/8 share (4,080
                    // tiles, 16 per CU) waited 0.175 ms by the whole-frame rule, 0.135-0.144 with
                    // its heaviest 1/25 as 16 waves; the 1/4 share (8,160) 0.175-0.192 against
                    // 0.156-0.160 with 1/25-1/50 as 8 waves; the 1/2 share mixed (C++ host loop,
                    // tools/share_sweep.py, profiles/r05s/r05t_share_sweep*.json)
                    // Off the tuned view the 4-wave split lost: four still cameras along
                    // bench.py's orbit waited 0.213 / 0.279 / 0.277 / 0.294 ms with it, 0.216 /
                    // 0.268 / 0.268 / 0.284 as 2 waves (geometric mean over the views 1.034
                    // against 1.011 of each view's best of a 4 x 3 grid; tools/view_sweep.py,
                    // profiles/r05za_view_sweep.json): whole frames that walk rays per lane take
                    // 2 waves. All-packet frames (the MT car) keep 4: 2.68 ms with 2 against 1.75
                    // (r05zl); the heaviest 1/400 as 8, best over two orbit views (geometric mean
                    // 1.782 against 1.864 ms, r05zn_view_sweep_mt.json), measured 1.770 against
                    // 1.755 at the bench's view and 1.933 against 1.844 animated (r05zo): kept 4
                    const int per_cu = k2.tiles / std::max(1, c->cu_count);
                    const bool lanes = std::min(k2.lane_from_depth, k2.shadow_lane_from) < k2.maxBounces;
                    hk = std::max(16, k2.tiles / (per_cu <= 40 ? 25 : 200));
                    hp = per_cu <= 20 ? 16 : per_cu <= 40 ? 8 : lanes ? 2 : 4;
                }
            }
            const bool stamps_fit =  // timed frames split only with a record per part
                !c->tile_times ||
                c->tile_times_cap >= static_cast<size_t>(k2.tiles) + static_cast<size_t>(std::min(hk, k2.tiles)) * hp;
            // In latency mode a dispatch that records wall-time costs runs every tile whole:
            // a split tile's parts run side by side, so no sum or maximum of theirs stands for
            // the whole tile's time, and a split set ranked by such an estimate locks in
            // whatever tiles were split first (the car's waited frame settled at 0.222 or
            // 0.237 ms by the split set it started from, r04z5). Recording whole tiles every
            // 16th frame keeps the split set the longest whole tiles. The all-packet frames'
            // own split (8 waves, above) stays on their cost frames: whole, those took 1.5x
            // (config 2, the MT car; r04zz profiles), and in flight the ranking matters less.
            const bool whole = k2.tile_cost && c->cost_time != 0 && !c->tile_times && latency &&
                               !(c->moving && c->moving_split);
            if (!c->persistent && stamps_fit && hp > 1 && hk > 0 && !whole) {
                k2.heavy_k = std::min(hk, k2.tiles);
                k2.heavy_parts = hp;
            }
        }
        // the cost measure: explicit (rt_debug_cost_time) or the waves' wall time
        k2.cost_time = c->cost_time != 0 ? 1 : 0;
        k2.heavy_acc = nullptr;
        if (k2.tile_cost && k2.heavy_k > 0) {  // the split tiles' part sums and counts (kernel comment)
            const size_t need = static_cast<size_t>(k2.heavy_k);
            if (c->heavy_acc_cap < need) {
                hipFree(c->heavy_acc);
                c->heavy_acc = nullptr;
                c->heavy_acc_cap = 0;
                if (hipMalloc(&c->heavy_acc, need * sizeof(unsigned long long)) != hipSuccess) return RT_ERR_NO_MEMORY;
                c->heavy_acc_cap = need;
            }
            HIP_TRY(hipMemsetAsync(c->heavy_acc, 0, need * sizeof(unsigned long long), c->stream));
            k2.heavy_acc = c->heavy_acc;
        }
        // Animated scenes keep the scene tree: rt_animate refits its boxes and items (prepare_animation).
        // (off while a rebuild for node boxes that stopped nesting runs: st_suspended)
        const int troot = c->tree_mode == RT_TREE_SCENE && !c->st_suspended ? c->st_root : kNoChild;
        // production shape on a dispatch that records no tile work: the counter-free kernel

        const AccelPtrs A{c->anodes, c->prims, c->lnodes, c->wnodes, c->tleaf, c->titems, troot,
                          c->scene_stack > 0 ? c->scene_stack : kMaxStack, c->nfew, kp.N, c->accel.origin_lim,
                          c->boxes_finite, c->split_max, c->split_g, c->prim_idx_dev,
                          {c->accel.mt_z[0], c->accel.mt_z[1], c->accel.mt_z[2]}};
        // compaction: bounces >= tail_from of the rays still alive run in k_accel_tail
        k2.tail_queue = nullptr;
        // RT_TAIL_AUTO: from bounce 2 on scenes of many scene-tree items (measured: config 5's
        // incoherent bounces -5 %; on the car's 1,302 items the extra kernel costs +18 %)
        const int tail_from = c->tail_from != RT_TAIL_AUTO
                                  ? c->tail_from
                                  : (c->accel.st.item_ref.size() >= kTailAutoItems ? 2 : 0);
        // the queue's pixel word is row * width + x in 32 bits (rt_device.h): larger
        // frames render without compaction
        const bool tail = tail_from > 0 && tail_from < k2.maxBounces && !c->persistent &&
                          static_cast<unsigned long long>(k2.width) * k2.out_rows < (1ull << 32);
        const int rx = (k2.tiles_x + 7) / 8, regions = rx * ((k2.tiles / k2.tiles_x + 7) / 8);
        if (tail) {
            const size_t need = static_cast<size_t>(regions) * kTailRegion;
            if (need > c->tail_cap) {
                hipFree(c->tail_queue);
                c->tail_queue = nullptr;
                c->tail_cap = 0;
                // 3 float4 records, then the pixel words (rt_device.h, tail_queue)
                if (hipMalloc(&c->tail_queue, need * (3 * sizeof(float4) + sizeof(int))) != hipSuccess)
                    return RT_ERR_NO_MEMORY;
                c->tail_cap = need;
            }
            if (regions > c->tail_regions_cap) {
                hipFree(c->tail_counts);
                c->tail_counts = nullptr;
                c->tail_regions_cap = 0;
                if (hipMalloc(&c->tail_counts, 2 * static_cast<size_t>(regions) * sizeof(int)) != hipSuccess)
                    return RT_ERR_NO_MEMORY;
                HIP_TRY(hipMemsetAsync(c->tail_counts, 0, 2 * static_cast<size_t>(regions) * sizeof(int), c->stream));
                c->tail_regions_cap = regions;
            }
            k2.tail_queue = c->tail_queue;
            k2.tail_px = reinterpret_cast<int*>(c->tail_queue + 3 * c->tail_cap);
            k2.tail_count = c->tail_counts + c->tail_parity * c->tail_regions_cap;
            k2.tail_count_next = c->tail_counts + (1 - c->tail_parity) * c->tail_regions_cap;
            k2.tail_from = tail_from;
            k2.tail_rx = rx;
            k2.tail_regions = regions;
            k2.tail_counters = c->tail_regions_cap;
            k2.tail_max_lanes = c->tail_max_lanes;
        }
        if (c->accel.mt) {
            // Moller-Trumbore accelerator: its own instances; no compaction
            k2.tail_queue = nullptr;
            // a dispatch recording wall-time costs: the counter-free instance that records
            kfn = spec ? (!k2.tile_cost   ? k_accel<false, false, true, false, false, true>
                          : k2.cost_time ? k_accel<false, false, true, false, false, true, true>
                                         : k_accel<false, false, true, true, false, true>)
                       : (!k2.tile_cost   ? k_accel<false, false, false, false, false, true>
                          : k2.cost_time ? k_accel<false, false, false, false, false, true, true>
                                         : k_accel<false, false, false, true, false, true>);
            blocks = (k2.tiles + wpb - 1) / wpb;
        } else if (kfn == k_accel<false, false, true>) {
            // production shape: the counter-free kernel on a dispatch that records no tile
            // work; the queueing kernel when the tail runs (other shapes: no compaction)
            if (tail || latency) {
                // the compacting instance; in latency mode without a queue (tail_from 0), for
                // its split walks in sparse waves (lane_walk_any), which the production
                // instance leaves out for its registers
                // (latency mode without compaction: the instance without the queue's code)
                if (tail)
                    kfn = !k2.tile_cost  ? k_accel<false, false, true, false, true>
                          : k2.cost_time ? k_accel<false, false, true, false, true, false, true>
                                         : k_accel<false, false, true, true, true>;
                else
                    kfn = !k2.tile_cost  ? k_accel<false, false, true, false, true, false, false, false>
                          : k2.cost_time ? k_accel<false, false, true, false, true, false, true, false>
                                         : k_accel<false, false, true, true, true, false, true, false>;
            } else if (!k2.tile_cost) {
                kfn = k_accel<false, false, true, false>;
            } else if (k2.cost_time) {
                kfn = k_accel<false, false, true, false, false, false, true>;  // records, no counters
            }
        } else if (tail) {
            k2.tail_queue = nullptr;
        }
        const bool tail_on = k2.tail_queue != nullptr;
        if (!c->persistent)  // every dispatch slot: the split heavy tiles' extra waves too
            blocks = (k2.tiles + k2.heavy_k * (k2.heavy_parts - 1) + wpb - 1) / wpb;
        hipLaunchKernelGGL(kfn, dim3(blocks), dim3(64 * wpb), lds, c->stream, A, c->mat, k2);
        if (tail_on) {
            const size_t tlds = static_cast<size_t>(k2.lane_stack) * 64 * 6;
            const int tgrid = kTailOneShot ? regions * (kTailRegion / 64) : c->cu_count * 16;
            hipLaunchKernelGGL(spec ? k_accel_tail<true> : k_accel_tail<false>, dim3(tgrid), dim3(64), tlds,
                               c->stream, A, c->mat, k2);
            c->tail_parity = 1 - c->tail_parity;
        }
        if (k2.tile_cost) {
            // the next frame's order; stream-ordered after this dispatch (and after its
            // end event, so rt_kernel_times is the render kernel alone), before the next
            if (rec) HIP_TRY(hipEventRecord(e1, c->stream));
            order_after = true;
            const unsigned* set = c->sched_sets + c->sched_parity * sched_set_words(c->sched_cap);
            unsigned* next = c->sched_sets + (1 - c->sched_parity) * sched_set_words(c->sched_cap);
            const int groups = (k2.tiles + kOrderThreads - 1) / kOrderThreads;
            const unsigned* cost = c->sched_cost;
            // the order stream (rt_debug_order_stream): behind the render's end, off the frame's end
            const bool side = c->order_mode == 2 || (c->order_mode == 1 && latency);
            hipStream_t os = c->stream;
            if (!side && latency && c->frame_event) {
                // a waited frame ends here (rt_sync_frame); the order runs behind it on the same
                // stream, within the host's turnaround to the next dispatch
                if (!c->frame_ev && hipEventCreateWithFlags(&c->frame_ev, hipEventDisableTiming) != hipSuccess)
                    return RT_ERR_DEVICE;
                HIP_TRY(hipEventRecord(c->frame_ev, c->stream));
                c->frame_ev_set = true;
            }
            if (side) {
                if (!c->order_stream) {
                    if (rtx::make_stream(&c->order_stream, false) != hipSuccess ||
                        hipEventCreateWithFlags(&c->order_ready, hipEventDisableTiming) != hipSuccess ||
                        hipEventCreateWithFlags(&c->order_done, hipEventDisableTiming) != hipSuccess)
                        return RT_ERR_DEVICE;
                }
                HIP_TRY(hipEventRecord(c->order_ready, c->stream));
                HIP_TRY(hipStreamWaitEvent(c->order_stream, c->order_ready, 0));
                os = c->order_stream;
            }
            if (dilate > 0) {
                const size_t need = static_cast<size_t>(k2.tiles) + static_cast<size_t>(groups) * kOrderBuckets;
                if (c->dil_cap < need) {
                    HIP_TRY(sync_order(c));
                    hipFree(c->dil_cost);
                    c->dil_cost = nullptr;
                    c->dil_cap = 0;
                    if (hipMalloc(&c->dil_cost, need * sizeof(unsigned)) != hipSuccess) return RT_ERR_NO_MEMORY;
                    c->dil_cap = need;
                }
                hipLaunchKernelGGL(k_cost_dilate, dim3(groups), dim3(kOrderThreads), 0, os, c->sched_cost,
                                   k2.tiles, k2.tiles_x, dilate, c->dil_cost, c->dil_cost + k2.tiles);
                cost = c->dil_cost;
                set = c->dil_cost + k2.tiles;
            }
            hipLaunchKernelGGL(k_tile_order, dim3(groups), dim3(kOrderThreads),
                               0, os, cost, k2.tiles, set, next,
                               static_cast<int>(sched_set_words(c->sched_cap)), c->sched_order,
                               c->schedule == RT_SCHED_COST_XCD ? 1 : 0);
            if (side) {
                HIP_TRY(hipEventRecord(c->order_done, os));
                c->order_pending = true;
            }
            c->sched_parity = 1 - c->sched_parity;
            c->sched_valid = k2.tiles;
        }
    } else {
        hipLaunchKernelGGL(k_packet, grid, dim3(kBlock), 0, c->stream, c->geo_leaf, c->geo_lin, c->mat, c->nodes,
                           kp);
    }
    c->last_kind = stats ? RT_KERNEL_LANE : kind;
    HIP_TRY(hipGetLastError());
    if (rec) {
        if (!order_after) HIP_TRY(hipEventRecord(e1, c->stream));
        c->last0 = e0;
        c->last1 = e1;
        if (c->ring_used < static_cast<int>(c->ring0.size())) ++c->ring_used;
        c->timed = true;
    } else if (!stats) {
        c->timed = false;  // rt_set_kernel_timing(0): rt_last_kernel_ms has no dispatch to report
    }
    return RT_OK;
}

}  // namespace

extern "C" {

const char* rt_status_string(int s) {
    switch (s) {
        case RT_OK: return "ok";
        case RT_ERR_INVALID: return "invalid argument";
        case RT_ERR_DEVICE: return "HIP runtime error";
        case RT_ERR_NO_MEMORY: return "device allocation failed";
        case RT_ERR_NO_SCENE: return "scene, camera or light not uploaded";
        case RT_ERR_BVH: return "node/index arrays out of range or deeper than the 64-entry stack";
        case RT_ERR_NO_DEVICE: return "no such HIP device";
        case RT_ERR_COMM: return "RCCL call failed (the group's communicator is aborted)";
        case RT_ERR_TIMEOUT: return "timed out waiting for a group's frames (the communicator is aborted)";
        default: return "unknown status";
    }
}

int rt_create(rt_ctx** out, int device) { return rtx::create_ctx(out, device, nullptr); }

}  // extern "C"

hipError_t rtx::make_stream(hipStream_t* s, bool own_queue) {
    if (own_queue) {
        int dev = 0;
        hipDeviceProp_t prop;
        if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess &&
            prop.multiProcessorCount > 0) {
            std::vector<uint32_t> mask((prop.multiProcessorCount + 31) / 32, 0xffffffffu);
            if (hipExtStreamCreateWithCUMask(s, static_cast<uint32_t>(mask.size()), mask.data()) == hipSuccess)
                return hipSuccess;
        }
    }
    return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}

namespace {
bool env_cumask() {
    static const bool on = [] {
        const char* e = std::getenv("RT_STREAMS_CUMASK");
        return e && e[0] == '1';
    }();
    return on;
}
}  // namespace

int rtx::create_ctx(rt_ctx** out, int device, hipStream_t stream) {
    if (!out) return RT_ERR_INVALID;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return RT_ERR_NO_DEVICE;
    rt_ctx* c = new (std::nothrow) rt_ctx();
    if (!c) return RT_ERR_NO_MEMORY;
    c->device = device;
    c->stream = stream;
    if (set_dev(c) != RT_OK || (!stream && rtx::make_stream(&c->stream, env_cumask()) != hipSuccess) ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
        hipMalloc(&c->stats_dev, ST_COUNT * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&c->tile_counter, 16) != hipSuccess) {
        rt_destroy(c);
        return RT_ERR_DEVICE;
    }
    c->own_stream = !stream;
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) == hipSuccess)
            c->cu_count = prop.multiProcessorCount;
        if (c->cu_count <= 0) c->cu_count = 256;
    }
    c->ring0.resize(kRing, nullptr);
    c->ring1.resize(kRing, nullptr);
    for (int i = 0; i < kRing; ++i)
        if (hipEventCreate(&c->ring0[i]) != hipSuccess || hipEventCreate(&c->ring1[i]) != hipSuccess) {
            rt_destroy(c);
            return RT_ERR_DEVICE;
        }
    *out = c;
    return RT_OK;
}

bool rtx::matches_view(const rt_ctx* c, const FlatCamera& cam, const float lo[3], const float hi[3]) {
    if (!c || !c->have_cam || std::memcmp(&c->cam, &cam, sizeof cam) != 0) return false;
    if (c->N <= 0) return true;
    return std::memcmp(c->root_lo, lo, sizeof c->root_lo) == 0 && std::memcmp(c->root_hi, hi, sizeof c->root_hi) == 0;
}

int rtx::animate_deferred(rt_ctx* c, const FlatShape* shapes) {
    if (!c || !c->have_scene || c->anim_ids.empty() || !shapes) return RT_ERR_INVALID;
    const int n = static_cast<int>(c->anim_ids.size());
    // node records the host wrote before this frame apply first (as rt_animate): a refit
    // never carries both the host's node records and growth (k_refit's roles would both
    // write the grown boxes)
    if (c->nodes_dirty) {
        if (set_dev(c) != RT_OK) return RT_ERR_DEVICE;
        if (const int rc = flush_updates(c)) return rc;
    }
    if (c->grow_box.size() != 6 * static_cast<size_t>(n)) return RT_ERR_INVALID;
    for (int i = 0; i < n; ++i) {
        const int id = c->anim_ids[i];
        c->host_shapes[id] = shapes[i];
        if (id < static_cast<int>(c->shape_moved.size())) c->shape_moved[id] = 1;
        // the growth of this frame, on the host with the device's operations
        // (reference_box: BoundingBox::growToInclude), unioned with the pending frames'
        float lo[3], hi[3];
        reference_box(shapes[i], lo, hi);
        float* b = &c->grow_box[6 * static_cast<size_t>(i)];
        for (int a = 0; a < 3; ++a) {
            b[a] = lo[a] < b[a] ? lo[a] : b[a];
            b[3 + a] = b[3 + a] < hi[a] ? hi[a] : b[3 + a];
        }
        const int e = c->refit_of[id];
        if (e >= 0 && e < static_cast<int>(c->entry_root.size()) && c->entry_root[e])
            for (int a = 0; a < 3; ++a) {
                c->root_lo[a] = lo[a] < c->root_lo[a] ? lo[a] : c->root_lo[a];
                c->root_hi[a] = c->root_hi[a] < hi[a] ? hi[a] : c->root_hi[a];
            }
    }
    c->grow_pending = true;
    // the sub-contexts follow as rt_animate makes them: brute force the records (no nodes),
    // Moller-Trumbore the same deferred frame
    if (c->brute && !c->brute_stale)
        for (int i = 0; i < n && !c->brute_stale; ++i)
            if (rt_update_shapes(c->brute, c->anim_ids[i], 1, &shapes[i]) != RT_OK) c->brute_stale = true;
    if (c->mtc && !c->mtc_stale && rtx::animate_deferred(c->mtc, shapes) != RT_OK) c->mtc_stale = true;
    return RT_OK;
}

bool rtx::view_root(const rt_ctx* c, float lo[3], float hi[3]) {
    if (!c || !c->have_scene || c->N <= 0) return false;
    std::memcpy(lo, c->root_lo, sizeof c->root_lo);
    std::memcpy(hi, c->root_hi, sizeof c->root_hi);
    return true;
}

extern "C" {

int rt_destroy(rt_ctx* c) {
    if (!c) return RT_ERR_INVALID;
    hipSetDevice(c->device);
    if (c->stream) sync_stream(c);
    if (c->brute) rt_destroy(c->brute);  // it runs on this context's stream
    c->brute = nullptr;
    if (c->mtc) rt_destroy(c->mtc);
    c->mtc = nullptr;
    free_scene(c);
    hipFree(c->staging_shapes);
    hipFree(c->staging_nodes);
    hipFree(c->staging_idx);
    hipFree(c->img);
    hipFree(c->stats_dev);
    hipFree(c->tile_counter);
    hipFree(c->tail_queue);
    hipFree(c->tail_counts);
    hipFree(c->tile_times);
    hipFree(c->tile_order);
    hipFree(c->sched_cost);
    hipFree(c->dil_cost);
    hipFree(c->heavy_acc);
    hipFree(c->sched_order);
    hipFree(c->sched_sets);
    hipFree(c->anim_maps);
    hipFree(c->anim_sbox);
    hipFree(c->refit_ctr);
    hipFree(c->refit_dev);
    for (int k = 0; k < rt_ctx::kAnimRing; ++k) {
        if (c->anim_pinned[k]) hipHostFree(c->anim_pinned[k]);
        if (c->anim_copied[k]) hipEventDestroy(c->anim_copied[k]);
    }
    for (hipEvent_t e : c->ring0) if (e) hipEventDestroy(e);
    for (hipEvent_t e : c->ring1) if (e) hipEventDestroy(e);
    if (c->sync_ev) hipEventDestroy(c->sync_ev);
    if (c->frame_ev) hipEventDestroy(c->frame_ev);
    if (c->order_ready) hipEventDestroy(c->order_ready);
    if (c->order_done) hipEventDestroy(c->order_done);
    if (c->order_stream) hipStreamDestroy(c->order_stream);
    if (c->ev0) hipEventDestroy(c->ev0);
    if (c->ev1) hipEventDestroy(c->ev1);
    if (c->own_stream && c->stream) hipStreamDestroy(c->stream);
    delete c;
    return RT_OK;
}

int rt_set_stream(rt_ctx* c, void* s) {
    if (!c) return RT_ERR_INVALID;
    if (set_dev(c) != RT_OK) return RT_ERR_DEVICE;
    if (const int rc = record_mark(c)) return rc;  // on the stream the k_refit ran on
    HIP_TRY(sync_stream(c));
    if (c->own_stream) hipStreamDestroy(c->stream);
    if (s) {
        c->stream = static_cast<hipStream_t>(s);
        c->own_stream = false;
    } else {
        HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        c->own_stream = true;
    }
    for (rt_ctx* sub : {c->brute, c->mtc})  // sub-contexts run on this context's stream (synchronised above)
        if (sub) {
            rt_set_stream(sub, c->stream);
        }
    return RT_OK;
}

int rt_upload_scene(rt_ctx* c, const FlatShape* shapes, int S, const FlatNode* nodes, int N, const int* idx,
                    int I) {
    if (!c || S < 0 || N < 0 || I < 0 || (S > 0 && !shapes) || (N > 0 && !nodes) || (I > 0 && !idx))
        return RT_ERR_INVALID;
    int ms = 0;
    int rc = check_tree(nodes, N, idx, I, S, &ms);
    if (rc != RT_OK) return rc;
    if (set_dev(c) != RT_OK) return RT_ERR_DEVICE;
    PhaseLaps lap("rt_upload_scene");
    HIP_TRY(sync_stream(c));
    free_scene(c);  // (joins a rebuild in flight: it reads the host copies)
    lap("free");
    c->host_nodes.assign(nodes, nodes + N);
    c->host_idx.assign(idx, idx + I);
    c->host_shapes.assign(shapes, shapes + S);
    lap("host copies");
    // The accelerator's host build (from the host copies into c->accel, which nothing
    // else touches meanwhile) runs on its own thread while this one uploads and packs
    // the records: the build does not wait for the device, nor the copies for the build
    // (config 5: 64 -> 53 ms). Small scenes build afterwards on this thread as before (a
    // new thread's allocations start in a fresh heap arena: the car's upload 3.0 -> 3.5 ms).
    constexpr int kOverlapShapes = 32768;
    const bool overlap = N > 0 && S >= kOverlapShapes;
    bool built = false;
    std::thread builder;
    if (overlap)
        builder = std::thread([c, S, N, I, &built] {
            try {  // (bad_alloc: no accelerator, as a failed build; never past the thread)
                built = rta::build_accel(c->host_shapes.data(), S, c->host_nodes.data(), N, c->host_idx.data(), I,
                                         kLeafScan, kMaxStack, c->accel, c->build_mt);
            } catch (...) {
                c->accel = rta::AccelHost();
                built = false;
            }
        });
    const auto records = [&]() -> int {
        const size_t sS = S > 0 ? S : 1, sI = I > 0 ? I : 1, sN = N > 0 ? N : 1;
        if (hipMalloc(&c->geo_lin, sS * 5 * sizeof(float4)) != hipSuccess ||
            hipMalloc(&c->geo_leaf, sI * 5 * sizeof(float4)) != hipSuccess ||
            hipMalloc(&c->mat, sS * 2 * sizeof(float4)) != hipSuccess ||
            hipMalloc(&c->nodes, sN * 2 * sizeof(float4)) != hipSuccess)
            return RT_ERR_NO_MEMORY;
        int r2;
        if ((r2 = ensure_staging(c->staging_shapes, c->staging_shapes_cap, sS)) != RT_OK) return r2;
        if ((r2 = ensure_staging(c->staging_nodes, c->staging_nodes_cap, sN)) != RT_OK) return r2;
        if ((r2 = ensure_staging(c->staging_idx, c->staging_idx_cap, sI)) != RT_OK) return r2;
        if (S > 0) HIP_TRY(hipMemcpyAsync(c->staging_shapes, shapes, S * sizeof(FlatShape), hipMemcpyHostToDevice, c->stream));
        if (N > 0) HIP_TRY(hipMemcpyAsync(c->staging_nodes, nodes, N * sizeof(FlatNode), hipMemcpyHostToDevice, c->stream));
        if (I > 0) HIP_TRY(hipMemcpyAsync(c->staging_idx, idx, I * sizeof(int), hipMemcpyHostToDevice, c->stream));
        if (S + I > 0)
            hipLaunchKernelGGL(k_pack_shapes, dim3((S + I + 255) / 256), dim3(256), 0, c->stream, c->staging_shapes, S,
                               c->staging_idx, I, c->geo_lin, c->geo_leaf, c->mat);
        if (N > 0)
            hipLaunchKernelGGL(k_pack_nodes, dim3((N + 255) / 256), dim3(256), 0, c->stream, c->staging_nodes, N,
                               c->nodes);
        HIP_TRY(hipGetLastError());
        HIP_TRY(sync_stream(c));
        return RT_OK;
    };
    rc = records();
    if (builder.joinable()) builder.join();
    lap("records (build alongside)");
    if (rc != RT_OK) {
        free_scene(c);
        return rc;
    }
    c->S = S;
    c->N = N;
    c->I = I;
    c->max_stack = ms;
    c->have_scene = true;
    c->nodes_on_device_newer = false;
    set_root(c);
    c->anim_ids.clear();  // ids refer to the previous scene
    c->refit_ids.clear();
    c->anim_base.clear();
    c->upd_ids.clear();
    c->upd_base.clear();
    c->upd_mark.assign(S, 0);
    c->nodes_dirty = c->nodes_rebuild = c->bounds_rebuild = false;
    c->brute_stale = c->mtc_stale = true;
    rc = upload_accel(c, overlap ? &built : nullptr);
    lap("accelerator");
    return rc;
}

int rt_update_shapes(rt_ctx* c, int first, int count, const FlatShape* shapes) {
    if (!c || !c->have_scene || first < 0 || count < 0 || first > c->S - count || (count > 0 && !shapes))
        return RT_ERR_INVALID;
    if (count == 0) return RT_OK;
    // glBufferSubData of shape records (updateScene, src/main.cpp:981-992): the host copy
    // now, the device copies at the next operation that reads them (flush_updates), as
    // one refit with whatever else was written by then. The host array may be reused
    // when this returns. Node boxes stay as they are until rt_update_nodes.
    for (int j = 0; j < count; ++j) {
        const int id = first + j;
        if (!c->upd_mark[id]) {
            if (c->refit_of[id] < 0) c->upd_base.emplace_back(id, c->host_shapes[id]);  // the build's record
            c->upd_mark[id] = 1;
            c->upd_ids.push_back(id);
        }
        c->host_shapes[id] = shapes[j];
        if (id < static_cast<int>(c->shape_moved.size())) c->shape_moved[id] = 1;
    }
    // the sub-contexts hold the same shapes in the same order (brute: under its one
    // leaf; mtc: the MT accelerator): they refit too
    if (c->brute && !c->brute_stale && rt_update_shapes(c->brute, first, count, shapes) != RT_OK)
        c->brute_stale = true;
    if (c->mtc && !c->mtc_stale && rt_update_shapes(c->mtc, first, count, shapes) != RT_OK) c->mtc_stale = true;
    return RT_OK;
}

int rt_update_nodes(rt_ctx* c, const FlatNode* nodes, int N) {
    if (!c || !c->have_scene || N != c->N || (N > 0 && !nodes)) return RT_ERR_INVALID;
    if (c->grow_pending) {  // deferred growth (rtx::animate_deferred) applies before these records
        if (set_dev(c) != RT_OK) return RT_ERR_DEVICE;
        if (const int rc = flush_updates(c)) return rc;
    }
    for (int k = 0; k < N; ++k) {
        const FlatNode &a = nodes[k], &b = c->host_nodes[k];
        if (a.leftChild != b.leftChild || a.rightChild != b.rightChild ||
            (a.leftChild == -1 && (a.startShapeIdx != b.startShapeIdx || a.numShapes != b.numShapes)))
            return RT_ERR_BVH;  // topology must not change: use rt_upload_scene
    }
    if (N == 0) return RT_OK;
    // glBufferSubData of the node records (src/main.cpp:340-345): the host copy now,
    // every device copy of the boxes at the next device operation (flush_updates).
    c->host_nodes.assign(nodes, nodes + N);
    c->nodes_on_device_newer = false;  // these boxes replace any the device grew
    set_root(c);
    c->nodes_dirty = true;
    c->boxes_finite = 1;
    for (int k = 0; k < N; ++k)
        for (float v : {nodes[k].boundsMin.x, nodes[k].boundsMin.y, nodes[k].boundsMin.z, nodes[k].boundsMax.x,
                        nodes[k].boundsMax.y, nodes[k].boundsMax.z})
            if (std::isnan(v)) c->boxes_finite = 0;
    // the scene tree holds only while the boxes nest (accel.h SceneTree)
    // (recomputed per call: a later write that restores nesting before the flush
    // cancels the rebuild an earlier one asked for)
    c->nodes_rebuild = c->accel_ok && c->accel.st.wroot >= 0 && !host_nodes_nest(c);
    if (c->mtc && !c->mtc_stale && rt_update_nodes(c->mtc, nodes, N) != RT_OK) c->mtc_stale = true;
    return RT_OK;
}

int rt_set_animated(rt_ctx* c, const int* ids, int count) {
    if (!c || !c->have_scene || count < 0 || (count > 0 && !ids)) return RT_ERR_INVALID;
    std::vector<char> seen(c->S, 0);
    for (int i = 0; i < count; ++i) {
        if (ids[i] < 0 || ids[i] >= c->S || seen[ids[i]]) return RT_ERR_INVALID;
        seen[ids[i]] = 1;
    }
    if (set_dev(c) != RT_OK) return RT_ERR_DEVICE;
    if (c->grow_pending) {  // deferred frames of the old set first (rtx::animate_deferred)
        const int rc = flush_updates(c);
        if (rc != RT_OK) return rc;
    }
    c->anim_ids.assign(ids, ids + count);
    c->grow_box.assign(6 * static_cast<size_t>(count), 0.f);
    for (int i = 0; i < count; ++i)
        for (int a = 0; a < 3; ++a) {
            c->grow_box[6 * i + a] = INFINITY;
            c->grow_box[6 * i + 3 + a] = -INFINITY;
        }
    // The refit set takes the new ids with the records the accelerator was built from
    // (a shape rewritten since: its record before the first rewrite); shapes already in
    // it keep their base, and shapes that stop being animated stay in it.
    bool added = false;
    for (int i = 0; i < count; ++i) {
        const int id = ids[i];
        if (c->refit_of[id] >= 0) continue;
        FlatShape base = c->host_shapes[id];
        if (c->upd_mark[id])
            for (const auto& ub : c->upd_base)
                if (ub.first == id) base = ub.second;
        c->refit_of[id] = static_cast<int>(c->refit_ids.size());
        c->refit_ids.push_back(id);
        c->anim_base.push_back(base);
        added = true;
    }
    if (c->mtc && !c->mtc_stale && rt_set_animated(c->mtc, ids, count) != RT_OK) c->mtc_stale = true;
    return added ? prepare_animation(c) : RT_OK;
}

int rt_animate(rt_ctx* c, const FlatShape* shapes) {
    if (!c || !c->have_scene || c->anim_ids.empty() || !shapes) return RT_ERR_INVALID;
    PhaseLaps lap(c->rebuild && c->rebuild->done.load() ? "rt_animate (swap)" : nullptr);
    if (set_dev(c) != RT_OK) return RT_ERR_DEVICE;
    int rc = RT_OK;
    if (c->grow_pending) {  // deferred frames pending (rtx::animate_deferred): this one joins them
        if ((rc = rtx::animate_deferred(c, shapes)) != RT_OK) return rc;
        return flush_updates(c);
    }
    // node records the host wrote before this frame apply first, then this frame's growth
    if (c->nodes_dirty && (rc = flush_updates(c)) != RT_OK) return rc;
    const int n = static_cast<int>(c->anim_ids.size());
    for (int i = 0; i < n; ++i) c->host_shapes[c->anim_ids[i]] = shapes[i];
    for (int i = 0; i < n; ++i)
        if (c->anim_ids[i] < static_cast<int>(c->shape_moved.size())) c->shape_moved[c->anim_ids[i]] = 1;
    // the root's box as k_refit grows it (grow_node: glm::min / max of the listed
    // shapes' growToInclude boxes), for rtx::view_root
    for (int i = 0; i < n; ++i) {
        const int e = c->refit_of[c->anim_ids[i]];
        if (e < 0 || e >= static_cast<int>(c->entry_root.size()) || !c->entry_root[e]) continue;
        float lo[3], hi[3];
        reference_box(shapes[i], lo, hi);
        for (int a = 0; a < 3; ++a) {
            c->root_lo[a] = lo[a] < c->root_lo[a] ? lo[a] : c->root_lo[a];
            c->root_hi[a] = c->root_hi[a] < hi[a] ? hi[a] : c->root_hi[a];
        }
    }
    if (c->brute && !c->brute_stale)  // the brute-force context: the same records, no nodes to grow
        for (int i = 0; i < n && !c->brute_stale; ++i)
            if (rt_update_shapes(c->brute, c->anim_ids[i], 1, &shapes[i]) != RT_OK) c->brute_stale = true;
    // the MT context: the same frame, its nodes grown the same way (its set follows c's)
    if (c->mtc && !c->mtc_stale && rt_animate(c->mtc, shapes) != RT_OK) c->mtc_stale = true;
    lap("host records");
    // the records and the growth on the device (one k_refit launch); a host rebuild
    // only after a bound changed kind
    rc = flush_updates(c, true);
    lap("flush");
    return rc;
}

int rt_build_lbvh(rt_ctx* c, float* device_ms) {
    if (!c || !c->have_scene) return RT_ERR_INVALID;
    if (set_dev(c) != RT_OK) return RT_ERR_DEVICE;
    if (const int rc0 = flush_updates(c)) return rc0;  // staging_shapes current
    const int S = c->S;
    const int N = S > 0 ? 2 * S - 1 : 0;
    std::vector<FlatNode> nodes(static_cast<size_t>(N));
    std::vector<int> idx(static_cast<size_t>(S));
    float ms = 0.f;
    if (S > 0) {
        FlatNode* dn = nullptr;
        int* di = nullptr;
        if (hipMalloc(&dn, N * sizeof(FlatNode)) != hipSuccess || hipMalloc(&di, S * sizeof(int)) != hipSuccess) {
            (void)hipFree(dn);
            return RT_ERR_NO_MEMORY;
        }
        // staging_shapes holds the current records (uploads, updates and rt_animate frames)
        int rc = rtl::lbvh_build(c->staging_shapes, S, dn, di, c->stream, &ms) == 0 ? RT_OK : RT_ERR_DEVICE;
        if (rc == RT_OK &&
            (hipMemcpyAsync(nodes.data(), dn, N * sizeof(FlatNode), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
             hipMemcpyAsync(idx.data(), di, S * sizeof(int), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
             sync_stream(c) != hipSuccess))
            rc = RT_ERR_DEVICE;
        (void)hipFree(dn);
        (void)hipFree(di);
        if (rc != RT_OK) return rc;
    }
    if (device_ms) *device_ms = ms;
    // adopt the tree exactly as if the host had uploaded it (validation, leaf
    // order, accelerator); the animated set is cleared as by any upload
    const std::vector<FlatShape> shapes(c->host_shapes);
    return rt_upload_scene(c, shapes.data(), S, nodes.data(), N, idx.data(), S);
}

int rt_scene_size(rt_ctx* c, int* num_shapes, int* num_nodes, int* num_indices) {
    if (!c || !c->have_scene) return RT_ERR_INVALID;
    if (num_shapes) *num_shapes = c->S;
    if (num_nodes) *num_nodes = c->N;
    if (num_indices) *num_indices = c->I;
    return RT_OK;
}

int rt_read_indices(rt_ctx* c, int* indices, int num_indices) {
    if (!c || !c->have_scene || num_indices != c->I || (num_indices > 0 && !indices)) return RT_ERR_INVALID;
    std::copy(c->host_idx.begin(), c->host_idx.end(), indices);
    return RT_OK;
}

int rt_read_nodes(rt_ctx* c, FlatNode* nodes, int N) {
    if (!c || !c->have_scene || N != c->N || (N > 0 && !nodes)) return RT_ERR_INVALID;
    if (N == 0) return RT_OK;
    if (set_dev(c) != RT_OK) return RT_ERR_DEVICE;
    if (const int rc = flush_updates(c)) return rc;
    HIP_TRY(hipMemcpyAsync(nodes, c->staging_nodes, N * sizeof(FlatNode), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(sync_stream(c));
    return RT_OK;
}

int rt_set_camera(rt_ctx* c, const FlatCamera* cam) {
    if (!c || !cam) return RT_ERR_INVALID;
    c->cam = *cam;
    c->have_cam = true;
    return RT_OK;
}

int rt_set_light(rt_ctx* c, const FlatLight* l) {
    if (!c || !l) return RT_ERR_INVALID;
    c->light = *l;
    c->have_light = true;
    return RT_OK;
}

int rt_set_params(rt_ctx* c, const rt_params* p) {
    if (!c || !p || p->maxBounces < 0) return RT_ERR_INVALID;
    c->params = *p;
    return RT_OK;
}

int rt_set_kernel(rt_ctx* c, int kernel) {
    if (!c || kernel < RT_KERNEL_AUTO || kernel > RT_KERNEL_ACCEL) return RT_ERR_INVALID;
    c->kernel = kernel;
    return RT_OK;
}

int rt_dispatch_rows(rt_ctx* c, int width, int height, int y0, int stripe, int step, int out_rows, float* dst,
                     size_t pitch) {
    return rt_dispatch_rows_fmt(c, width, height, y0, stripe, step, out_rows, dst, pitch, RT_FORMAT_RGBA32F);
}

// period = stripe * step, refused when it does not fit an int
static int stripe_period(int stripe, int step) {
    if (stripe <= 0 || step <= 0 || step > INT_MAX / stripe) return -1;
    return stripe * step;
}

int rt_dispatch_rows_fmt(rt_ctx* c, int width, int height, int y0, int stripe, int step, int out_rows, float* dst,
                         size_t pitch, int format) {
    return rt_dispatch_rows_ex(c, width, height, y0, stripe, stripe_period(stripe, step), out_rows, dst, pitch,
                               format);
}

int rt_dispatch_rows_ex(rt_ctx* c, int width, int height, int y0, int stripe, int period, int out_rows, float* dst,
                        size_t pitch, int format) {
    if (!c) return RT_ERR_INVALID;
    KParams kp;
    int rc = fill_kparams(c, width, height, y0, stripe, period, out_rows, dst, pitch, kp, format);
    if (rc != RT_OK) return rc;
    if (set_dev(c) != RT_OK) return RT_ERR_DEVICE;
    return render(c, kp);
}

int rt_dispatch(rt_ctx* c, int width, int height, int y0, int y1) {
    if (!c || width <= 0 || height <= 0 || y0 < 0 || y1 > height || y0 > y1) return RT_ERR_INVALID;
    if (set_dev(c) != RT_OK) return RT_ERR_DEVICE;
    if (width != c->img_w || height != c->img_h || !c->img) {
        HIP_TRY(sync_stream(c));
        hipFree(c->img);
        c->img = nullptr;
        c->img_w = c->img_h = 0;
        size_t pitch = 0;
        if (hipMallocPitch(reinterpret_cast<void**>(&c->img), &pitch, static_cast<size_t>(width) * 16, height) !=
            hipSuccess)
            return RT_ERR_NO_MEMORY;
        HIP_TRY(hipMemset2DAsync(c->img, pitch, 0, static_cast<size_t>(width) * 16, height, c->stream));
        c->img_pitch = pitch;
        c->img_w = width;
        c->img_h = height;
    }
    return rt_dispatch_rows(c, width, height, y0, 1, 1, y1 - y0,
                            reinterpret_cast<float*>(reinterpret_cast<char*>(c->img) + y0 * c->img_pitch),
                            c->img_pitch);
}

int rt_sync(rt_ctx* c) {
    if (!c) return RT_ERR_INVALID;
    if (set_dev(c) != RT_OK) return RT_ERR_DEVICE;
    // A host that waits for every frame (the reference's loop, src/main.cpp:290-462)
    // waits ~0.25 ms per frame: poll back to back (yielding the core) for the first
    // rtg::kSpinMs, then nap between polls (csrc/group_wait.h). The poll is on an event
    // recorded behind the stream's work, not on the stream: hipStreamQuery saw an empty
    // kernel end 15.2 us after its launch, the event 10.7 us (and 247.3 against 245.8 us
    // for a 235-us kernel; tools/native/wait_probe.hip, profiles/r04_wait_probe.txt). No
    // deadline: a single context has no peer to wait on.
    if (!c->sync_ev && hipEventCreateWithFlags(&c->sync_ev, hipEventDisableTiming) != hipSuccess) return RT_ERR_DEVICE;
    HIP_TRY(hipEventRecord(c->sync_ev, c->stream));
    const hipEvent_t ev = c->sync_ev;
    const rtg::WaitResult w = rtg::wait_bounded(
        [ev] {
            const hipError_t e = hipEventQuery(ev);
            return e == hipSuccess ? 0 : (e == hipErrorNotReady ? 1 : -1);
        },
        [] { return false; }, 0.0);
    if (w != rtg::kWaitDone) return RT_ERR_DEVICE;
    for (rt_ctx* x : {c, c->brute, c->mtc})  // the sub-contexts run on this stream
        if (x) stream_drained(x);
    return RT_OK;
}

int rt_sync_frame(rt_ctx* c) {
    if (!c) return RT_ERR_INVALID;
    // The last dispatch's frame ended at frame_ev if its launch recorded one (a latency-mode
    // cost frame, before the cost order's kernels) and no refit slot was taken since;
    // otherwise (and for work enqueued after the dispatch) the whole stream, as rt_sync.
    rt_ctx* t = c->frame_from;
    const bool known = t && (t == c || t == c->brute || t == c->mtc || (c->brute && t == c->brute->mtc) ||
                             (c->mtc && t == c->mtc->brute));
    if (!known || !t->frame_ev_set || !t->frame_ev || refit_launches(c) != c->frame_refits) return rt_sync(c);
    if (set_dev(c) != RT_OK) return RT_ERR_DEVICE;
    const hipEvent_t ev = t->frame_ev;
    const rtg::WaitResult w = rtg::wait_bounded(
        [ev] {
            const hipError_t e = hipEventQuery(ev);
            return e == hipSuccess ? 0 : (e == hipErrorNotReady ? 1 : -1);
        },
        [] { return false; }, 0.0);
    if (w != rtg::kWaitDone) return RT_ERR_DEVICE;
    // every refit slot in use was taken before the frame's render (none since): free
    for (rt_ctx* x : {c, c->brute, c->mtc})
        if (x) stream_drained(x);
    return RT_OK;
}

int rt_read_image(rt_ctx* c, float* dst, size_t pitch, int width, int height) {
    if (!c || !dst || !c->img || width != c->img_w || height != c->img_h ||
        pitch < static_cast<size_t>(c->img_w) * 16)
        return RT_ERR_INVALID;
    if (set_dev(c) != RT_OK) return RT_ERR_DEVICE;
    HIP_TRY(hipMemcpy2DAsync(dst, pitch, c->img, c->img_pitch, static_cast<size_t>(c->img_w) * 16, c->img_h,
                             hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(sync_stream(c));
    return RT_OK;
}

int rt_device_image(rt_ctx* c, void** p, size_t* pitch) {
    if (!c || !p || !pitch || !c->img) return RT_ERR_INVALID;
    *p = c->img;
    *pitch = c->img_pitch;
    return RT_OK;
}

int rt_collect_stats(rt_ctx* c, int width, int height, int y0, int stripe, int step, int out_rows, rt_stats* out) {
    return rt_collect_stats_ex(c, width, height, y0, stripe, stripe_period(stripe, step), out_rows, out);
}

int rt_collect_stats_ex(rt_ctx* c, int width, int height, int y0, int stripe, int period, int out_rows,
                        rt_stats* out) {
    if (!c || !out) return RT_ERR_INVALID;
    if (set_dev(c) != RT_OK) return RT_ERR_DEVICE;
    // The counting kernel needs a destination; use a scratch surface.
    float* scratch = nullptr;
    const size_t pitch = static_cast<size_t>(width > 0 ? width : 1) * 16;
    if (hipMalloc(&scratch, pitch * static_cast<size_t>(out_rows > 0 ? out_rows : 1)) != hipSuccess)
        return RT_ERR_NO_MEMORY;
    KParams kp;
    int rc = fill_kparams(c, width, height, y0, stripe, period, out_rows, scratch, pitch, kp);
    if (rc == RT_OK) {
        kp.stats = c->stats_dev;
        if (hipMemsetAsync(c->stats_dev, 0, ST_COUNT * sizeof(unsigned long long), c->stream) != hipSuccess)
            rc = RT_ERR_DEVICE;
        if (rc == RT_OK) rc = launch(c, kp, true);
        unsigned long long h[ST_COUNT];
        if (rc == RT_OK && (hipMemcpyAsync(h, c->stats_dev, sizeof h, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
                            sync_stream(c) != hipSuccess))
            rc = RT_ERR_DEVICE;
        if (rc == RT_OK) {
            out->pixels = h[ST_PIXELS];
            out->closest_rays = h[ST_CLOSEST];
            out->shadow_rays = h[ST_SHADOW];
            out->node_visits = h[ST_NODES];
            for (int i = 0; i < 4; ++i) {
                out->bvh_tests[i] = h[ST_BVH0 + i];
                out->brute_tests[i] = h[ST_BR0 + i];
            }
            out->closest_updates = h[ST_UPD];
            out->hits = h[ST_HITS];
        }
    }
    sync_stream(c);
    hipFree(scratch);
    return rc;
}

int rt_kernel_times(rt_ctx* c, float* ms, int cap) {
    if (!c || (cap > 0 && !ms) || cap < 0) return RT_ERR_INVALID;
    if (set_dev(c) != RT_OK) return RT_ERR_DEVICE;
    const int n = c->ring_used;
    for (int i = 0; i < n; ++i) {
        HIP_TRY(hipEventSynchronize(c->ring1[i]));
        float t = 0.f;
        HIP_TRY(hipEventElapsedTime(&t, c->ring0[i], c->ring1[i]));
        if (i < cap) ms[i] = t;
    }
    c->ring_used = 0;
    return n;
}

int rt_last_kernel_ms(rt_ctx* c, float* ms) {
    if (!c || !ms || !c->timed) return RT_ERR_INVALID;
    if (set_dev(c) != RT_OK) return RT_ERR_DEVICE;
    HIP_TRY(hipEventSynchronize(c->last1));
    HIP_TRY(hipEventElapsedTime(ms, c->last0, c->last1));
    return RT_OK;
}

}  // extern "C"

extern "C" int rt_accel_info_get(rt_ctx* c, rt_accel_info* out) {
    if (!c || !out) return RT_ERR_INVALID;
    // the accelerator the next dispatch uses: pending updates applied first (a flush may rebuild it)
    if (c->have_scene) {
        if (set_dev(c) != RT_OK) return RT_ERR_DEVICE;
        if (const int rc = flush_updates(c)) return rc;
    }
    out->built = c->accel_ok ? 1 : 0;
    out->local_nodes = static_cast<int>(c->accel.lbox.size());
    out->local_leaves = c->accel.local_leaves;
    out->bounded_prims = c->accel.bounded_prims;
    out->always_prims = c->accel.always_prims;
    out->max_stack = c->accel.max_stack;
    out->last_kernel = c->last_kind;
    out->scene_tree = c->accel_ok && c->st_root != kNoChild ? 1 : 0;
    out->scene_nodes = static_cast<int>(c->accel.st.wchild.size() / rta::kWide);
    out->scene_items = static_cast<int>(c->accel.st.item_ref.size());
    out->scene_height = c->accel.st.height;
    out->tree_nested = c->accel.st.nested;
    out->record_bytes = c->accel_ok ? static_cast<int>(std::min<size_t>(c->record_bytes, 0x7fffffff)) : 0;
    return RT_OK;
}

extern "C" int rt_set_tree(rt_ctx* c, int mode) {
    if (!c || (mode != RT_TREE_REFERENCE && mode != RT_TREE_SCENE)) return RT_ERR_INVALID;
    c->tree_mode = mode;
    return RT_OK;
}

extern "C" int rt_debug_anim_rebuilds(rt_ctx* c) { return c ? c->anim_rebuilds : -1; }
extern "C" int rt_debug_refits(rt_ctx* c) { return c ? c->updates_flushed : -1; }
// Diagnostics: how flush_updates launches the refit (RefitArgs: 0 one launch whose box
// roles wait for the record role, 1 two launches, 2 one launch deriving every box from
// the records). Same device state either way.
// out[7]: dirty slots, their largest and total prim range, reference nodes listing an
// entry, refit entries, bytes of the last flush's pinned records, compactions
// Diagnostics: the rebuild a refit asks for runs on a host thread (1, default) or in that
// refit's flush (0). rt_debug_rebuild_state: out[0] a rebuild is running, out[1] rebuilds
// asked for, out[2] rebuilt accelerators swapped in, out[3] the scene tree is suspended.
extern "C" int rt_debug_async_rebuild(rt_ctx* c, int on) {
    if (!c) return RT_ERR_INVALID;
    c->async_rebuild = on ? 1 : 0;
    return RT_OK;
}
extern "C" int rt_debug_rebuild_state(rt_ctx* c, int* out) {
    if (!c || !out) return RT_ERR_INVALID;
    out[0] = c->rebuild ? 1 : 0;
    out[1] = c->anim_rebuilds;
    out[2] = c->async_swaps;
    out[3] = c->st_suspended ? 1 : 0;
    return RT_OK;
}

extern "C" int rt_debug_refit_stats(rt_ctx* c, long long* out) {
    if (!c || !out) return RT_ERR_INVALID;
    out[0] = c->n_dirty;
    out[1] = c->dirty_max;
    out[2] = c->dirty_sum;
    out[3] = c->anim.nodes;
    out[4] = static_cast<long long>(c->refit_ids.size());
    out[5] = c->last_flush_bytes;
    out[6] = c->refit_compactions;
    return RT_OK;
}

extern "C" int rt_debug_refit(rt_ctx* c, int mode) {
    if (!c || mode < -1 || mode > 4) return RT_ERR_INVALID;
    c->refit_mode = mode;
    return RT_OK;
}

extern "C" int rt_set_walk(rt_ctx* c, int lane_from_depth) {
    if (!c || lane_from_depth < -1) return RT_ERR_INVALID;
    c->lane_from_depth = lane_from_depth;  // -1: back to the automatic policy (walk_from)
    return RT_OK;
}

// Diagnostics: back-face cone culling on/off (takes effect at the next upload).
extern "C" int rt_debug_cone_cull(rt_ctx* c, int on) {
    if (!c) return RT_ERR_INVALID;
    c->cone_cull = on ? 1 : 0;
    return c->have_scene ? upload_accel(c) : RT_OK;
}

// Diagnostics: cap the stack entries of scene-tree walks (0 = none). Exact at
// any value: a lane that runs out walks the reference tree (lane_walk).
extern "C" int rt_debug_scene_stack(rt_ctx* c, int n) {
    if (!c || n < 0) return RT_ERR_INVALID;
    c->scene_stack = n;
    return RT_OK;
}

// Diagnostics: override the per-lane LDS stack depth of k_accel (0 = computed
// bound). A value below the bound can drop stack entries: timing studies only.
// Diagnostics: shadow walks of bounces >= from walk per lane (-1: the default policy).
extern "C" int rt_debug_shadow_walk(rt_ctx* c, int from) {
    if (!c || from < -1) return RT_ERR_INVALID;
    c->shadow_walk_override = from;
    return RT_OK;
}

// Diagnostics: only waves with at most `lanes` rays alive hand them to the tail kernel.
extern "C" int rt_debug_tail_lanes(rt_ctx* c, int lanes) {
    if (!c || lanes < 0 || lanes > 64) return RT_ERR_INVALID;
    c->tail_max_lanes = lanes;
    return RT_OK;
}

extern "C" int rt_set_tail(rt_ctx* c, int from_bounce) {
    if (!c || from_bounce < RT_TAIL_AUTO) return RT_ERR_INVALID;
    c->tail_from = from_bounce;
    return RT_OK;
}

// Diagnostics: re-derive the cost order every `period` dispatches (1: every one).
extern "C" int rt_debug_sched_period(rt_ctx* c, int period) {
    if (!c || period < 1) return RT_ERR_INVALID;
    c->sched_period = period;
    c->sched_frame = 0;
    return RT_OK;
}

extern "C" int rt_debug_moving(rt_ctx* c, int period, int dilate, int split) {
    if (!c || period < 0 || dilate < 0 || dilate > 64) return RT_ERR_INVALID;
    c->moving_period = period;
    c->moving_dilate = dilate;
    c->moving_split = split ? 1 : 0;
    return RT_OK;
}

// Diagnostics / policy: where the cost order's kernels run (0: the context's stream after
// the render; 1: an order stream in latency-mode dispatches; 2: the order stream always).
extern "C" int rt_debug_order_stream(rt_ctx* c, int mode) {
    if (!c || mode < 0 || mode > 2) return RT_ERR_INVALID;
    c->order_mode = mode;
    return RT_OK;
}

// Diagnostics / policy: latency-mode cost frames record the event rt_sync_frame waits for (1, default) or not (0).
extern "C" int rt_debug_frame_event(rt_ctx* c, int on) {
    if (!c || on < 0 || on > 1) return RT_ERR_INVALID;
    c->frame_event = on;
    return RT_OK;
}

extern "C" int rt_debug_cost_dilate(rt_ctx* c, int r) {
    if (!c || r < 0 || r > 64) return RT_ERR_INVALID;
    c->cost_dilate = r;
    return RT_OK;
}

extern "C" int rt_debug_lane_stack(rt_ctx* c, int n) {
    if (!c || n < 0 || n > kMaxStack) return RT_ERR_INVALID;
    c->lane_stack_override = n;
    return RT_OK;
}

extern "C" int rt_set_kernel_timing(rt_ctx* c, int on) {
    if (!c) return RT_ERR_INVALID;
    c->timing = on != 0;
    return RT_OK;
}

extern "C" int rt_set_latency_mode(rt_ctx* c, int on) {
    if (!c || on < 0 || on > 1) return RT_ERR_INVALID;
    c->latency_mode = on;
    return RT_OK;
}

extern "C" int rt_set_schedule(rt_ctx* c, int mode) {
    if (!c || mode < RT_SCHED_ROWS || mode > RT_SCHED_COST_XCD) return RT_ERR_INVALID;
    c->schedule = mode;
    c->sched_valid = 0;
    return RT_OK;
}

// Diagnostics: dispatch order of k_accel's tiles (a permutation of [0, n)),
// used when n equals the launch's tile count; n = 0 clears it.
extern "C" int rt_debug_tile_order(rt_ctx* c, const int* order, int n) {
    if (!c || n < 0 || (n > 0 && !order)) return RT_ERR_INVALID;
    if (set_dev(c) != RT_OK) return RT_ERR_DEVICE;
    hipFree(c->tile_order);
    c->tile_order = nullptr;
    c->tile_order_n = 0;
    if (n == 0) return RT_OK;
    std::vector<char> seen(n, 0);
    for (int i = 0; i < n; ++i) {
        if (order[i] < 0 || order[i] >= n || seen[order[i]]) return RT_ERR_INVALID;
        seen[order[i]] = 1;
    }
    if (hipMalloc(&c->tile_order, n * sizeof(int)) != hipSuccess) return RT_ERR_NO_MEMORY;
    HIP_TRY(hipMemcpy(c->tile_order, order, n * sizeof(int), hipMemcpyHostToDevice));
    c->tile_order_n = n;
    return RT_OK;
}

// Diagnostics: the current cost order (tile indices, longest first) into out[0, n);
// returns the tiles copied (0 when no order exists yet).
extern "C" int rt_debug_sched_order(rt_ctx* c, int* out, int n) {
    if (!c || n < 0 || (n > 0 && !out)) return RT_ERR_INVALID;
    if (set_dev(c) != RT_OK) return RT_ERR_DEVICE;
    HIP_TRY(sync_stream(c));
    const int k = std::min(n, c->sched_valid);
    if (k > 0 && c->sched_order)
        HIP_TRY(hipMemcpy(out, c->sched_order, static_cast<size_t>(k) * sizeof(int), hipMemcpyDeviceToHost));
    return c->sched_order ? k : 0;
}

// Diagnostics: the first k tiles of the cost order (the heaviest) each run as `parts`
// waves (1, 2, 4 or 8), one band of 64 / parts pixels per wave; parts = 1: off;
// k = -1: the default policy (kHeavyAutoSlots).
extern "C" int rt_debug_heavy(rt_ctx* c, int k, int parts) {
    if (!c || k < -1 || parts < 1 || parts > 64 || (parts & (parts - 1)) != 0) return RT_ERR_INVALID;
    c->heavy_k = k;
    c->heavy_parts = parts;
    return RT_OK;
}

// Diagnostics: the first k dispatch slots of the cost order (the heaviest tiles) walk
// their camera rays (mode bit 0) and / or the camera rays' shadow rays (bit 1) per lane;
// k = -1: the default policy.
// Diagnostics: a cost-recording dispatch ranks the tiles by their waves' wall time
// (1) or by their lanes' node steps + tests (0); -1: the default policy.
extern "C" int rt_debug_cost_time(rt_ctx* c, int mode) {
    if (!c || mode < -1 || mode > 1) return RT_ERR_INVALID;
    c->cost_time = mode;
    c->sched_valid = 0;
    return RT_OK;
}

extern "C" int rt_debug_lane_k(rt_ctx* c, int k, int mode) {
    if (!c || k < -1 || mode < 0 || mode > 3) return RT_ERR_INVALID;
    c->lane_k = k;
    c->lane_k_mode = mode;
    return RT_OK;
}

// Diagnostics: split per-lane walks (lane_walk_any) of waves with at most max_rays rays
// over groups of at most group lanes (a power of two, 2..64); max_rays = 0 turns it off.
extern "C" int rt_debug_split(rt_ctx* c, int max_rays, int group) {
    if (!c || max_rays < 0 || max_rays > 32 || group < 2 || group > 64 || (group & (group - 1))) return RT_ERR_INVALID;
    c->split_max = max_rays;
    c->split_g = group;
    return RT_OK;
}

// Diagnostics: speculative while-while in the per-lane walk (1 on, the default; 0 off).
extern "C" int rt_debug_spec(rt_ctx* c, int mode) {
    if (!c || mode < 0 || mode > 1) return RT_ERR_INVALID;
    c->spec_mode = mode;
    return RT_OK;
}

extern "C" int rt_set_launch(rt_ctx* c, int waves_per_block, int persistent) {
    if (!c || (waves_per_block != 1 && waves_per_block != 2 && waves_per_block != 4)) return RT_ERR_INVALID;
    c->waves_per_block = waves_per_block;
    c->persistent = persistent ? 1 : 0;
    return RT_OK;
}

// Diagnostics (not part of rt_api.h): enable per-tile records for k_accel
// (cap tiles; 0 disables) and read them back (kTileRec u64 per tile, layout
// at kTileRec). Synchronous.
extern "C" int rt_debug_tile_times(rt_ctx* c, int cap, unsigned long long* out) {
    if (!c || cap < 0) return RT_ERR_INVALID;
    if (set_dev(c) != RT_OK) return RT_ERR_DEVICE;
    HIP_TRY(sync_stream(c));
    if (out && c->tile_times && cap > 0) {
        const size_t n = std::min(static_cast<size_t>(cap), c->tile_times_cap);
        HIP_TRY(hipMemcpy(out, c->tile_times, n * kTileRec * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        return static_cast<int>(n);
    }
    hipFree(c->tile_times);
    c->tile_times = nullptr;
    c->tile_times_cap = 0;
    if (cap > 0) {
        if (hipMalloc(&c->tile_times, static_cast<size_t>(cap) * kTileRec * sizeof(unsigned long long)) != hipSuccess)
            return RT_ERR_NO_MEMORY;
        c->tile_times_cap = cap;
    }
    return RT_OK;
}

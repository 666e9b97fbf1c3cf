// rt_device.h — device-side scene layout and the per-ray primitives shared by
// every render kernel. Included by rt_kernels.hip only.
//
// All arithmetic follows the reference shader (src/shaders/gpu_shader.comp)
// with glm's operation order (dot = (x+y)+z, normalize = v*(1/sqrt(v.v)),
// reflect = I - N*dot(N,I)*2, mix = x+a*(y-x)); the file is compiled with
// -ffp-contract=off and IEEE div/sqrt so a pixel's discrete decisions (hit or
// miss, shadowed or lit, which shape is closest) are those of the CPU oracle.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rtd {

// ---------------------------------------------------------------------------
// HBM layout (built on device by the pack kernels from the uploaded FlatShape
// / FlatNode records; see DESIGN.md "Data layout in HBM").
//
// Shape record: 80 B = 5 x float4, one per shape, stored twice: in shape order
// (brute-force branch) and in leaf order, i.e. geo_leaf[j] is the shape
// bvhIndices[j], so a leaf scan is a contiguous stream and the index
// indirection of gpu_shader.comp:404 is paid once at upload.
//   w0 = type (int bits), w1 = shape index (int bits), f[0..17] = payload:
//   sphere   : f0-2 centre, f3 radius
//   plane    : f0-2 normal, f3 D
//   wall     : f0-2 normal, f3 D, f4-6 start, f7 width, f8 height,
//              f9-11 u axis, f12-14 v axis (gpu_shader.comp:305-307, precomputed)
//   triangle : f0-2 normal, f3 D, f4-6 P1, f7-9 E1=P2-P1, f10-12 E2=P3-P1,
//              f13 d00, f14 d01, f15 d11, f16 denom (gpu_shader.comp:218-229)
// Material: 32 B = 2 x float4 per shape index: color.xyz, fresnel |
//   ambient, diffuse, specular, float(shininess).
// Node: 32 B = 2 x float4: bmin.xyz, a | bmax.xyz, b (int bits);
//   inner: a = left, b = right; leaf: a = -(start+1), b = numShapes.
struct GeoRec {
    int type, idx;
    float f[18];
};
static_assert(sizeof(GeoRec) == 80, "GeoRec is 5 float4");

// The accelerated walks' prim record (k_pack_prims), 64 B: f[0..14] as GeoRec's,
// except that triangles keep d01 in f[13] and the barycentric denominator in
// f[14]; d00 and d11 are recomputed from the stored edges with pack_geo's float
// operations, so they have the same bits. st = seq << 2 | type, seq the shape's
// rank in the reference walk: (distance, st) orders candidates as (distance, seq).
// Shape types outside 0-3 are packed as planes with a NaN normal (no hit, as in
// the reference). The shape index is kept apart (AccelPtrs::prim_shape), read
// once per bounce for the winner's material.
struct PrimRec {
    float f[15];
    int st;
};
static_assert(sizeof(PrimRec) == 64, "PrimRec is 4 float4");
__device__ __forceinline__ int prim_type(const PrimRec& g) { return g.st & 3; }

struct V {
    float x, y, z;
};
__host__ __device__ __forceinline__ V mk(float x, float y, float z) { return V{x, y, z}; }
__host__ __device__ __forceinline__ V operator+(V a, V b) { return V{a.x + b.x, a.y + b.y, a.z + b.z}; }
__host__ __device__ __forceinline__ V operator-(V a, V b) { return V{a.x - b.x, a.y - b.y, a.z - b.z}; }
__host__ __device__ __forceinline__ V operator-(V a) { return V{-a.x, -a.y, -a.z}; }
__host__ __device__ __forceinline__ V operator*(V a, float s) { return V{a.x * s, a.y * s, a.z * s}; }
__host__ __device__ __forceinline__ V operator*(float s, V a) { return V{s * a.x, s * a.y, s * a.z}; }
__device__ __forceinline__ V mulv(V a, V b) { return V{a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ V divs(V a, float s) { return V{a.x / s, a.y / s, a.z / s}; }
__host__ __device__ __forceinline__ float dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__host__ __device__ __forceinline__ V cross(V a, V b) {
    return V{a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y};
}
__host__ __device__ __forceinline__ float len(V a) { return __builtin_sqrtf(dot(a, a)); }
__host__ __device__ __forceinline__ V normalize(V a) { return a * (1.0f / __builtin_sqrtf(dot(a, a))); }
__host__ __device__ __forceinline__ float dist(V a, V b) { return len(b - a); }
__host__ __device__ __forceinline__ V reflect(V i, V n) { return i - (n * dot(n, i)) * 2.0f; }
__device__ __forceinline__ V mix(V x, V y, float a) { return x + a * (y - x); }
__device__ __forceinline__ float gmax(float a, float b) { return (a < b) ? b : a; }  // GLSL/glm max
__device__ __forceinline__ float gmin(float a, float b) { return (b < a) ? b : a; }  // GLSL/glm min

enum { NONE = 0, INNER = 1, OUTER = 2 };

struct Ray {
    V o, d;
};

// Everything a render kernel needs, passed by value.
struct KParams {
    const float4* __restrict__ geo_leaf;  // I records
    const float4* __restrict__ geo_lin;   // S records
    const float4* __restrict__ mat;       // S materials
    const float4* __restrict__ nodes;     // N nodes
    int S, N, I;
    int max_stack;                        // reference walk's stack need (host-computed)
    V cam_pos, cam_front, cam_right, cam_up;
    float plane_w, plane_h;               // imagePlaneWidth/Height (gpu_shader.comp:156-157)
    V light_pos, light_color;
    float resX, resY;
    int maxBounces, useBVH, useFresnel, useMT;
    int width, height, y0, stripe, period, out_rows;  // compact row r -> image row (image_row)
    char* __restrict__ dst;
    size_t pitch;
    unsigned long long* __restrict__ stats;  // rt_stats layout, STATS kernels only
    int* __restrict__ tile_counter;          // persistent launches: next 8x8 tile (zeroed per launch)
    unsigned long long* __restrict__ tile_times;  // optional: start/end wall clock per tile
    int tiles_x, tiles;                      // 8x8 tiles per row, total
    const int* __restrict__ tile_order;      // optional dispatch order of the tiles (rt_set_schedule)
    int lane_k, lane_k_mode;                 // the first lane_k dispatch slots: camera rays (bit 0) /
                                             // their shadows (bit 1) walk per lane
    int heavy_k, heavy_parts;                // the first heavy_k tiles of tile_order run as heavy_parts
                                             // waves each, one band of 64/heavy_parts pixels per wave
    unsigned* __restrict__ tile_cost;        // optional: each tile's work (rt_set_schedule)
    int cost_time;                           // tile_cost in wave wall-clock ticks, not lane work
    unsigned long long* __restrict__ heavy_acc;  // with tile_cost and heavy_k: per split tile its parts done
                                                 // (bits 56..63) and summed work (bits 0..55), zeroed per dispatch
    unsigned* __restrict__ sched_hist;       // with tile_cost: work-bucket histogram copies of this frame
    int lane_from_depth;                     // k_accel: bounces >= this walk per lane
    int shadow_lane_from;                    // k_accel: shadow walks of bounces >= this walk per lane
    int root_ok;                             // root_lo/hi hold node N-1's current bounds (k_accel)
    float root_lo[3], root_hi[3];
    int lane_stack;                          // per-lane LDS stack entries
    // compaction (rt_set_tail): k_accel queues the rays alive after bounce tail_from - 1,
    // k_accel_tail runs their remaining bounces 64 to a wave; tail_queue == nullptr: off
    float4* __restrict__ tail_queue;         // 3 float4 per ray: o|acc.x, d|acc.y, att|acc.z
    int* __restrict__ tail_px;               // per queued ray its pixel, row * width + x (52 B a ray, was 64)
    int* __restrict__ tail_count;            // per region: rays queued by this dispatch
    int* __restrict__ tail_count_next;       // the next dispatch's counters (zeroed by k_accel_tail)
    int tail_from;
    int tail_rx, tail_regions;               // 64x64-pixel regions: per row, total (one counter each)
    int tail_counters;                       // counters per set (>= tail_regions; all zeroed for the next)
    int tail_max_lanes;                      // a wave queues its rays only if at most this many are alive
    int rgb;                                 // output format (rt_dispatch_rows_fmt): 0 RGBA32F, 1 packed RGB32F
                                             // (12 B per pixel), 2 RGBA32F at the image row (RT_FORMAT_RGBA32F_IMAGE)
    float shadow_off;                        // k_accel's shadow-ray offset: 1e-3 (BVH branch, gpu_shader.comp:469);
                                             // 1e-5 when it renders the brute branch (:565, rt_ctx::brute)
};

// Row mapping of rt_dispatch_rows_ex (include/rt_api.h): stripes of `stripe` rows
// starting at y0, one every `period` rows (rt_dispatch_rows: period = stripe * step),
// i.e. y0 + (r / stripe) * period + r % stripe. Written this way because it keeps
// the register allocation of every production k_accel instance as it was (the
// direct form moved 23 VGPRs of the compacting instance to scratch).
__device__ __forceinline__ int image_row(const KParams& kp, int r) {
    return kp.y0 + r + (r / kp.stripe) * (kp.period - kp.stripe);
}

// getRay (gpu_shader.comp:155-168); imagePlaneHeight/Width come from the host
// (same tanf as the oracle) since they are per-frame constants.
__device__ __forceinline__ Ray get_ray(const KParams& kp, float ndcX, float ndcY) {
    V p = ((kp.cam_pos + kp.cam_front) + (ndcX * kp.plane_w / 2.0f) * kp.cam_right) +
          (ndcY * kp.plane_h / 2.0f) * kp.cam_up;
    return Ray{kp.cam_pos, normalize(p - kp.cam_pos)};
}

// Result of one primitive test. Only INNER hits matter to every caller.
struct Hit {
    int type;
    V p;
};

// get_intersection (gpu_shader.comp:242-328) on a packed record.
//   sphere :246-271, plane :272-286, wall :287-316,
//   triangle barycentric :196-240 / Moller-Trumbore :170-195.
__device__ __forceinline__ Hit intersect(const GeoRec& g, const Ray& r, int use_mt) {
    Hit h{NONE, V{0.f, 0.f, 0.f}};
    const float* f = g.f;
    if (g.type == 0) {
        V c = mk(f[0], f[1], f[2]);
        V oc = r.o - c;
        float aa = dot(r.d, r.d);
        float bb = 2.0f * dot(r.d, oc);
        float cc = dot(oc, oc) - f[3] * f[3];
        float D = bb * bb - 4.0f * aa * cc;
        if (D > 0.0f) {
            float sD = __builtin_sqrtf(D);
            float t1 = (-bb - sD) / (2.0f * aa);
            if (t1 > 0.0f) {
                h.type = INNER;
                h.p = r.o + t1 * r.d;
            }
            // t2 > 0 is OUTER (:263-268): never used, not computed.
        }
        return h;
    }
    if (g.type < 1 || g.type > 3) return h;
    if (g.type == 3 && use_mt) {
        V p1 = mk(f[4], f[5], f[6]), e1 = mk(f[7], f[8], f[9]), e2 = mk(f[10], f[11], f[12]);
        V hh = cross(r.d, e2);
        float a = dot(e1, hh);
        if (__builtin_fabsf(a) < 1e-5f) return h;
        float fi = 1.0f / a;
        V s = r.o - p1;
        float u = fi * dot(s, hh);
        if (u < 0.0f || u > 1.0f) return h;
        V q = cross(s, e1);
        float v = fi * dot(r.d, q);
        if (v < 0.0f || u + v > 1.0f) return h;
        float t = fi * dot(e2, q);
        if (t > 0.0f) {
            h.type = INNER;
            h.p = r.o + t * r.d;
        }
        return h;
    }
    // plane test shared by plane, wall and barycentric triangle
    V n = mk(f[0], f[1], f[2]);
    float np = dot(n, r.d);
    if (np == 0.0f) return h;
    float t = -(f[3] + dot(n, r.o)) / np;
    if (!(t > 0.0f) || !(np > 0.0f)) return h;  // t<=0: NONE; np<=0: OUTER
    V p = r.o + t * r.d;
    if (g.type == 2) {
        V lp = p - mk(f[4], f[5], f[6]);
        float up = dot(lp, mk(f[9], f[10], f[11]));
        float vp = dot(lp, mk(f[12], f[13], f[14]));
        if (up < 0.0f || up > f[7] || vp < 0.0f || vp > f[8]) return h;
    } else if (g.type == 3) {
        V tp = p - mk(f[4], f[5], f[6]);
        float d20 = dot(tp, mk(f[7], f[8], f[9]));
        float d21 = dot(tp, mk(f[10], f[11], f[12]));
        float v = (f[15] * d20 - f[14] * d21) / f[16];
        float w = (f[13] * d21 - f[14] * d20) / f[16];
        float u = 1.0f - v - w;
        if (u < 0.0f || v < 0.0f || w < 0.0f) return h;
    }
    h.type = INNER;
    h.p = p;
    return h;
}

// getNormalFromShape (gpu_shader.comp:64-71).
__device__ __forceinline__ V shape_normal(const GeoRec& g, V p) {
    if (g.type == 0) return normalize(p - mk(g.f[0], g.f[1], g.f[2]));
    return mk(g.f[0], g.f[1], g.f[2]);
}
__device__ __forceinline__ V shape_normal(const PrimRec& g, V p) {
    if (prim_type(g) == 0) return normalize(p - mk(g.f[0], g.f[1], g.f[2]));
    return mk(g.f[0], g.f[1], g.f[2]);
}

struct Mat {
    V color;
    float fresnel, ambient, diffuse, specular, shininess;
};

__device__ __forceinline__ Mat load_mat(const float4* __restrict__ mat, int idx) {
    float4 a = mat[2 * idx], b = mat[2 * idx + 1];
    return Mat{mk(a.x, a.y, a.z), a.w, b.x, b.y, b.z, b.w};
}

// phong (gpu_shader.comp:331-361).
__device__ __forceinline__ V phong(V p, V n, V view, V lpos, V lcol, const Mat& m) {
    float dl = dist(lpos, p);
    V lc = divs(lcol, dl);
    V amb = m.ambient * lc;
    V ldir = normalize(lpos - p);
    float diff = gmax(dot(n, ldir), 0.0f);
    V dif = (m.diffuse * diff) * lc;
    V spc = mk(0.f, 0.f, 0.f);
    if (diff > 0.0f) {
        V rd = reflect(-ldir, n);
        float sp = powf(gmax(dot(view, rd), 0.0f), m.shininess);
        spc = (m.specular * sp) * lc;
    }
    return mulv((amb + dif) + spc, m.color);
}

// rayIntersectsAABB (gpu_shader.comp:364-377); inv computed once per ray.
__device__ __forceinline__ bool ray_aabb(V o, V inv, V bmin, V bmax) {
    V t0 = mulv(bmin - o, inv), t1 = mulv(bmax - o, inv);
    float lx = gmin(t0.x, t1.x), ly = gmin(t0.y, t1.y), lz = gmin(t0.z, t1.z);
    float hx = gmax(t0.x, t1.x), hy = gmax(t0.y, t1.y), hz = gmax(t0.z, t1.z);
    float tmin = gmax(gmax(lx, ly), lz);
    float tmax = gmin(gmin(hx, hy), hz);
    return tmax >= tmin && tmax > 0.0f;
}

__device__ __forceinline__ V inv_dir(V d) { return mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z); }

// ray_aabb with IEEE min/max (v_min3/v_max3). GLSL min/max differ from them
// only on NaN operands (and the sign of an equal zero, which no comparison
// sees), so the result is the same whenever no slab value can be NaN: finite
// origin, finite non-zero reciprocals and NaN-free bounds (aabb_fast_ok).
__device__ __forceinline__ bool ray_aabb_fast(V o, V inv, V bmin, V bmax) {
    V t0 = mulv(bmin - o, inv), t1 = mulv(bmax - o, inv);
    float tmin = fmaxf(fmaxf(fminf(t0.x, t1.x), fminf(t0.y, t1.y)), fminf(t0.z, t1.z));
    float tmax = fminf(fminf(fmaxf(t0.x, t1.x), fmaxf(t0.y, t1.y)), fmaxf(t0.z, t1.z));
    return tmax >= tmin && tmax > 0.0f;
}
__device__ __forceinline__ bool aabb_fast_ok(V o, V inv) {
    const float big = 3.0e38f;
    return fabsf(o.x) < big && fabsf(o.y) < big && fabsf(o.z) < big && fabsf(inv.x) < big &&
           fabsf(inv.y) < big && fabsf(inv.z) < big && inv.x != 0.0f && inv.y != 0.0f && inv.z != 0.0f;
}

__device__ __forceinline__ GeoRec load_rec(const float4* __restrict__ base, int j) {
    GeoRec g;
    float4* dst = reinterpret_cast<float4*>(&g);
    const float4* src = base + 5 * static_cast<size_t>(j);
#pragma unroll
    for (int k = 0; k < 5; ++k) dst[k] = src[k];
    return g;
}

__device__ __forceinline__ PrimRec load_prim(const float4* __restrict__ base, int j) {
    PrimRec g;
    float4* dst = reinterpret_cast<float4*>(&g);
    const float4* src = base + 4 * static_cast<size_t>(j);
#pragma unroll
    for (int k = 0; k < 4; ++k) dst[k] = src[k];
    return g;
}

// Writes the pixel for output row r, column x.
__device__ __forceinline__ void store_px(const KParams& kp, int r, int x, float4 v) {
    if (kp.rgb == 1) {  // alpha is always 1 (gpu_shader.comp:437,623): the multi-GPU gather sends 12 B per pixel
        float* p = reinterpret_cast<float*>(kp.dst + static_cast<size_t>(r) * kp.pitch) + 3 * x;
        __builtin_nontemporal_store(v.x, p);
        __builtin_nontemporal_store(v.y, p + 1);
        __builtin_nontemporal_store(v.z, p + 2);
        return;
    }
    // RT_FORMAT_RGBA32F_IMAGE (rgb == 2): the pixel goes to its image row of a whole
    // W x H surface (rt_group's rank 0 renders its stripes straight into the frame)
    const int row_i = kp.rgb == 2 ? image_row(kp, r) : r;
    float4* row = reinterpret_cast<float4*>(kp.dst + static_cast<size_t>(row_i) * kp.pitch);
    // streaming store (one global_store_dwordx4 ... nt): the kernel never reads the image
    // back, so it should not displace the scene records from L2 (config 3 -1.1 %, config 2 -1.7 %)
    __builtin_nontemporal_store(v.x, &row[x].x);
    __builtin_nontemporal_store(v.y, &row[x].y);
    __builtin_nontemporal_store(v.z, &row[x].z);
    __builtin_nontemporal_store(v.w, &row[x].w);
}

}  // namespace rtd

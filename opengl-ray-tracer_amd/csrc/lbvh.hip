// lbvh.hip — opt-in device BVH build: a linear BVH
// (Karras, "Maximizing parallelism in the construction of BVHs, octrees and
// k-d trees", HPG 2012) over the shapes already in HBM, written in the
// reference's FlatNode / bvhIndices layout so that every consumer of a
// reference tree (the kernels, the accelerator, rt_read_nodes) takes it as is.
//
// It is NOT the reference builder's tree (split/buildBVH, src/main.cpp:1111-1193,
// is a sequential top-down spatial-midpoint split): frames rendered over it are
// the reference shader's frames for THIS tree, which the tests check against
// the oracle rendering the same tree. What it keeps from the reference:
//   * node boxes: BoundingBox::growToInclude per shape (src/BoundingBox.hpp:44-95,
//     sphere c±r, wall start ∪ Wall::end() with its own tangent basis,
//     triangles only when their x components are finite, planes nothing);
//     an inner box is the union of its children, i.e. of its shapes;
//   * primitive centres: the ones split() sorts by (src/main.cpp:1127-1140);
//   * the root is node N-1 (gpu_shader.comp:386), leaves have leftChild == -1.
// Layout: leaf j (one shape: bvhIndices[j]) is node j; Karras inner node i is
// node (2n-2) - i, so inner node 0 (the root) is N-1 = 2n-2.
//
// Steps (one stream, no host round trip):
//   k_lbvh_prep     shape boxes + centres, centre bounds (atomic min/max on
//                   order-preserving integer images of the floats)
//   k_lbvh_morton   30-bit Morton code of the centre in the bounds, key =
//                   code << 32 | shape (unique keys: equal codes split by index)
//   radix sort      rocprim::radix_sort_keys on the 62 key bits
//   k_lbvh_inner    per inner node: its key range and split (longest common
//                   prefix), children and parent links
//   k_lbvh_leaves   leaf records, then bottom-up box unions: the second thread
//                   to reach a node (acq_rel counter) unions its children.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

#include <cmath>
#include <cstdint>

#include "../../include/rt_flat.h"
#include "lbvh.h"

namespace {

constexpr int kThreads = 256;

struct P3 {
    float x, y, z;
};
__device__ __forceinline__ P3 p3(rt_vec3 v) { return P3{v.x, v.y, v.z}; }
__device__ __forceinline__ float gmin(float a, float b) { return (b < a) ? b : a; }  // glm::min
__device__ __forceinline__ float gmax(float a, float b) { return (a < b) ? b : a; }  // glm::max
__device__ __forceinline__ float dot3(P3 a, P3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ P3 normalize3(P3 v) {
    const float s = 1.0f / __builtin_sqrtf(dot3(v, v));
    return P3{v.x * s, v.y * s, v.z * s};
}
__device__ __forceinline__ P3 cross3(P3 a, P3 b) {
    return P3{a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y};
}

// Wall::end() (src/shapes/wall.hpp:16-31).
__device__ P3 wall_end(const FlatShape& s) {
    const P3 n = p3(s.planeNormal);
    P3 t1 = (fabsf(n.x) > fabsf(n.y)) ? normalize3(P3{-n.z, 0.f, n.x}) : normalize3(P3{0.f, -n.z, n.y});
    const P3 t2 = normalize3(cross3(n, t1));
    const P3 a = p3(s.wallStart);
    const float w = s.wallWidth, h = s.wallHeight;
    const P3 b{a.x + w * t1.x, a.y + w * t1.y, a.z + w * t1.z};
    return P3{b.x + h * t2.x, b.y + h * t2.y, b.z + h * t2.z};
}

struct Box {
    float lo[3], hi[3];
    __device__ void empty() {
        lo[0] = lo[1] = lo[2] = INFINITY;
        hi[0] = hi[1] = hi[2] = -INFINITY;
    }
    __device__ void grow(P3 p) {
        lo[0] = gmin(lo[0], p.x);
        lo[1] = gmin(lo[1], p.y);
        lo[2] = gmin(lo[2], p.z);
        hi[0] = gmax(hi[0], p.x);
        hi[1] = gmax(hi[1], p.y);
        hi[2] = gmax(hi[2], p.z);
    }
};

// BoundingBox::growToInclude(shape) from an empty box (src/BoundingBox.hpp:44-95).
__device__ Box shape_box(const FlatShape& s) {
    Box b;
    b.empty();
    if (s.type == RT_SPHERE) {
        const P3 c = p3(s.sphereCenter);
        const float r = s.sphereRadius;
        b.grow(P3{c.x + r, c.y + r, c.z + r});
        b.grow(P3{c.x - r, c.y - r, c.z - r});
    } else if (s.type == RT_WALL) {
        b.grow(p3(s.wallStart));
        b.grow(wall_end(s));
    } else if (s.type == RT_TRIANGLE) {
        if (isfinite(s.triP1.x) && isfinite(s.triP2.x) && isfinite(s.triP3.x)) {
            b.grow(p3(s.triP1));
            b.grow(p3(s.triP2));
            b.grow(p3(s.triP3));
        }
    }
    return b;
}

// The centre split() sorts by (src/main.cpp:1127-1140); planes keep (0,0,0).
__device__ P3 split_centre(const FlatShape& s) {
    if (s.type == RT_SPHERE) return p3(s.sphereCenter);
    if (s.type == RT_WALL) {
        const P3 a = p3(s.wallStart), e = wall_end(s);
        return P3{(a.x + e.x) * 0.5f, (a.y + e.y) * 0.5f, (a.z + e.z) * 0.5f};
    }
    if (s.type == RT_TRIANGLE) {
        const P3 a = p3(s.triP1), b = p3(s.triP2), c = p3(s.triP3);
        return P3{((a.x + b.x) + c.x) / 3.0f, ((a.y + b.y) + c.y) / 3.0f, ((a.z + b.z) + c.z) / 3.0f};
    }
    return P3{0.f, 0.f, 0.f};
}

// Order-preserving int image of a float (atomic min/max on the bounds).
__device__ __forceinline__ int ord(float f) {
    const int i = __float_as_int(f);
    return i >= 0 ? i : i ^ 0x7fffffff;
}
__device__ __forceinline__ float unord(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7fffffff); }

__global__ __launch_bounds__(kThreads) void k_lbvh_prep(const FlatShape* __restrict__ shapes, int n,
                                                         float4* __restrict__ boxes, float4* __restrict__ centres,
                                                         int* __restrict__ bounds) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    float c[3] = {0.f, 0.f, 0.f};
    bool ok = false;
    if (i < n) {
        const FlatShape s = shapes[i];
        const Box b = shape_box(s);
        boxes[2 * i] = make_float4(b.lo[0], b.lo[1], b.lo[2], 0.f);
        boxes[2 * i + 1] = make_float4(b.hi[0], b.hi[1], b.hi[2], 0.f);
        const P3 p = split_centre(s);
        c[0] = p.x;
        c[1] = p.y;
        c[2] = p.z;
        ok = isfinite(p.x) && isfinite(p.y) && isfinite(p.z);
        centres[i] = make_float4(p.x, p.y, p.z, ok ? 1.f : 0.f);
    }
    // wave reduction of the finite centres, then one atomic per wave and bound
    for (int a = 0; a < 3; ++a) {
        int lo = ok ? ord(c[a]) : 0x7fffffff, hi = ok ? ord(c[a]) : static_cast<int>(0x80000000);
        for (int off = 32; off > 0; off >>= 1) {
            lo = min(lo, __shfl_xor(lo, off));
            hi = max(hi, __shfl_xor(hi, off));
        }
        if ((threadIdx.x & 63) == 0) {
            atomicMin(&bounds[a], lo);
            atomicMax(&bounds[3 + a], hi);
        }
    }
}

__device__ __forceinline__ unsigned spread10(unsigned v) {
    v = (v | (v << 16)) & 0x030000ffu;
    v = (v | (v << 8)) & 0x0300f00fu;
    v = (v | (v << 4)) & 0x030c30c3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}

__global__ __launch_bounds__(kThreads) void k_lbvh_morton(const float4* __restrict__ centres, int n,
                                                           const int* __restrict__ bounds,
                                                           unsigned long long* __restrict__ keys) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 c = centres[i];
    unsigned q[3] = {0u, 0u, 0u};
    if (c.w != 0.f) {
        const float v[3] = {c.x, c.y, c.z};
        for (int a = 0; a < 3; ++a) {
            const float lo = unord(bounds[a]), hi = unord(bounds[3 + a]);
            const float ext = hi - lo;
            float u = ext > 0.f ? (v[a] - lo) / ext : 0.5f;
            u = fminf(fmaxf(u, 0.f), 1.f);
            q[a] = static_cast<unsigned>(fminf(u * 1024.f, 1023.f));
        }
    }
    const unsigned m = (spread10(q[0]) << 2) | (spread10(q[1]) << 1) | spread10(q[2]);
    keys[i] = (static_cast<unsigned long long>(m) << 32) | static_cast<unsigned>(i);
}

// Longest common prefix of keys i and j (-1 outside [0, n)); keys are unique.
__device__ __forceinline__ int delta(const unsigned long long* __restrict__ k, int n, int i, int j) {
    if (j < 0 || j >= n) return -1;
    return __clzll(k[i] ^ k[j]);
}

// Karras inner node i (0 = root) -> FlatNode index; leaf j -> j.
__device__ __forceinline__ int inner_index(int n, int i) { return (2 * n - 2) - i; }

__global__ __launch_bounds__(kThreads) void k_lbvh_inner(const unsigned long long* __restrict__ k, int n,
                                                          FlatNode* __restrict__ nodes, int* __restrict__ parent,
                                                          int* __restrict__ arrivals) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n - 1) return;
    const int d = (delta(k, n, i, i + 1) - delta(k, n, i, i - 1)) >= 0 ? 1 : -1;
    const int dmin = delta(k, n, i, i - d);
    int lmax = 2;
    while (delta(k, n, i, i + lmax * d) > dmin) lmax <<= 1;
    int l = 0;
    for (int t = lmax >> 1; t >= 1; t >>= 1)
        if (delta(k, n, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = delta(k, n, i, j);
    int s = 0;
    for (int t = (l + 1) >> 1;; t = (t + 1) >> 1) {
        if (delta(k, n, i, i + (s + t) * d) > dnode) s += t;
        if (t == 1) break;
    }
    const int g = i + s * d + min(d, 0);
    const int first = min(i, j), last = max(i, j);
    const int left = (first == g) ? g : inner_index(n, g);
    const int right = (last == g + 1) ? g + 1 : inner_index(n, g + 1);
    const int me = inner_index(n, i);
    FlatNode& nd = nodes[me];
    nd.leftChild = left;
    nd.rightChild = right;
    nd.startShapeIdx = first;       // its shapes are bvhIndices[first .. last]
    nd.numShapes = last - first + 1;
    nd.padding1 = 0.f;
    nd.padding2 = 0.f;
    parent[left] = me;
    parent[right] = me;
    arrivals[me] = 0;
    if (i == 0) parent[me] = -1;
}

__device__ __forceinline__ float ld(const float* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(kThreads) void k_lbvh_leaves(const unsigned long long* __restrict__ keys, int n,
                                                           const float4* __restrict__ boxes, FlatNode* nodes,
                                                           const int* __restrict__ parent, int* arrivals,
                                                           int* __restrict__ indices) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const int s = static_cast<int>(keys[j] & 0xffffffffull);
    indices[j] = s;
    const float4 lo = boxes[2 * s], hi = boxes[2 * s + 1];
    FlatNode& leaf = nodes[j];
    leaf.boundsMin = rt_vec3{lo.x, lo.y, lo.z};
    leaf.boundsMax = rt_vec3{hi.x, hi.y, hi.z};
    leaf.padding1 = 0.f;
    leaf.padding2 = 0.f;
    leaf.leftChild = -1;
    leaf.rightChild = -1;
    leaf.startShapeIdx = j;
    leaf.numShapes = 1;
    if (n == 1) return;
    // Bottom-up unions: the second arrival at a node has both children's boxes.
    int p = parent[j];
    while (p >= 0) {
        if (__hip_atomic_fetch_add(&arrivals[p], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
        FlatNode& nd = nodes[p];
        const FlatNode& a = nodes[nd.leftChild];
        const FlatNode& b = nodes[nd.rightChild];
        nd.boundsMin = rt_vec3{gmin(ld(&a.boundsMin.x), ld(&b.boundsMin.x)), gmin(ld(&a.boundsMin.y), ld(&b.boundsMin.y)),
                               gmin(ld(&a.boundsMin.z), ld(&b.boundsMin.z))};
        nd.boundsMax = rt_vec3{gmax(ld(&a.boundsMax.x), ld(&b.boundsMax.x)), gmax(ld(&a.boundsMax.y), ld(&b.boundsMax.y)),
                               gmax(ld(&a.boundsMax.z), ld(&b.boundsMax.z))};
        p = parent[p];
    }
}

}  // namespace

namespace rtl {

int lbvh_build(const FlatShape* shapes, int n, FlatNode* nodes, int* indices, void* stream_ptr, float* ms) {
    hipStream_t stream = static_cast<hipStream_t>(stream_ptr);
    if (ms) *ms = 0.f;
    if (n <= 0) return 0;
    const int N = 2 * n - 1;
    // scratch: boxes (2 float4/shape), centres (float4), keys in/out (u64), parent/arrivals (int/node), bounds
    size_t sort_bytes = 0;
    unsigned long long* knull = nullptr;
    if (rocprim::radix_sort_keys(nullptr, sort_bytes, knull, knull, static_cast<size_t>(n), 0, 62, stream) !=
        hipSuccess)
        return -1;
    const size_t bytes = 2 * sizeof(float4) * n + sizeof(float4) * n + 2 * sizeof(unsigned long long) * n +
                         2 * sizeof(int) * N + 8 * sizeof(int) + sort_bytes + 256 * 8;
    char* base = nullptr;
    if (hipMalloc(&base, bytes) != hipSuccess) return -2;
    size_t off = 0;
    auto take = [&](size_t b) {
        char* p = base + off;
        off += (b + 255) & ~static_cast<size_t>(255);
        return p;
    };
    float4* boxes = reinterpret_cast<float4*>(take(2 * sizeof(float4) * n));
    float4* centres = reinterpret_cast<float4*>(take(sizeof(float4) * n));
    unsigned long long* kin = reinterpret_cast<unsigned long long*>(take(sizeof(unsigned long long) * n));
    unsigned long long* kout = reinterpret_cast<unsigned long long*>(take(sizeof(unsigned long long) * n));
    int* parent = reinterpret_cast<int*>(take(sizeof(int) * N));
    int* arrivals = reinterpret_cast<int*>(take(sizeof(int) * N));
    int* bounds = reinterpret_cast<int*>(take(8 * sizeof(int)));
    void* sort_tmp = take(sort_bytes);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = 0;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) rc = -3;
    const int init[8] = {0x7fffffff, 0x7fffffff, 0x7fffffff, static_cast<int>(0x80000000), static_cast<int>(0x80000000),
                         static_cast<int>(0x80000000), 0, 0};
    if (rc == 0 && hipMemcpyAsync(bounds, init, sizeof init, hipMemcpyHostToDevice, stream) != hipSuccess) rc = -4;
    if (rc == 0) {
        const dim3 gs((n + kThreads - 1) / kThreads), gi((n - 1 + kThreads - 1) / kThreads);
        (void)hipEventRecord(e0, stream);
        hipLaunchKernelGGL(k_lbvh_prep, gs, dim3(kThreads), 0, stream, shapes, n, boxes, centres, bounds);
        hipLaunchKernelGGL(k_lbvh_morton, gs, dim3(kThreads), 0, stream, centres, n, bounds, kin);
        if (rocprim::radix_sort_keys(sort_tmp, sort_bytes, kin, kout, static_cast<size_t>(n), 0, 62, stream) !=
            hipSuccess)
            rc = -5;
        if (rc == 0 && n > 1)
            hipLaunchKernelGGL(k_lbvh_inner, gi, dim3(kThreads), 0, stream, kout, n, nodes, parent, arrivals);
        if (rc == 0)
            hipLaunchKernelGGL(k_lbvh_leaves, gs, dim3(kThreads), 0, stream, kout, n, boxes, nodes, parent, arrivals,
                               indices);
        (void)hipEventRecord(e1, stream);
        if (hipGetLastError() != hipSuccess) rc = -6;
        if (hipStreamSynchronize(stream) != hipSuccess) rc = -7;
        if (rc == 0 && ms) (void)hipEventElapsedTime(ms, e0, e1);
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipFree(base);
    return rc;
}

}  // namespace rtl

// rt_group.hip — one frame split over several GPUs by interleaved row stripes,
// gathered to rank 0 (include/rt_group.h).
//
// The reference's frame is one glDispatchCompute(W, H, 1) (src/main.cpp:352-354)
// whose invocations read no other pixel (gpu_shader.comp:434-623). The rows are
// dealt in periods of Q = share + P - 1 stripes: rank 0 renders the first `share`
// stripes of every period (one stripe of share*stripe rows), rank r >= 1 the
// stripe share - 1 + r (rt_group_set_root_share; share 1 = the plain interleave
// { y : (y / stripe) mod P == r }). Every rank renders through
// rt_dispatch_rows_ex into a compact packed-RGB buffer (alpha is always 1, so
// 12 B per pixel); rank 0 renders straight into its staging buffer, since its
// own rows never move. The fan-in is one grouped ncclSend/ncclRecv per frame
// (each peer's rows to rank 0 over its own xGMI link), or, in one process with
// repeated devices, peer copies into rank 0's staging. k_unstripe then scatters
// the slots back into image order in rank 0's pitched surface: one coalesced
// read and one streaming write per pixel (25 + 33 MB at 1080p, ~10 us).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/rt_api.h"
#include "../../include/rt_group.h"

namespace {

struct Member {
    int rank = 0, device = 0;
    rt_ctx* ctx = nullptr;
    hipStream_t stream = nullptr;
    float* buf = nullptr;  // ranks >= 1: compact stripes, rows x W packed RGB32F (12 B per pixel)
    size_t buf_cap = 0;    // bytes
    ncclComm_t comm = nullptr;
    hipEvent_t rendered = nullptr;  // copy transport: this member's stripes are in buf
};

// The rows of rank `rank` (stripe `s`, P ranks, rank 0's share k): rank 0 owns
// rows [0, k*s) of every period of (k + P - 1) * s rows, rank r >= 1 the s rows
// from (k - 1 + r) * s.
struct Rows {
    int y0, stripe, period, rows;
};
Rows rank_rows(int height, int nranks, int s, int k, int rank) {
    Rows o;
    o.period = (k + nranks - 1) * s;
    o.y0 = rank == 0 ? 0 : (k - 1 + rank) * s;
    o.stripe = rank == 0 ? k * s : s;
    const int full = height / o.period, rem = height % o.period;
    o.rows = full * o.stripe + std::max(0, std::min(o.stripe, rem - o.y0));
    return o;
}

typedef float f4v __attribute__((ext_vector_type(4)));

// out[y][x]: stripe band = y / s sits at position c = band % Q of its period
// (Q = k + P - 1). c < k: rank 0's slot (offset 0), compact row (band / Q) * k * s
// + c * s + y % s; otherwise rank c - k + 1's slot, at rows0 + (c - k) * rows1
// rows from the start, compact row (band / Q) * s + y % s. The slots hold packed
// RGB (rt_dispatch_rows_ex RGB32F), the image RGBA with alpha 1.
__global__ __launch_bounds__(256) void k_unstripe(const float* __restrict__ staging, int rows0, int rows1, int width,
                                                   int s, int k, int q, f4v* __restrict__ img, size_t pitch_f4) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    if (x >= width) return;
    const int band = y / s, c = band % q, cyc = band / q;
    const int r = c < k ? cyc * k * s + c * s + (y - band * s) : rows0 + (c - k) * rows1 + cyc * s + (y - band * s);
    const float* p = staging + 3 * (static_cast<size_t>(r) * width + x);
    const f4v v = {__builtin_nontemporal_load(p), __builtin_nontemporal_load(p + 1), __builtin_nontemporal_load(p + 2),
                   1.0f};
    __builtin_nontemporal_store(v, &img[static_cast<size_t>(y) * pitch_f4 + x]);
}

}  // namespace

struct rt_group {
    int nranks = 0;
    int transport = RT_GATHER_COPY;
    std::vector<Member> m;
    int root = -1;  // local index of rank 0, -1 if another process holds it
    int share = 1;  // rank 0's stripes per period (rt_group_set_root_share)
    float* staging = nullptr;  // root: rank 0's rows, then P - 1 slots of rows1 x W packed RGB
    size_t staging_cap = 0;
    float* img = nullptr;      // root: the gathered frame
    size_t img_pitch = 0;
    int img_w = 0, img_h = 0;
    hipEvent_t gathered = nullptr;  // copy transport: root has read every member's buf
    bool gathered_valid = false;
};

namespace {

#define G_HIP(x)                                          \
    do {                                                  \
        if ((x) != hipSuccess) return RT_ERR_DEVICE;      \
    } while (0)
#define G_NCCL(x)                                         \
    do {                                                  \
        if ((x) != ncclSuccess) return RT_ERR_COMM;       \
    } while (0)

int add_member(rt_group* g, int rank, int device) {
    Member mb;
    mb.rank = rank;
    mb.device = device;
    int rc = rt_create(&mb.ctx, device);
    if (rc != RT_OK) return rc;
    g->m.push_back(mb);  // owned from here (rt_group_destroy frees it)
    Member& b = g->m.back();
    G_HIP(hipSetDevice(device));
    G_HIP(hipStreamCreateWithFlags(&b.stream, hipStreamNonBlocking));
    G_HIP(hipEventCreateWithFlags(&b.rendered, hipEventDisableTiming));
    return rt_set_stream(b.ctx, b.stream);
}

int finish_create(rt_group* g) {
    for (size_t k = 0; k < g->m.size(); ++k)
        if (g->m[k].rank == 0) g->root = static_cast<int>(k);
    if (g->root >= 0) {
        G_HIP(hipSetDevice(g->m[g->root].device));
        G_HIP(hipEventCreateWithFlags(&g->gathered, hipEventDisableTiming));
    }
    return RT_OK;
}

template <class T>
int grow(T*& p, size_t& cap, size_t bytes) {
    if (p && cap >= bytes) return RT_OK;
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(&p, bytes) != hipSuccess) return RT_ERR_NO_MEMORY;
    cap = bytes;
    return RT_OK;
}

}  // namespace

extern "C" {

int rt_group_unique_id(void* id, size_t cap) {
    static_assert(sizeof(ncclUniqueId) == RT_GROUP_ID_BYTES, "ncclUniqueId size");
    if (!id || cap < sizeof(ncclUniqueId)) return RT_ERR_INVALID;
    ncclUniqueId u;
    G_NCCL(ncclGetUniqueId(&u));
    std::memcpy(id, &u, sizeof u);
    return RT_OK;
}

int rt_group_create(rt_group** out, const int* devices, int n, int transport) {
    if (!out || !devices || n < 1 || transport < RT_GATHER_AUTO || transport > RT_GATHER_COPY) return RT_ERR_INVALID;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess) return RT_ERR_NO_DEVICE;
    bool distinct = true;
    for (int i = 0; i < n; ++i) {
        if (devices[i] < 0 || devices[i] >= ndev) return RT_ERR_NO_DEVICE;
        for (int j = 0; j < i; ++j) distinct = distinct && devices[i] != devices[j];
    }
    if (transport == RT_GATHER_RCCL && !distinct) return RT_ERR_COMM;  // RCCL: one rank per device
    rt_group* g = new (std::nothrow) rt_group();
    if (!g) return RT_ERR_NO_MEMORY;
    g->nranks = n;
    g->transport = (transport == RT_GATHER_RCCL || (transport == RT_GATHER_AUTO && distinct && n > 1))
                       ? RT_GATHER_RCCL
                       : RT_GATHER_COPY;
    int rc = RT_OK;
    for (int k = 0; k < n && rc == RT_OK; ++k) rc = add_member(g, k, devices[k]);
    if (rc == RT_OK && g->transport == RT_GATHER_RCCL) {
        std::vector<ncclComm_t> comms(n);
        if (ncclCommInitAll(comms.data(), n, devices) != ncclSuccess) rc = RT_ERR_COMM;
        else
            for (int k = 0; k < n; ++k) g->m[k].comm = comms[k];
    }
    if (rc == RT_OK) rc = finish_create(g);
    if (rc != RT_OK) {
        rt_group_destroy(g);
        return rc;
    }
    *out = g;
    return RT_OK;
}

int rt_group_create_rank(rt_group** out, const void* id, int nranks, int rank, int device) {
    if (!out || !id || nranks < 1 || rank < 0 || rank >= nranks) return RT_ERR_INVALID;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return RT_ERR_NO_DEVICE;
    rt_group* g = new (std::nothrow) rt_group();
    if (!g) return RT_ERR_NO_MEMORY;
    g->nranks = nranks;
    g->transport = RT_GATHER_RCCL;
    int rc = add_member(g, rank, device);
    if (rc == RT_OK) {
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof u);
        if (hipSetDevice(device) != hipSuccess) rc = RT_ERR_DEVICE;
        else if (ncclCommInitRank(&g->m[0].comm, nranks, u, rank) != ncclSuccess) rc = RT_ERR_COMM;
    }
    if (rc == RT_OK) rc = finish_create(g);
    if (rc != RT_OK) {
        rt_group_destroy(g);
        return rc;
    }
    *out = g;
    return RT_OK;
}

int rt_group_destroy(rt_group* g) {
    if (!g) return RT_ERR_INVALID;
    for (Member& b : g->m) {
        hipSetDevice(b.device);
        if (b.stream) hipStreamSynchronize(b.stream);
    }
    for (Member& b : g->m) {
        hipSetDevice(b.device);
        if (b.comm) ncclCommDestroy(b.comm);
        if (b.ctx) rt_destroy(b.ctx);  // before its stream goes: it is ordered on it
        if (b.buf) hipFree(b.buf);
        if (b.rendered) hipEventDestroy(b.rendered);
        if (b.stream) hipStreamDestroy(b.stream);
    }
    if (g->root >= 0) {
        hipSetDevice(g->m[g->root].device);
        hipFree(g->staging);
        hipFree(g->img);
        if (g->gathered) hipEventDestroy(g->gathered);
    }
    delete g;
    return RT_OK;
}

int rt_group_info(rt_group* g, int* nranks, int* nlocal, int* transport) {
    if (!g) return RT_ERR_INVALID;
    if (nranks) *nranks = g->nranks;
    if (nlocal) *nlocal = static_cast<int>(g->m.size());
    if (transport) *transport = g->transport;
    return RT_OK;
}

int rt_group_member(rt_group* g, int k, rt_ctx** ctx) {
    if (!g || !ctx || k < 0 || k >= static_cast<int>(g->m.size())) return RT_ERR_INVALID;
    *ctx = g->m[k].ctx;
    return RT_OK;
}

int rt_group_upload_scene(rt_group* g, const FlatShape* shapes, int S, const FlatNode* nodes, int N, const int* idx,
                          int I) {
    if (!g) return RT_ERR_INVALID;
    for (Member& b : g->m) {
        const int rc = rt_upload_scene(b.ctx, shapes, S, nodes, N, idx, I);
        if (rc != RT_OK) return rc;
    }
    return RT_OK;
}

int rt_group_set_camera(rt_group* g, const FlatCamera* cam) {
    if (!g) return RT_ERR_INVALID;
    for (Member& b : g->m) {
        const int rc = rt_set_camera(b.ctx, cam);
        if (rc != RT_OK) return rc;
    }
    return RT_OK;
}

int rt_group_set_light(rt_group* g, const FlatLight* l) {
    if (!g) return RT_ERR_INVALID;
    for (Member& b : g->m) {
        const int rc = rt_set_light(b.ctx, l);
        if (rc != RT_OK) return rc;
    }
    return RT_OK;
}

int rt_group_set_params(rt_group* g, const rt_params* p) {
    if (!g) return RT_ERR_INVALID;
    for (Member& b : g->m) {
        const int rc = rt_set_params(b.ctx, p);
        if (rc != RT_OK) return rc;
    }
    return RT_OK;
}

int rt_group_dispatch(rt_group* g, int width, int height, int stripe) {
    if (!g || width <= 0 || height <= 0 || stripe <= 0 || height > 65535 ||
        stripe > 65535 / (g->share + g->nranks - 1))
        return RT_ERR_INVALID;
    const int P = g->nranks, k = g->share;
    const size_t row_b = static_cast<size_t>(width) * 12;  // packed RGB32F
    const int rows0 = rank_rows(height, P, stripe, k, 0).rows;
    const int rows1 = P > 1 ? rank_rows(height, P, stripe, k, 1).rows : 0;  // the most among ranks >= 1
    const size_t slot = std::max<size_t>(1, static_cast<size_t>(rows1) * row_b);
    const size_t stage = static_cast<size_t>(rows0) * row_b + static_cast<size_t>(P - 1) * rows1 * row_b;
    auto slot_ptr = [&](int rank) {  // rank's rows in the staging buffer
        return reinterpret_cast<char*>(g->staging) +
               (rank == 0 ? 0 : static_cast<size_t>(rows0) * row_b + static_cast<size_t>(rank - 1) * rows1 * row_b);
    };
    // (Re)size the buffers; a resize waits for the frames that still use them.
    bool resize = false;
    for (Member& b : g->m) resize = resize || (b.rank != 0 && b.buf_cap < slot);
    if (g->root >= 0)
        resize = resize || g->staging_cap < stage || g->img_w != width || g->img_h != height;
    if (resize) {
        for (Member& b : g->m) {
            G_HIP(hipSetDevice(b.device));
            G_HIP(hipStreamSynchronize(b.stream));
            if (b.rank == 0) continue;
            const int rc = grow(b.buf, b.buf_cap, slot);
            if (rc != RT_OK) return rc;
        }
        if (g->root >= 0) {
            Member& r = g->m[g->root];
            G_HIP(hipSetDevice(r.device));
            int rc = grow(g->staging, g->staging_cap, std::max<size_t>(stage, 16));
            if (rc != RT_OK) return rc;
            if (g->img_w != width || g->img_h != height) {
                hipFree(g->img);
                g->img = nullptr;
                g->img_w = g->img_h = 0;
                size_t pitch = 0;
                if (hipMallocPitch(reinterpret_cast<void**>(&g->img), &pitch, static_cast<size_t>(width) * 16,
                                   height) != hipSuccess)
                    return RT_ERR_NO_MEMORY;
                g->img_pitch = pitch;
                g->img_w = width;
                g->img_h = height;
            }
        }
    }
    // 1. every local rank renders its stripes on its own stream (rank 0 straight into
    //    its staging rows; the others into buf, sent after the render)
    for (Member& b : g->m) {
        G_HIP(hipSetDevice(b.device));
        if (g->transport == RT_GATHER_COPY && g->gathered_valid && b.rank != 0)
            G_HIP(hipStreamWaitEvent(b.stream, g->gathered, 0));  // root has read the previous frame's buf
        const Rows w = rank_rows(height, P, stripe, k, b.rank);
        if (w.rows == 0) continue;
        float* dst = b.rank == 0 ? g->staging : b.buf;
        const int rc = rt_dispatch_rows_ex(b.ctx, width, height, w.y0, w.stripe, w.period, w.rows, dst, row_b,
                                           RT_FORMAT_RGB32F);
        if (rc != RT_OK) return rc;
    }
    // 2. fan-in to rank 0's staging: rank r's rows to slot r
    if (g->transport == RT_GATHER_RCCL && P > 1) {
        G_NCCL(ncclGroupStart());
        for (Member& b : g->m) {
            ncclResult_t res = ncclSuccess;
            if (b.rank == 0) {
                for (int r = 1; r < P && res == ncclSuccess; ++r) {
                    const size_t n = static_cast<size_t>(rank_rows(height, P, stripe, k, r).rows) * width * 3;
                    if (n) res = ncclRecv(slot_ptr(r), n, ncclFloat32, r, b.comm, b.stream);
                }
            } else {
                const size_t n = static_cast<size_t>(rank_rows(height, P, stripe, k, b.rank).rows) * width * 3;
                if (n) res = ncclSend(b.buf, n, ncclFloat32, 0, b.comm, b.stream);
            }
            if (res != ncclSuccess) {
                ncclGroupEnd();
                return RT_ERR_COMM;
            }
        }
        G_NCCL(ncclGroupEnd());
    } else if (g->transport == RT_GATHER_COPY) {
        Member& r = g->m[g->root];
        for (Member& b : g->m) {
            if (b.rank == 0) continue;
            G_HIP(hipSetDevice(b.device));
            G_HIP(hipEventRecord(b.rendered, b.stream));
        }
        G_HIP(hipSetDevice(r.device));
        for (Member& b : g->m) {
            if (b.rank == 0) continue;
            const size_t n = static_cast<size_t>(rank_rows(height, P, stripe, k, b.rank).rows) * row_b;
            G_HIP(hipStreamWaitEvent(r.stream, b.rendered, 0));
            if (n) G_HIP(hipMemcpyPeerAsync(slot_ptr(b.rank), r.device, b.buf, b.device, n, r.stream));
        }
        G_HIP(hipEventRecord(g->gathered, r.stream));
        g->gathered_valid = true;
    }
    // 3. rank 0: stripes back into image order
    if (g->root >= 0) {
        Member& r = g->m[g->root];
        G_HIP(hipSetDevice(r.device));
        hipLaunchKernelGGL(k_unstripe, dim3((width + 255) / 256, height), dim3(256), 0, r.stream, g->staging, rows0,
                           rows1, width, stripe, k, k + P - 1, reinterpret_cast<f4v*>(g->img), g->img_pitch / 16);
        G_HIP(hipGetLastError());
    }
    return RT_OK;
}

int rt_group_set_root_share(rt_group* g, int share) {
    if (!g || share < 1 || share > 64) return RT_ERR_INVALID;
    g->share = share;
    return RT_OK;
}

int rt_group_collect_stats(rt_group* g, int width, int height, int stripe, rt_stats* out) {
    if (!g || !out || width <= 0 || height <= 0 || stripe <= 0 || stripe > 65535 / (g->share + g->nranks - 1))
        return RT_ERR_INVALID;
    std::memset(out, 0, sizeof *out);
    for (Member& b : g->m) {
        const Rows w = rank_rows(height, g->nranks, stripe, g->share, b.rank);
        if (w.rows == 0) continue;
        rt_stats st;
        const int rc = rt_collect_stats_ex(b.ctx, width, height, w.y0, w.stripe, w.period, w.rows, &st);
        if (rc != RT_OK) return rc;
        uint64_t* o = reinterpret_cast<uint64_t*>(out);
        const uint64_t* a = reinterpret_cast<const uint64_t*>(&st);
        for (size_t i = 0; i < sizeof st / sizeof(uint64_t); ++i) o[i] += a[i];
    }
    return RT_OK;
}

int rt_group_sync(rt_group* g) {
    if (!g) return RT_ERR_INVALID;
    for (Member& b : g->m) {
        G_HIP(hipSetDevice(b.device));
        G_HIP(hipStreamSynchronize(b.stream));
    }
    return RT_OK;
}

int rt_group_read_image(rt_group* g, float* dst, size_t pitch, int width, int height) {
    if (!g || g->root < 0 || !dst || !g->img || width != g->img_w || height != g->img_h ||
        pitch < static_cast<size_t>(width) * 16)
        return RT_ERR_INVALID;
    Member& r = g->m[g->root];
    G_HIP(hipSetDevice(r.device));
    G_HIP(hipMemcpy2DAsync(dst, pitch, g->img, g->img_pitch, static_cast<size_t>(width) * 16, height,
                           hipMemcpyDeviceToHost, r.stream));
    G_HIP(hipStreamSynchronize(r.stream));
    return RT_OK;
}

int rt_group_device_image(rt_group* g, void** p, size_t* pitch) {
    if (!g || g->root < 0 || !p || !pitch || !g->img) return RT_ERR_INVALID;
    *p = g->img;
    *pitch = g->img_pitch;
    return RT_OK;
}

}  // extern "C"

// rt_group.hip — one frame split over several GPUs by interleaved row stripes,
// gathered to rank 0 (include/rt_group.h).
//
// The reference's frame is one glDispatchCompute(W, H, 1) (src/main.cpp:352-354)
// whose invocations read no other pixel (gpu_shader.comp:434-623). Rank r of P
// renders rows { y : (y / stripe) mod P == r } through rt_dispatch_rows into a
// compact [rows_max][W] packed-RGB buffer on its own stream (alpha is always 1,
// so 12 B per pixel). The fan-in is one ncclGather per frame (every rank sends
// rows_max*W*12 bytes; RCCL moves them
// over xGMI, each peer on its own link), or, in one process with repeated
// devices, peer copies into rank 0's staging. k_unstripe then scatters the
// P slots back into image order in rank 0's pitched surface: one coalesced
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
    float* buf = nullptr;  // compact stripes, rows_max x W packed RGB32F (12 B per pixel)
    size_t buf_cap = 0;    // bytes
    ncclComm_t comm = nullptr;
    hipEvent_t rendered = nullptr;  // copy transport: this member's stripes are in buf
};

// Image rows owned by `rank` (the rt_dispatch_rows stripe mapping).
int stripe_rows(int height, int nranks, int stripe, int rank) {
    const int full = height / (stripe * nranks), rem = height % (stripe * nranks);
    return full * stripe + std::max(0, std::min(stripe, rem - rank * stripe));
}

typedef float f4v __attribute__((ext_vector_type(4)));

// out[y][x] = slot k = (y / stripe) % P, its compact row (y / stripe / P) * stripe + y % stripe;
// the slots hold packed RGB (rt_dispatch_rows_fmt RGB32F), the image RGBA with alpha 1.
__global__ __launch_bounds__(256) void k_unstripe(const float* __restrict__ staging, int rows_max, int width,
                                                   int stripe, int nranks, f4v* __restrict__ img, size_t pitch_f4) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    if (x >= width) return;
    const int band = y / stripe;
    const int k = band % nranks;
    const int r = (band / nranks) * stripe + (y - band * stripe);
    const float* p = staging + 3 * ((static_cast<size_t>(k) * rows_max + r) * width + x);
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
    float* staging = nullptr;  // root: P slots of rows_max x W float4
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
    if (!g || width <= 0 || height <= 0 || stripe <= 0 || height > 65535) return RT_ERR_INVALID;
    const int P = g->nranks;
    const int rows_max = stripe_rows(height, P, stripe, 0);  // rank 0 owns the most rows
    const size_t slot = static_cast<size_t>(rows_max) * width * 12;  // packed RGB32F
    // (Re)size the buffers; a resize waits for the frames that still use them.
    bool resize = false;
    for (Member& b : g->m) resize = resize || b.buf_cap < slot;
    if (g->root >= 0)
        resize = resize || g->staging_cap < slot * P || g->img_w != width || g->img_h != height;
    if (resize) {
        for (Member& b : g->m) {
            G_HIP(hipSetDevice(b.device));
            G_HIP(hipStreamSynchronize(b.stream));
            const int rc = grow(b.buf, b.buf_cap, slot);
            if (rc != RT_OK) return rc;
        }
        if (g->root >= 0) {
            Member& r = g->m[g->root];
            G_HIP(hipSetDevice(r.device));
            int rc = grow(g->staging, g->staging_cap, slot * P);
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
    // 1. every local rank renders its stripes (its own stream; RCCL sends after it)
    for (Member& b : g->m) {
        G_HIP(hipSetDevice(b.device));
        if (g->transport == RT_GATHER_COPY && g->gathered_valid)
            G_HIP(hipStreamWaitEvent(b.stream, g->gathered, 0));  // root has read the previous frame's buf
        const int rows = stripe_rows(height, P, stripe, b.rank);
        const int rc = rt_dispatch_rows_fmt(b.ctx, width, height, b.rank * stripe, stripe, P, rows, b.buf,
                                            static_cast<size_t>(width) * 12, RT_FORMAT_RGB32F);
        if (rc != RT_OK) return rc;
    }
    // 2. fan-in to rank 0's staging, slot k = rank k
    if (g->transport == RT_GATHER_RCCL) {
        const size_t count = static_cast<size_t>(rows_max) * width * 3;
        G_NCCL(ncclGroupStart());
        for (Member& b : g->m) {
            // recvbuff is only read at the root; the others pass their own buffer (never null)
            const ncclResult_t r = ncclGather(b.buf, b.rank == 0 ? g->staging : b.buf, count, ncclFloat32, 0,
                                              b.comm, b.stream);
            if (r != ncclSuccess) {
                ncclGroupEnd();
                return RT_ERR_COMM;
            }
        }
        G_NCCL(ncclGroupEnd());
    } else {
        Member& r = g->m[g->root];
        for (Member& b : g->m) {
            G_HIP(hipSetDevice(b.device));
            G_HIP(hipEventRecord(b.rendered, b.stream));
        }
        G_HIP(hipSetDevice(r.device));
        for (Member& b : g->m) {
            G_HIP(hipStreamWaitEvent(r.stream, b.rendered, 0));
            G_HIP(hipMemcpyPeerAsync(reinterpret_cast<char*>(g->staging) + slot * b.rank, r.device, b.buf, b.device,
                                     slot, r.stream));
        }
        G_HIP(hipEventRecord(g->gathered, r.stream));
        g->gathered_valid = true;
    }
    // 3. rank 0: stripes back into image order
    if (g->root >= 0) {
        Member& r = g->m[g->root];
        G_HIP(hipSetDevice(r.device));
        hipLaunchKernelGGL(k_unstripe, dim3((width + 255) / 256, height), dim3(256), 0, r.stream,
                           g->staging, rows_max, width, stripe, P,
                           reinterpret_cast<f4v*>(g->img), g->img_pitch / 16);
        G_HIP(hipGetLastError());
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

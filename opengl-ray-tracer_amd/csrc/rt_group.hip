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
// 12 B per pixel), except rank 0, which renders its stripes straight into the
// frame at their image rows (RT_FORMAT_RGBA32F_IMAGE): its rows never move. The
// fan-in is one grouped ncclSend/ncclRecv per frame (each peer's rows to rank
// 0's staging over its own xGMI link), or, in one process with repeated
// devices, peer copies into rank 0's staging. k_unstripe then scatters the
// peers' rows into image order in rank 0's pitched surface: one coalesced read
// and one streaming write per pixel of (P - 1) / (share + P - 1) of the frame.
// With one rank there is no fan-in and no unstripe: the group's frame is the
// single-GPU frame.
//
// Frames in flight (rt_group_set_frames): every member holds F slots -- a
// context, a render stream and the frame's buffers -- and ONE communicator with
// ONE fan-in stream. Frame f renders in slot f mod F; its fan-in is queued on
// the fan-in stream behind the slot's render (an event), so frame f + 1 renders
// while frame f crosses the links, and every rank posts its send/recv in the
// same frame order on one stream of one communicator: no two communicators ever
// wait on each other. rank 0 unstripes each slot into that slot's own surface.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/rt_api.h"
#include "../../include/rt_group.h"
#include "group_wait.h"
#include "sky_rows.h"
#include "rt_internal.h"

namespace {

constexpr int kMaxFrames = 16;   // rt_group_set_frames
constexpr int kPhaseRing = 64;   // frames whose phase events are kept before they are read

struct Slot {
    rt_ctx* ctx = nullptr;
    hipStream_t stream = nullptr;  // this slot's render (and, on rank 0, unstripe) stream
    float* buf = nullptr;          // ranks >= 1: compact stripes, rows x W packed RGB32F (12 B per pixel)
    size_t buf_cap = 0;            // bytes
    float* staging = nullptr;      // rank 0: P - 1 slots of rows1 x W packed RGB, one per peer
    size_t staging_cap = 0;
    float* img = nullptr;          // rank 0: this slot's gathered frame (RGBA32F, pitched)
    size_t img_pitch = 0;
    int img_w = 0, img_h = 0;
    hipEvent_t rendered = nullptr;  // this member's stripes are written
    hipEvent_t fanned = nullptr;    // the fan-in of the slot's frame is done (sent / received / copied)
    hipEvent_t released = nullptr;  // the slot's buffers may be written again
    hipEvent_t sync_ev = nullptr;   // recorded behind the stream's work by a bounded wait
    bool dirty = false;             // work was queued on `stream` since sync_ev was last recorded
    bool used = false;              // `released` / `fanned` have been recorded
};

struct Member {
    int rank = 0, device = 0;
    std::vector<Slot> slot;
    hipStream_t cstream = nullptr;  // fan-in stream: every frame's send/recv (or copies) in frame order
    hipEvent_t csync_ev = nullptr;  // recorded behind cstream's work by a bounded wait
    bool cdirty = false;            // work was queued on cstream since csync_ev was last recorded
    ncclComm_t comm = nullptr;
};

// Device-time events of one frame of the timed member (rt_group_phase_times).
struct PhaseRec {
    hipEvent_t ev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};  // render 0/1, fan-in 0/1, unstripe 0/1
    bool pending = false, has_fan = false, has_unstripe = false;
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

// The peers' rows into image order. Staging holds P - 1 slots of rows1 packed-RGB
// rows (rt_dispatch_rows_ex RGB32F), one per rank r >= 1 in rank order; compact
// row cr of rank r is image row (k - 1 + r) * s + (cr / s) * (k + P - 1) * s + cr % s
// (rank_rows). Rows past a rank's count map to y >= height and are skipped. One
// coalesced read and one streaming RGBA store (alpha 1) per pixel. Rows outside
// [yb0, yb1) were not sent (sky_rows.h): they are the background of their row,
// written here with the shader's own float operations (gpu_shader.comp:436,
// mix = x + a (y - x); rt_kernels.hip background()).
__global__ __launch_bounds__(256) void k_unstripe(const float* __restrict__ staging, int rows1, int width, int height,
                                                   int s, int k, int P, f4v* __restrict__ img, size_t pitch_f4,
                                                   int yb0, int yb1, float resY) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int by = blockIdx.y;  // (rank - 1) * rows1 + compact row
    if (x >= width) return;
    const int rank = 1 + by / rows1, cr = by - (rank - 1) * rows1;
    const int y = (k - 1 + rank) * s + (cr / s) * (k + P - 1) * s + cr % s;
    if (y >= height) return;
    f4v v;
    if (y >= yb0 && y < yb1) {
        const float* p = staging + 3 * (static_cast<size_t>(by) * width + x);
        v = f4v{__builtin_nontemporal_load(p), __builtin_nontemporal_load(p + 1), __builtin_nontemporal_load(p + 2),
                1.0f};
    } else {
        const float a = static_cast<float>(y) / resY;
        v = f4v{0.05f + a * (0.5f - 0.05f), 0.07f + a * (0.7f - 0.07f), 0.1f + a * (1.0f - 0.1f), 1.0f};
    }
    __builtin_nontemporal_store(v, &img[static_cast<size_t>(y) * pitch_f4 + x]);
}

// The rank's rows (rank_rows) that lie above image row y: its compact rows below y.
int rows_below(int y0, int stripe, int period, int rows, int y) {
    if (y <= y0) return 0;
    const int t = y - y0;
    return std::min(rows, (t / period) * stripe + std::min(t % period, stripe));
}

}  // namespace

struct rt_group {
    int nranks = 0;
    int transport = RT_GATHER_COPY;
    std::vector<Member> m;
    int root = -1;     // local index of rank 0, -1 if another process holds it
    int share = 1;     // rank 0's stripes per period (rt_group_set_root_share)
    int frames = 1;    // slots per member (rt_group_set_frames)
    long long next = 0;  // frames dispatched
    int last_slot = -1;  // slot of the last dispatched frame
    bool have_scene = false;
    bool broken = false;        // an RCCL group after an abort: every call fails
    // sky rows (sky_rows.h): the frame's camera, parameters and root box as set on every rank
    FlatCamera cam{};
    rt_params params{};
    float root_lo[3] = {0, 0, 0}, root_hi[3] = {0, 0, 0};
    bool have_cam = false, have_params = false, have_root = false;
    bool sky_rows = true;       // rt_group_set_sky_rows
    int band_y0 = 0, band_y1 = 0;  // the last dispatch's band (rt_group_sky_band)
    double timeout_ms = 60000;  // rt_group_set_timeout
    bool phase_timing = true;   // rt_group_set_phase_timing
    // phase times of member `tm` (rank 0 when local, else the first member)
    int tm = 0;
    std::vector<PhaseRec> ring;
    int ring_pos = 0;
    double sum[4] = {0, 0, 0, 0};  // render, fan-in, unstripe, frame (ms)
    int nsum[4] = {0, 0, 0, 0};
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
#define G_TRY(x)                             \
    do {                                     \
        const int rc__ = (x);                \
        if (rc__ != RT_OK) return rc__;      \
    } while (0)

int add_slot(Member& b) {
    b.slot.emplace_back();
    Slot& s = b.slot.back();
    G_HIP(hipSetDevice(b.device));
    G_HIP(rtx::make_stream(&s.stream, true));  // a hardware queue per slot (rt_internal.h)
    G_HIP(hipEventCreateWithFlags(&s.rendered, hipEventDisableTiming));
    G_HIP(hipEventCreateWithFlags(&s.fanned, hipEventDisableTiming));
    G_HIP(hipEventCreateWithFlags(&s.released, hipEventDisableTiming));
    G_HIP(hipEventCreateWithFlags(&s.sync_ev, hipEventDisableTiming));
    return rtx::create_ctx(&s.ctx, b.device, s.stream);  // straight on the slot's stream (rt_internal.h)
}

int add_member(rt_group* g, int rank, int device) {
    Member mb;
    mb.rank = rank;
    mb.device = device;
    g->m.push_back(mb);  // owned from here (rt_group_destroy frees it)
    Member& b = g->m.back();
    G_HIP(hipSetDevice(device));
    G_HIP(rtx::make_stream(&b.cstream, true));
    G_HIP(hipEventCreateWithFlags(&b.csync_ev, hipEventDisableTiming));
    return add_slot(b);
}

int finish_create(rt_group* g) {
    for (size_t k = 0; k < g->m.size(); ++k)
        if (g->m[k].rank == 0) g->root = static_cast<int>(k);
    g->tm = g->root >= 0 ? g->root : 0;
    G_HIP(hipSetDevice(g->m[g->tm].device));
    g->ring.resize(kPhaseRing);
    for (PhaseRec& p : g->ring)
        for (hipEvent_t& e : p.ev) G_HIP(hipEventCreate(&e));
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

// Every communicator aborted: its pending kernels return, and the group is unusable
// (a peer may have posted a send or receive this process will never match).
void abort_comms(rt_group* g) {
    for (Member& b : g->m)
        if (b.comm) {
            hipSetDevice(b.device);
            ncclCommAbort(b.comm);
            b.comm = nullptr;
        }
    if (g->transport == RT_GATHER_RCCL) g->broken = true;
}

// An error after this process may have left its peers waiting on a fan-in.
int fail(rt_group* g, int rc) {
    if (g->transport == RT_GATHER_RCCL && g->nranks > 1) abort_comms(g);
    return rc;
}

// Outstanding work on any of the group's streams: 1 yes, 0 none, -1 device error.
// Polls the events mark_streams recorded behind each stream's work (an event query
// sees a kernel end ~1.5 us sooner than hipStreamQuery, tools/native/wait_probe.hip);
// the last dispatched frame's slot first: while it runs one query answers.
int pending(rt_group* g) {
    auto q = [](hipEvent_t e) {
        if (!e) return 0;
        const hipError_t r = hipEventQuery(e);
        return r == hipSuccess ? 0 : (r == hipErrorNotReady ? 1 : -1);
    };
    if (g->last_slot >= 0)
        for (Member& b : g->m)
            if (g->last_slot < static_cast<int>(b.slot.size())) {
                const int r = q(b.slot[g->last_slot].sync_ev);
                if (r) return r;
            }
    for (Member& b : g->m) {
        int r = q(b.csync_ev);
        if (r) return r;
        for (Slot& s : b.slot)
            if ((r = q(s.sync_ev))) return r;
    }
    return 0;
}

// Records the sync event of every stream that was given work since its last record,
// behind that work (before a bounded wait). A waited frame marks one or two streams:
// each record is a marker packet on the stream (every stream marked each time cost a
// 1-rank group's waited frame 22 us, r04o).
int mark_streams(rt_group* g) {
    for (Member& b : g->m) {
        if (hipSetDevice(b.device) != hipSuccess) return RT_ERR_DEVICE;
        if (b.cdirty && b.cstream && b.csync_ev) {
            if (hipEventRecord(b.csync_ev, b.cstream) != hipSuccess) return RT_ERR_DEVICE;
            b.cdirty = false;
        }
        for (Slot& s : b.slot)
            if (s.dirty && s.stream && s.sync_ev) {
                if (hipEventRecord(s.sync_ev, s.stream) != hipSuccess) return RT_ERR_DEVICE;
                s.dirty = false;
            }
    }
    return RT_OK;
}

void mark_all_dirty(rt_group* g) {
    for (Member& b : g->m) {
        b.cdirty = true;
        for (Slot& s : b.slot) s.dirty = true;
    }
}

bool comm_error(rt_group* g) {
    for (Member& b : g->m) {
        if (!b.comm) continue;
        ncclResult_t st = ncclSuccess;
        if (ncclCommGetAsyncError(b.comm, &st) != ncclSuccess) return true;
        if (st != ncclSuccess && st != ncclInProgress) return true;
    }
    return false;
}

// The bounded wait (group_wait.h); on a timeout or an RCCL error the communicators
// are aborted.
int wait_all(rt_group* g) {
    if (mark_streams(g) != RT_OK) return fail(g, RT_ERR_DEVICE);
    const rtg::WaitResult w = rtg::wait_bounded([g] { return pending(g); }, [g] { return comm_error(g); },
                                                 g->timeout_ms);
    if (w == rtg::kWaitDone) return RT_OK;
    if (w == rtg::kWaitDeviceError) return fail(g, RT_ERR_DEVICE);
    abort_comms(g);
    return w == rtg::kWaitTimeout ? RT_ERR_TIMEOUT : RT_ERR_COMM;
}

void harvest(rt_group* g, PhaseRec& p) {
    if (!p.pending) return;
    p.pending = false;
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, p.ev[0], p.ev[1]) == hipSuccess) {
        g->sum[0] += ms;
        ++g->nsum[0];
    }
    if (p.has_fan && hipEventElapsedTime(&ms, p.ev[2], p.ev[3]) == hipSuccess) {
        g->sum[1] += ms;
        ++g->nsum[1];
    }
    if (p.has_unstripe && hipEventElapsedTime(&ms, p.ev[4], p.ev[5]) == hipSuccess) {
        g->sum[2] += ms;
        ++g->nsum[2];
    }
    const hipEvent_t last = p.has_unstripe ? p.ev[5] : (p.has_fan ? p.ev[3] : p.ev[1]);
    if (hipEventElapsedTime(&ms, p.ev[0], last) == hipSuccess) {
        g->sum[3] += ms;
        ++g->nsum[3];
    }
}

// Whether a frame's sky-row band is computed (rt_group_dispatch): rows that miss the
// root box are background only on the BVH branch with at least one bounce.
bool sky_applies(const rt_group* g) {
    return g->sky_rows && g->nranks > 1 && g->have_cam && g->have_params && g->have_root && g->params.useBVH &&
           g->params.maxBounces >= 1 && g->params.resY > 0;
}

// Every slot context of every local member.
template <class F>
int each_ctx(rt_group* g, F f) {
    if (!g) return RT_ERR_INVALID;
    if (g->broken) return RT_ERR_COMM;
    for (Member& b : g->m)
        for (Slot& s : b.slot) G_TRY(f(s.ctx));
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
    g->m.reserve(n);
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
    // a group whose fan-in never completes must not hang its owner: bounded, then abort
    if (!g->broken && wait_all(g) != RT_OK) abort_comms(g);
    for (Member& b : g->m) {
        hipSetDevice(b.device);
        if (b.comm) ncclCommDestroy(b.comm);
        for (Slot& s : b.slot) {
            if (!g->broken) hipStreamSynchronize(s.stream);
            if (s.ctx) rt_destroy(s.ctx);  // before its stream goes: it is ordered on it
            hipFree(s.buf);
            hipFree(s.staging);
            hipFree(s.img);
            if (s.rendered) hipEventDestroy(s.rendered);
            if (s.fanned) hipEventDestroy(s.fanned);
            if (s.released) hipEventDestroy(s.released);
            if (s.sync_ev) hipEventDestroy(s.sync_ev);
            if (s.stream) hipStreamDestroy(s.stream);
        }
        if (b.csync_ev) hipEventDestroy(b.csync_ev);
        if (b.cstream) hipStreamDestroy(b.cstream);
    }
    if (!g->m.empty()) {
        hipSetDevice(g->m[g->tm].device);
        for (PhaseRec& p : g->ring)
            for (hipEvent_t e : p.ev)
                if (e) hipEventDestroy(e);
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

int rt_group_set_frames(rt_group* g, int frames) {
    if (!g || frames < 1 || frames > kMaxFrames || g->have_scene || g->next > 0) return RT_ERR_INVALID;
    if (g->broken) return RT_ERR_COMM;
    for (Member& b : g->m) {
        while (static_cast<int>(b.slot.size()) < frames) G_TRY(add_slot(b));
        // fewer slots than before: nothing has been dispatched or uploaded yet, so the
        // extra ones go (each_ctx and pending() iterate every slot a member holds)
        while (static_cast<int>(b.slot.size()) > frames) {
            Slot& s = b.slot.back();
            G_HIP(hipSetDevice(b.device));
            if (s.ctx) rt_destroy(s.ctx);
            hipFree(s.buf);
            hipFree(s.staging);
            hipFree(s.img);
            if (s.rendered) hipEventDestroy(s.rendered);
            if (s.fanned) hipEventDestroy(s.fanned);
            if (s.released) hipEventDestroy(s.released);
            if (s.sync_ev) hipEventDestroy(s.sync_ev);
            if (s.stream) hipStreamDestroy(s.stream);
            b.slot.pop_back();
        }
    }
    g->frames = frames;
    return RT_OK;
}

int rt_group_frames(rt_group* g) { return g ? g->frames : RT_ERR_INVALID; }

int rt_group_member(rt_group* g, int k, rt_ctx** ctx) { return rt_group_member_slot(g, k, 0, ctx); }

int rt_group_member_slot(rt_group* g, int k, int slot, rt_ctx** ctx) {
    if (!g || !ctx || k < 0 || k >= static_cast<int>(g->m.size()) || slot < 0 || slot >= g->frames)
        return RT_ERR_INVALID;
    *ctx = g->m[k].slot[slot].ctx;
    return RT_OK;
}

int rt_group_upload_scene(rt_group* g, const FlatShape* shapes, int S, const FlatNode* nodes, int N, const int* idx,
                          int I) {
    const int rc = each_ctx(g, [&](rt_ctx* c) { return rt_upload_scene(c, shapes, S, nodes, N, idx, I); });
    if (g) mark_all_dirty(g);
    if (rc == RT_OK) {
        g->have_scene = true;
        g->have_root = N > 0 && nodes;  // the root the shader starts from (gpu_shader.comp:386)
        if (g->have_root) {
            const FlatNode& r = nodes[N - 1];
            const float lo[3] = {r.boundsMin.x, r.boundsMin.y, r.boundsMin.z}, hi[3] = {r.boundsMax.x, r.boundsMax.y, r.boundsMax.z};
            std::memcpy(g->root_lo, lo, sizeof lo);
            std::memcpy(g->root_hi, hi, sizeof hi);
        }
    }
    return rc;
}

int rt_group_set_camera(rt_group* g, const FlatCamera* cam) {
    const int rc = each_ctx(g, [&](rt_ctx* c) { return rt_set_camera(c, cam); });
    if (rc == RT_OK) {
        g->cam = *cam;
        g->have_cam = true;
    }
    return rc;
}

int rt_group_set_light(rt_group* g, const FlatLight* l) {
    return each_ctx(g, [&](rt_ctx* c) { return rt_set_light(c, l); });
}

int rt_group_set_params(rt_group* g, const rt_params* p) {
    const int rc = each_ctx(g, [&](rt_ctx* c) { return rt_set_params(c, p); });
    if (rc == RT_OK) {
        g->params = *p;
        g->have_params = true;
    }
    return rc;
}

// The reference's per-frame upload of an animated scene (src/main.cpp:336-346) on
// every local member x frame slot: each slot context holds its own copy of the scene
// and renders every F-th frame, so each one is given every update, in order (a slot
// that skipped a frame's rt_animate would miss that frame's updateBVH growth). The
// calls are the single-context ones, deferred or stream-ordered alike.
int rt_group_update_shapes(rt_group* g, int first, int count, const FlatShape* shapes) {
    return each_ctx(g, [&](rt_ctx* c) { return rt_update_shapes(c, first, count, shapes); });
}

int rt_group_update_nodes(rt_group* g, const FlatNode* nodes, int num_nodes) {
    const int rc = each_ctx(g, [&](rt_ctx* c) { return rt_update_nodes(c, nodes, num_nodes); });
    if (rc == RT_OK) g->have_root = rtx::view_root(g->m[0].slot[0].ctx, g->root_lo, g->root_hi);
    return rc;
}

int rt_group_set_animated(rt_group* g, const int* ids, int count) {
    return each_ctx(g, [&](rt_ctx* c) { return rt_set_animated(c, ids, count); });
}

int rt_group_animate(rt_group* g, const FlatShape* shapes) {
    // deferred per slot (rtx::animate_deferred): each slot context refits once, at the
    // dispatch of the next frame it renders, with the growth of every frame since its last
    const int rc = each_ctx(g, [&](rt_ctx* c) { return rtx::animate_deferred(c, shapes); });
    // the grown root (the sky-row band follows it): the same host computation in every
    // slot context and on every rank
    if (rc == RT_OK) g->have_root = rtx::view_root(g->m[0].slot[0].ctx, g->root_lo, g->root_hi);
    return rc;
}

int rt_group_set_sky_rows(rt_group* g, int on) {
    if (!g) return RT_ERR_INVALID;
    g->sky_rows = on != 0;
    return RT_OK;
}

int rt_group_dispatch(rt_group* g, int width, int height, int stripe) {
    if (!g || width <= 0 || height <= 0 || stripe <= 0 || height > 65535 ||
        stripe > 65535 / (g->share + g->nranks - 1))
        return RT_ERR_INVALID;
    if (g->broken) return RT_ERR_COMM;
    const int jj = static_cast<int>(g->next % g->frames);
    // Rows that can only be background (sky_rows.h) stay off the links: every rank
    // computes the same band [yb0, yb1) from the same camera, box and parameters; a
    // peer sends its compact rows inside it, rank 0 writes the rest as background.
    // Only where the reference draws the background for a ray missing the root:
    // the BVH branch with at least one bounce and a root box. The band follows the
    // group's camera and the root box its update calls leave (rt_group_update_nodes
    // sets it, rt_group_animate grows it as the device does), so it is recomputed
    // every frame. A member whose camera or node boxes were changed through its own
    // context instead (rt_group_member: rt_set_camera, rt_animate, rt_update_nodes)
    // would draw geometry in rows the band calls sky, so such a frame is refused
    // before this process posts anything (RT_ERR_INVALID; rt_group_set_sky_rows(g, 0)
    // lifts it). In a group of one process per GPU only the rank holding that member
    // refuses: the others post the frame and their fan-in runs into the timeout, which
    // aborts the communicator. That is the documented misuse (rt_group.h); the group
    // calls keep every rank's members equal.
    const bool sky = sky_applies(g);
    if (sky)
        for (Member& b : g->m)
            if (!rtx::matches_view(b.slot[jj].ctx, g->cam, g->root_lo, g->root_hi)) return RT_ERR_INVALID;
    // Every error from here on goes through fail(): in a multi-rank RCCL group the
    // peers may already wait on this frame's fan-in, so the communicator is aborted.
#define F_HIP(x)                                                     \
    do {                                                             \
        if ((x) != hipSuccess) return fail(g, RT_ERR_DEVICE);        \
    } while (0)
#define F_TRY(x)                                  \
    do {                                          \
        const int rc__ = (x);                     \
        if (rc__ != RT_OK) return fail(g, rc__);  \
    } while (0)
    const int P = g->nranks, k = g->share;
    const int j = static_cast<int>(g->next % g->frames);
    const size_t row_b = static_cast<size_t>(width) * 12;  // packed RGB32F
    const int rows1 = P > 1 ? rank_rows(height, P, stripe, k, 1).rows : 0;  // the most among ranks >= 1
    if (static_cast<long long>(P - 1) * rows1 > 65535) return RT_ERR_INVALID;  // k_unstripe's grid
    const size_t slot_b = std::max<size_t>(1, static_cast<size_t>(rows1) * row_b);
    // rank 0's staging holds the peers' rows only: its own go straight into the frame
    const size_t stage = static_cast<size_t>(P - 1) * rows1 * row_b;
    // (Re)size slot j's buffers; a resize waits for the frames that still use them.
    bool resize = false;
    for (Member& b : g->m) {
        const Slot& s = b.slot[j];
        resize = resize || (b.rank != 0 && s.buf_cap < slot_b) ||
                 (b.rank == 0 && (s.staging_cap < stage || s.img_w != width || s.img_h != height));
    }
    if (resize) {
        G_TRY(wait_all(g));  // aborts the communicators itself on a timeout or an RCCL error
        for (Member& b : g->m) {
            Slot& s = b.slot[j];
            F_HIP(hipSetDevice(b.device));
            if (b.rank != 0) {
                F_TRY(grow(s.buf, s.buf_cap, slot_b));
                continue;
            }
            F_TRY(grow(s.staging, s.staging_cap, std::max<size_t>(stage, 16)));
            if (s.img_w != width || s.img_h != height) {
                hipFree(s.img);
                s.img = nullptr;
                s.img_w = s.img_h = 0;
                size_t pitch = 0;
                if (hipMallocPitch(reinterpret_cast<void**>(&s.img), &pitch, static_cast<size_t>(width) * 16,
                                   height) != hipSuccess)
                    return fail(g, RT_ERR_NO_MEMORY);
                s.img_pitch = pitch;
                s.img_w = width;
                s.img_h = height;
            }
        }
    }
    int yb0 = 0, yb1 = height;  // the sky-row band (above)
    if (sky) rtg::sky_band(g->cam, g->root_lo, g->root_hi, height, g->params.resY, &yb0, &yb1);
    g->band_y0 = yb0;
    g->band_y1 = yb1;
    // the peers' compact row range inside the band (one contiguous run each)
    auto band_of = [&](int rank, int& c0, int& c1) {
        const Rows w = rank_rows(height, P, stripe, k, rank);
        c0 = rows_below(w.y0, w.stripe, w.period, w.rows, yb0);
        c1 = rows_below(w.y0, w.stripe, w.period, w.rows, yb1);
    };
    for (Member& b : g->m) {  // the streams this frame queues work on (mark_streams), errors included
        b.slot[j].dirty = true;
        b.cdirty = b.cdirty || P > 1;
    }
    if (!g->phase_timing && P > 1) {
        // Back-pressure without the phase events: the host issues this frame into slot j
        // only once slot j's frame F frames back has released its buffers (bounded, so a
        // stalled peer surfaces here within F frames, not only at the final sync).
        for (Member& b : g->m) {
            const Slot& s = b.slot[j];
            if (!s.used) continue;
            F_HIP(hipSetDevice(b.device));
            const hipEvent_t rel = s.released;
            const rtg::WaitResult w = rtg::wait_bounded(
                [rel] {
                    const hipError_t e = hipEventQuery(rel);
                    return e == hipSuccess ? 0 : (e == hipErrorNotReady ? 1 : -1);
                },
                [g] { return comm_error(g); }, g->timeout_ms);
            if (w == rtg::kWaitDeviceError) return fail(g, RT_ERR_DEVICE);
            if (w != rtg::kWaitDone) {
                abort_comms(g);
                return w == rtg::kWaitTimeout ? RT_ERR_TIMEOUT : RT_ERR_COMM;
            }
        }
    }
    PhaseRec& ph = g->ring[g->ring_pos];
    if (ph.pending) {
        // kPhaseRing frames ago. Nothing makes the host wait between dispatches, so that
        // frame may still be pending (a peer that never posts its send): never block on
        // it unbounded -- the group's bounded wait decides (RT_ERR_TIMEOUT, comms aborted).
        // Only that frame's last event is waited for (the host may run up to kPhaseRing
        // frames ahead; draining every stream here would empty the pipeline).
        F_HIP(hipSetDevice(g->m[g->tm].device));
        const hipEvent_t last = ph.ev[ph.has_unstripe ? 5 : (ph.has_fan ? 3 : 1)];
        const rtg::WaitResult w = rtg::wait_bounded(
            [last] {
                const hipError_t e = hipEventQuery(last);
                return e == hipSuccess ? 0 : (e == hipErrorNotReady ? 1 : -1);
            },
            [g] { return comm_error(g); }, g->timeout_ms);
        if (w == rtg::kWaitDeviceError) return fail(g, RT_ERR_DEVICE);
        if (w != rtg::kWaitDone) {
            abort_comms(g);
            return w == rtg::kWaitTimeout ? RT_ERR_TIMEOUT : RT_ERR_COMM;
        }
        harvest(g, ph);
    }
    ph.has_fan = ph.has_unstripe = false;
    // 1. every local rank renders its stripes on slot j's stream: rank 0 straight into
    //    slot j's surface at their image rows, the others into buf once the fan-in of
    //    the frame that last used the slot has sent it
    for (size_t mi = 0; mi < g->m.size(); ++mi) {
        Member& b = g->m[mi];
        Slot& s = b.slot[j];
        const bool timed = g->phase_timing && static_cast<int>(mi) == g->tm;
        F_HIP(hipSetDevice(b.device));
        if (s.used && b.rank != 0) {
            // RCCL: released on this member's fan-in stream; copies: rank 0's copy of it
            const hipEvent_t free_ev = g->transport == RT_GATHER_COPY ? g->m[g->root].slot[j].fanned : s.released;
            F_HIP(hipStreamWaitEvent(s.stream, free_ev, 0));
        }
        if (timed) F_HIP(hipEventRecord(ph.ev[0], s.stream));
        const Rows w = rank_rows(height, P, stripe, k, b.rank);
        if (w.rows > 0) {
            const int rc = b.rank == 0 ? rt_dispatch_rows_ex(s.ctx, width, height, w.y0, w.stripe, w.period, w.rows,
                                                             s.img, s.img_pitch, RT_FORMAT_RGBA32F_IMAGE)
                                       : rt_dispatch_rows_ex(s.ctx, width, height, w.y0, w.stripe, w.period, w.rows,
                                                             s.buf, row_b, RT_FORMAT_RGB32F);
            if (rc != RT_OK) return fail(g, rc);
        }
        if (timed) F_HIP(hipEventRecord(ph.ev[1], s.stream));
        if (P > 1) F_HIP(hipEventRecord(s.rendered, s.stream));  // the fan-in waits for it
    }
    auto slot_ptr = [&](int rank) {  // rank's rows in slot j's staging buffer (rank >= 1)
        return reinterpret_cast<char*>(g->m[g->root].slot[j].staging) + static_cast<size_t>(rank - 1) * rows1 * row_b;
    };
    // 2. fan-in to rank 0's staging on the members' fan-in streams, in frame order
    if (g->transport == RT_GATHER_RCCL && P > 1) {
        for (size_t mi = 0; mi < g->m.size(); ++mi) {
            Member& b = g->m[mi];
            Slot& s = b.slot[j];
            F_HIP(hipSetDevice(b.device));
            // a sender waits for its rows; rank 0 for the previous unstripe of this slot's staging
            const hipEvent_t before = b.rank == 0 ? (s.used ? s.released : nullptr) : s.rendered;
            if (before) F_HIP(hipStreamWaitEvent(b.cstream, before, 0));
            if (g->phase_timing && static_cast<int>(mi) == g->tm) F_HIP(hipEventRecord(ph.ev[2], b.cstream));
        }
        if (ncclGroupStart() != ncclSuccess) return fail(g, RT_ERR_COMM);
        for (Member& b : g->m) {
            Slot& s = b.slot[j];
            ncclResult_t res = ncclSuccess;
            if (b.rank == 0) {
                for (int r = 1; r < P && res == ncclSuccess; ++r) {
                    int c0, c1;
                    band_of(r, c0, c1);
                    const size_t n = static_cast<size_t>(c1 - c0) * width * 3;
                    if (n) res = ncclRecv(slot_ptr(r) + c0 * row_b, n, ncclFloat32, r, b.comm, b.cstream);
                }
            } else {
                int c0, c1;
                band_of(b.rank, c0, c1);
                const size_t n = static_cast<size_t>(c1 - c0) * width * 3;
                if (n) res = ncclSend(reinterpret_cast<char*>(s.buf) + c0 * row_b, n, ncclFloat32, 0, b.comm, b.cstream);
            }
            if (res != ncclSuccess) {
                ncclGroupEnd();
                return fail(g, RT_ERR_COMM);
            }
        }
        if (ncclGroupEnd() != ncclSuccess) return fail(g, RT_ERR_COMM);
        for (size_t mi = 0; mi < g->m.size(); ++mi) {
            Member& b = g->m[mi];
            Slot& s = b.slot[j];
            F_HIP(hipSetDevice(b.device));
            if (g->phase_timing && static_cast<int>(mi) == g->tm) {
                F_HIP(hipEventRecord(ph.ev[3], b.cstream));
                ph.has_fan = true;
            }
            F_HIP(hipEventRecord(s.fanned, b.cstream));
            if (b.rank != 0) {
                F_HIP(hipEventRecord(s.released, b.cstream));
                s.used = true;
            }
        }
    } else if (g->transport == RT_GATHER_COPY && P > 1) {
        Member& r = g->m[g->root];
        Slot& rs = r.slot[j];
        F_HIP(hipSetDevice(r.device));
        if (rs.used) F_HIP(hipStreamWaitEvent(r.cstream, rs.released, 0));
        if (g->phase_timing && g->tm == g->root) F_HIP(hipEventRecord(ph.ev[2], r.cstream));
        for (Member& b : g->m) {
            if (b.rank == 0) continue;
            int c0, c1;
            band_of(b.rank, c0, c1);
            const size_t n = static_cast<size_t>(c1 - c0) * row_b;
            F_HIP(hipStreamWaitEvent(r.cstream, b.slot[j].rendered, 0));
            if (n)
                F_HIP(hipMemcpyPeerAsync(slot_ptr(b.rank) + c0 * row_b, r.device,
                                         reinterpret_cast<char*>(b.slot[j].buf) + c0 * row_b, b.device, n, r.cstream));
            b.slot[j].used = true;  // its next render waits for rs.fanned
        }
        if (g->phase_timing && g->tm == g->root) {
            F_HIP(hipEventRecord(ph.ev[3], r.cstream));
            ph.has_fan = true;
        }
        F_HIP(hipEventRecord(rs.fanned, r.cstream));
    }
    // 3. rank 0: the peers' stripes into image order, into slot j's surface (its own
    //    rows are there already; with one rank there is nothing to move)
    if (g->root >= 0) {
        Member& r = g->m[g->root];
        Slot& rs = r.slot[j];
        F_HIP(hipSetDevice(r.device));
        if (P > 1 && rows1 > 0) {
            F_HIP(hipStreamWaitEvent(rs.stream, rs.fanned, 0));
            if (g->phase_timing && g->tm == g->root) F_HIP(hipEventRecord(ph.ev[4], rs.stream));
            hipLaunchKernelGGL(k_unstripe, dim3((width + 255) / 256, (P - 1) * rows1), dim3(256), 0, rs.stream,
                               rs.staging, rows1, width, height, stripe, k, P, reinterpret_cast<f4v*>(rs.img),
                               rs.img_pitch / 16, yb0, yb1, g->params.resY);
            F_HIP(hipGetLastError());
            if (g->phase_timing && g->tm == g->root) {
                F_HIP(hipEventRecord(ph.ev[5], rs.stream));
                ph.has_unstripe = true;
            }
        }
        // the next fan-in into this slot's staging waits for it (one rank: no fan-in)
        if (P > 1) {
            F_HIP(hipEventRecord(rs.released, rs.stream));
            rs.used = true;
        }
    }
#undef F_HIP
#undef F_TRY
    ph.pending = g->phase_timing;
    g->ring_pos = (g->ring_pos + 1) % kPhaseRing;
    g->last_slot = j;
    ++g->next;
    return RT_OK;
}

int rt_group_sky_band(rt_group* g, int* y0, int* y1) {
    if (!g || !y0 || !y1 || g->next == 0) return RT_ERR_INVALID;
    *y0 = g->band_y0;
    *y1 = g->band_y1;
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
    if (g->broken) return RT_ERR_COMM;
    std::memset(out, 0, sizeof *out);
    for (Member& b : g->m) {
        const Rows w = rank_rows(height, g->nranks, stripe, g->share, b.rank);
        if (w.rows == 0) continue;
        rt_stats st;
        G_TRY(rt_collect_stats_ex(b.slot[0].ctx, width, height, w.y0, w.stripe, w.period, w.rows, &st));
        uint64_t* o = reinterpret_cast<uint64_t*>(out);
        const uint64_t* a = reinterpret_cast<const uint64_t*>(&st);
        for (size_t i = 0; i < sizeof st / sizeof(uint64_t); ++i) o[i] += a[i];
    }
    return RT_OK;
}

int rt_group_set_phase_timing(rt_group* g, int on) {
    if (!g) return RT_ERR_INVALID;
    g->phase_timing = on != 0;
    return RT_OK;
}

int rt_group_set_timeout(rt_group* g, double ms) {
    if (!g || !(ms >= 0)) return RT_ERR_INVALID;
    g->timeout_ms = ms;
    return RT_OK;
}

int rt_group_check(rt_group* g) {
    if (!g) return RT_ERR_INVALID;
    if (g->broken) return RT_ERR_COMM;
    if (comm_error(g)) {
        abort_comms(g);
        return RT_ERR_COMM;
    }
    return RT_OK;
}

int rt_group_sync(rt_group* g) {
    if (!g) return RT_ERR_INVALID;
    if (g->broken) return RT_ERR_COMM;
    return wait_all(g);
}

int rt_group_phase_times(rt_group* g, rt_group_phases* out) {
    if (!g || !out) return RT_ERR_INVALID;
    G_TRY(rt_group_sync(g));
    hipSetDevice(g->m[g->tm].device);
    for (PhaseRec& p : g->ring) harvest(g, p);
    out->frames = g->nsum[3];
    out->render_ms = g->nsum[0] ? static_cast<float>(g->sum[0] / g->nsum[0]) : 0.f;
    out->fanin_ms = g->nsum[1] ? static_cast<float>(g->sum[1] / g->nsum[1]) : 0.f;
    out->unstripe_ms = g->nsum[2] ? static_cast<float>(g->sum[2] / g->nsum[2]) : 0.f;
    out->frame_ms = g->nsum[3] ? static_cast<float>(g->sum[3] / g->nsum[3]) : 0.f;
    for (int i = 0; i < 4; ++i) {
        g->sum[i] = 0;
        g->nsum[i] = 0;
    }
    return RT_OK;
}

int rt_group_read_image(rt_group* g, float* dst, size_t pitch, int width, int height) {
    if (!g || g->root < 0 || !dst || g->last_slot < 0) return RT_ERR_INVALID;
    Member& r = g->m[g->root];
    Slot& s = r.slot[g->last_slot];
    if (!s.img || width != s.img_w || height != s.img_h || pitch < static_cast<size_t>(width) * 16)
        return RT_ERR_INVALID;
    G_TRY(rt_group_sync(g));
    G_HIP(hipSetDevice(r.device));
    G_HIP(hipMemcpy2DAsync(dst, pitch, s.img, s.img_pitch, static_cast<size_t>(width) * 16, height,
                           hipMemcpyDeviceToHost, s.stream));
    G_HIP(hipStreamSynchronize(s.stream));
    return RT_OK;
}

int rt_group_device_image(rt_group* g, void** p, size_t* pitch) {
    if (!g || g->root < 0 || !p || !pitch || g->last_slot < 0) return RT_ERR_INVALID;
    if (g->broken) return RT_ERR_COMM;
    const Slot& s = g->m[g->root].slot[g->last_slot];
    if (!s.img) return RT_ERR_INVALID;
    *p = s.img;
    *pitch = s.img_pitch;
    return RT_OK;
}

}  // extern "C"

// group_check.cpp — a C++ host (no Python, no torch) drives the multi-GPU
// entry points of librtamd.so (include/rt_group.h) and checks that the
// gathered frame equals the single-dispatch frame bit for bit.
//
//   group_check W H [config [ranks]]   exit 0 = every case identical
//
// Cases run on whatever devices the box has:
//   * copy transport, 1..ranks (default 4) ranks all on device 0 (stripes + peer copies + unstripe);
//   * the same with rank 0 taking 2 stripes per period (rt_group_set_root_share);
//   * RCCL transport, one rank per distinct device (ncclCommInitAll + send/recv),
//     which on a 1-GPU box is the 1-rank communicator;
//   * on >= 2 devices, RCCL over the first 2 and all devices, root share 1 and 2;
//   * animated frames (rt_group_set_animated / rt_group_animate, and
//     rt_group_update_shapes + rt_group_update_nodes with rts_update_bvh's nodes)
//     against one context given the same calls, every frame, 1 and 3 in flight.
// The scene is the config's own (rts_generate: the reference's builder and
// serialisers), uploaded as the reference uploads its SSBOs (src/main.cpp:256-275).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/rt_api.h"
#include "../../include/rt_group.h"
#include "../../include/rt_scene.h"

#define CHECK(x)                                                                         \
    do {                                                                                 \
        int rc__ = (x);                                                                  \
        if (rc__ != RT_OK) {                                                             \
            std::fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #x, rc__,  \
                         rt_status_string(rc__));                                        \
            std::exit(2);                                                                \
        }                                                                                \
    } while (0)

struct Scene {
    std::vector<FlatShape> shapes;
    std::vector<FlatNode> nodes;
    std::vector<int> idx;
    FlatCamera cam;
    FlatLight light;
};

static Scene make_scene(int config, int W, int H) {
    Scene s;
    rts_scene* h = rts_new();
    if (!h || rts_generate(h, config, 0, static_cast<float>(W) / static_cast<float>(H)) < 0) std::exit(3);
    int S = 0, N = 0, I = 0;
    rts_counts(h, &S, &N, &I);
    s.shapes.resize(S);
    s.nodes.resize(N);
    s.idx.resize(I);
    if (rts_serialize(h, s.shapes.data(), s.nodes.data(), s.idx.data(), &s.cam, &s.light) < 0) std::exit(3);
    rts_free(h);
    return s;
}

static int compare(const char* what, const std::vector<float>& ref, const std::vector<float>& img) {
    size_t bad = 0;
    for (size_t i = 0; i < ref.size(); ++i) bad += std::memcmp(&ref[i], &img[i], 4) != 0;
    std::printf("%-44s %s (%zu of %zu floats differ)\n", what, bad ? "DIFFERS" : "identical", bad, ref.size());
    return bad ? 1 : 0;
}

static int run_group(const char* what, const Scene& s, const rt_params& p, int W, int H, int stripe,
                     const int* devs, int n, int transport, const std::vector<float>& ref, int share = 1,
                     int frames = 1) {
    rt_group* g = nullptr;
    const int rc = rt_group_create(&g, devs, n, transport);
    if (rc != RT_OK) {
        std::printf("%-44s create failed: %s\n", what, rt_status_string(rc));
        return 1;
    }
    CHECK(rt_group_set_frames(g, frames));
    CHECK(rt_group_upload_scene(g, s.shapes.data(), static_cast<int>(s.shapes.size()), s.nodes.data(),
                                static_cast<int>(s.nodes.size()), s.idx.data(), static_cast<int>(s.idx.size())));
    CHECK(rt_group_set_camera(g, &s.cam));
    CHECK(rt_group_set_light(g, &s.light));
    CHECK(rt_group_set_params(g, &p));
    CHECK(rt_group_set_root_share(g, share));
    // 2F + 1 frames: every slot's buffers are reused across frames, as in a render loop
    for (int f = 0; f < 2 * frames + 1; ++f) CHECK(rt_group_dispatch(g, W, H, stripe));
    CHECK(rt_group_sync(g));
    std::vector<float> img(static_cast<size_t>(W) * H * 4);
    CHECK(rt_group_read_image(g, img.data(), static_cast<size_t>(W) * 16, W, H));
    int nr = 0, nl = 0, tr = 0;
    CHECK(rt_group_info(g, &nr, &nl, &tr));
    char label[96];
    std::snprintf(label, sizeof label, "%s [%d ranks, %s, share %d, %d in flight]", what, nr,
                  tr == RT_GATHER_RCCL ? "rccl" : "copy", share, frames);
    // a short destination is refused, not overrun
    const int short_rc = rt_group_read_image(g, img.data(), static_cast<size_t>(W) * 16, W, H - 1);
    CHECK(rt_group_destroy(g));
    if (short_rc != RT_ERR_INVALID) {
        std::printf("%s: short read_image returned %d\n", label, short_rc);
        return 1;
    }
    return compare(label, ref, img);
}

// Frame f's records of the animated shapes: triangles turn 0.05 rad per frame about
// z through their centroid, spheres bounce in y (the two animations the reference
// runs, src/main.cpp:1079-1109); other kinds keep their records.
static void animate_records(const Scene& s, const std::vector<int>& ids, int f, std::vector<FlatShape>& out) {
    out.resize(ids.size());
    const float a = 0.05f * static_cast<float>(f + 1), ca = std::cos(a), sa = std::sin(a);
    for (size_t i = 0; i < ids.size(); ++i) {
        FlatShape r = s.shapes[ids[i]];
        if (r.type == RT_TRIANGLE) {
            const float cx = (r.triP1.x + r.triP2.x + r.triP3.x) / 3.f, cy = (r.triP1.y + r.triP2.y + r.triP3.y) / 3.f;
            for (rt_vec3* p : {&r.triP1, &r.triP2, &r.triP3}) {
                const float qx = p->x - cx, qy = p->y - cy;
                p->x = cx + qx * ca - qy * sa;
                p->y = cy + qx * sa + qy * ca;
            }
        } else if (r.type == RT_SPHERE) {
            r.sphereCenter.y += 0.5f * std::sin(0.7f * static_cast<float>(f + 1));
        }
        out[i] = r;
    }
}

// Animated frames through the group calls (rt_group_set_animated / rt_group_animate,
// or rt_group_update_shapes + rt_group_update_nodes with the nodes grown on the host
// by rts_update_bvh) against one context given the same calls, frame by frame.
static int run_group_animated(const char* what, const Scene& s, const rt_params& p, int W, int H, int n,
                              int frames, bool updates, const std::vector<float>& still) {
    std::vector<int> ids;  // every 7th sphere or triangle, up to 96 of them
    for (int i = 0; i < static_cast<int>(s.shapes.size()) && ids.size() < 96; i += 7)
        if (s.shapes[i].type == RT_SPHERE || s.shapes[i].type == RT_TRIANGLE) ids.push_back(i);
    if (ids.empty()) {
        std::printf("%-44s skipped (no spheres or triangles)\n", what);
        return 0;
    }
    const std::vector<int> zeros(n, 0);
    rt_group* g = nullptr;
    rt_ctx* c = nullptr;
    CHECK(rt_group_create(&g, zeros.data(), n, RT_GATHER_COPY));
    CHECK(rt_group_set_frames(g, frames));
    CHECK(rt_create(&c, 0));
    const int S = static_cast<int>(s.shapes.size()), N = static_cast<int>(s.nodes.size()),
              I = static_cast<int>(s.idx.size());
    CHECK(rt_group_upload_scene(g, s.shapes.data(), S, s.nodes.data(), N, s.idx.data(), I));
    CHECK(rt_upload_scene(c, s.shapes.data(), S, s.nodes.data(), N, s.idx.data(), I));
    CHECK(rt_group_set_camera(g, &s.cam));
    CHECK(rt_group_set_light(g, &s.light));
    CHECK(rt_group_set_params(g, &p));
    CHECK(rt_set_camera(c, &s.cam));
    CHECK(rt_set_light(c, &s.light));
    CHECK(rt_set_params(c, &p));
    if (!updates) {
        CHECK(rt_group_set_animated(g, ids.data(), static_cast<int>(ids.size())));
        CHECK(rt_set_animated(c, ids.data(), static_cast<int>(ids.size())));
    }
    std::vector<FlatShape> rec, shapes = s.shapes;
    std::vector<FlatNode> nodes = s.nodes;
    std::vector<float> ref(static_cast<size_t>(W) * H * 4), img(ref.size());
    int bad_frames = 0, moved_frames = 0;  // moved: the frame differs from the still scene's
    size_t bad = 0;
    for (int f = 0; f < 3 * frames + 2; ++f) {
        animate_records(s, ids, f, rec);
        if (updates) {
            for (size_t i = 0; i < ids.size(); ++i) {
                shapes[ids[i]] = rec[i];
                CHECK(rt_group_update_shapes(g, ids[i], 1, &rec[i]));
                CHECK(rt_update_shapes(c, ids[i], 1, &rec[i]));
            }
            if (rts_update_bvh(shapes.data(), S, nodes.data(), N, s.idx.data(), I, ids.data(),
                               static_cast<int>(ids.size())) != 0)
                std::exit(3);
            CHECK(rt_group_update_nodes(g, nodes.data(), N));
            CHECK(rt_update_nodes(c, nodes.data(), N));
        } else {
            CHECK(rt_group_animate(g, rec.data()));
            CHECK(rt_animate(c, rec.data()));
        }
        CHECK(rt_group_dispatch(g, W, H, 8));
        CHECK(rt_dispatch(c, W, H, 0, H));
        CHECK(rt_group_sync(g));
        CHECK(rt_sync(c));
        CHECK(rt_group_read_image(g, img.data(), static_cast<size_t>(W) * 16, W, H));
        CHECK(rt_read_image(c, ref.data(), static_cast<size_t>(W) * 16, W, H));
        size_t b = 0;
        for (size_t i = 0; i < ref.size(); ++i) b += std::memcmp(&ref[i], &img[i], 4) != 0;
        bad += b;
        bad_frames += b != 0;
        moved_frames += std::memcmp(still.data(), img.data(), img.size() * 4) != 0;
    }
    CHECK(rt_group_destroy(g));
    CHECK(rt_destroy(c));
    char label[112];
    std::snprintf(label, sizeof label, "%s [%d ranks, %zu shapes, %d in flight]", what, n, ids.size(), frames);
    std::printf("%-44s %s (%d of %d frames differ, %zu floats; %d frames moved)\n", label,
                bad ? "DIFFERS" : "identical", bad_frames, 3 * frames + 2, bad, moved_frames);
    return bad || moved_frames == 0 ? 1 : 0;
}

int main(int argc, char** argv) {
    const int W = argc > 1 ? std::atoi(argv[1]) : 480;
    const int H = argc > 2 ? std::atoi(argv[2]) : 270;
    const int config = argc > 3 ? std::atoi(argv[3]) : 3;
    const int max_ranks = argc > 4 ? std::atoi(argv[4]) : 4;
    int ndev = 0;  // devices, probed through the C ABI (rt_create refuses an absent ordinal)
    for (rt_ctx* probe = nullptr; rt_create(&probe, ndev) == RT_OK; ++ndev) rt_destroy(probe);
    if (ndev < 1) {
        std::fprintf(stderr, "no HIP device\n");
        return 4;
    }
    std::printf("%d HIP device(s)\n", ndev);
    const Scene s = make_scene(config, W, H);
    const rt_params p{static_cast<float>(W), static_cast<float>(H), 3, 1, 0, 0};

    // the single-dispatch frame (rt_dispatch of the whole image on device 0)
    rt_ctx* c = nullptr;
    CHECK(rt_create(&c, 0));
    CHECK(rt_upload_scene(c, s.shapes.data(), static_cast<int>(s.shapes.size()), s.nodes.data(),
                          static_cast<int>(s.nodes.size()), s.idx.data(), static_cast<int>(s.idx.size())));
    CHECK(rt_set_camera(c, &s.cam));
    CHECK(rt_set_light(c, &s.light));
    CHECK(rt_set_params(c, &p));
    CHECK(rt_dispatch(c, W, H, 0, H));
    CHECK(rt_sync(c));
    std::vector<float> ref(static_cast<size_t>(W) * H * 4);
    CHECK(rt_read_image(c, ref.data(), static_cast<size_t>(W) * 16, W, H));
    CHECK(rt_destroy(c));

    int fails = 0;
    const std::vector<int> zeros(max_ranks > 3 ? max_ranks : 3, 0);
    for (int n = 1; n <= max_ranks; ++n) {
        char what[64];
        std::snprintf(what, sizeof what, "config %d %dx%d, stripes of 8", config, W, H);
        fails += run_group(what, s, p, W, H, 8, zeros.data(), n, RT_GATHER_COPY, ref);
        if (n > 1) fails += run_group(what, s, p, W, H, 8, zeros.data(), n, RT_GATHER_COPY, ref, 2);
    }
    fails += run_group("stripes of 5 (ragged last stripe)", s, p, W, H, 5, zeros.data(), 3, RT_GATHER_COPY, ref);
    fails += run_group("stripe taller than the frame", s, p, W, H, H + 3, zeros.data(), 2, RT_GATHER_COPY, ref);
    fails += run_group("rccl, one rank per device", s, p, W, H, 8, zeros.data(), 1, RT_GATHER_RCCL, ref);
    fails += run_group("frames in flight", s, p, W, H, 8, zeros.data(), 3, RT_GATHER_COPY, ref, 2, 4);
    fails += run_group("rccl, frames in flight", s, p, W, H, 8, zeros.data(), 1, RT_GATHER_RCCL, ref, 1, 3);
    fails += run_group_animated("animated (rt_group_animate)", s, p, W, H, 3, 1, false, ref);
    fails += run_group_animated("animated (rt_group_animate)", s, p, W, H, 2, 3, false, ref);
    fails += run_group_animated("updated (update_shapes + update_nodes)", s, p, W, H, 2, 2, true, ref);
    {
        rt_group* g = nullptr;
        const int rc = rt_group_create(&g, zeros.data(), 2, RT_GATHER_RCCL);
        std::printf("%-44s %s\n", "rccl forced on a repeated device", rc == RT_ERR_COMM ? "refused" : "NOT refused");
        fails += rc == RT_ERR_COMM ? 0 : 1;
        if (g) rt_group_destroy(g);
    }
    if (ndev >= 2) {
        std::vector<int> all(ndev);
        for (int d = 0; d < ndev; ++d) all[d] = d;
        fails += run_group("rccl over 2 devices", s, p, W, H, 8, all.data(), 2, RT_GATHER_RCCL, ref);
        fails += run_group("rccl over every device", s, p, W, H, 8, all.data(), ndev, RT_GATHER_RCCL, ref);
        fails += run_group("rccl over 2 devices", s, p, W, H, 8, all.data(), 2, RT_GATHER_RCCL, ref, 2);
        fails += run_group("rccl over every device", s, p, W, H, 8, all.data(), ndev, RT_GATHER_RCCL, ref, 2);
        fails += run_group("rccl over every device", s, p, W, H, 8, all.data(), ndev, RT_GATHER_RCCL, ref, 1, 4);
    }
    std::printf("%s\n", fails ? "FAIL" : "OK");
    return fails ? 1 : 0;
}

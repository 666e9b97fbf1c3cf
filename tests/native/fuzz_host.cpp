// fuzz_host.cpp — TEST HARNESS: drives the product's host code (librtscene's
// scene.cpp: OBJ parser, builder, serialisers, image dump; accel.cpp: the
// accelerator build that rt_upload_scene runs on the host) over malformed and
// randomly mutated inputs. tests/test_sanitize.py compiles it together with
// those two sources under AddressSanitizer + UndefinedBehaviorSanitizer
// (-fno-sanitize-recover: the first finding aborts) and runs it on the CPU.
//
// The reference reads meshes through assimp (src/model.hpp:49-65) and walks
// them in mesh2triangles (src/mesh.hpp:163-189); here the input is untrusted
// OBJ text, so every path must either load or return an error code.
//
//   fuzz_host [iterations] [seed]        exit 0 = no crash, no sanitizer report
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rt_scene.h"
#include "../../opengl-ray-tracer_amd/csrc/accel.h"

namespace {

uint64_t g_state = 0x9E3779B97F4A7C15ull;
uint32_t rnd() {
    g_state ^= g_state << 13;
    g_state ^= g_state >> 7;
    g_state ^= g_state << 17;
    return static_cast<uint32_t>(g_state >> 11);
}

const char* kSeeds[] = {
    // a valid cube (quads: fan triangulation), all corner forms
    "o cube\nv -1 -1 -1\nv 1 -1 -1\nv 1 1 -1\nv -1 1 -1\nv -1 -1 1\nv 1 -1 1\nv 1 1 1\nv -1 1 1\n"
    "vt 0 0\nvt 1 0\nvn 0 0 1\n"
    "f 1 2 3 4\nf 5/1 6/2 7/1 8/2\nf 1//1 5//1 8//1 4//1\nf 2/1/1 6/2/1 7/1/1 3/2/1\nf -8 -7 -3\n",
    // malformed records
    "v 1 2\nv a b c\nv 1e40 -1e40 nan\nf 1 2 3\nf 0 1 2\nf 1 2 99\nf -100 1 2\nf\nf 1\nf 1 2\nf 1/ 2// 3/x/\n",
    // comments, blank lines, CRLF, tabs, no trailing newline
    "# comment\r\n\r\nv\t0 0 0\r\nv 1 0 0\r\nv 0 1 0\r\nf 1 2 3",
    // numbers at the edges of float
    "v 3.4e38 3.4e38 3.4e38\nv -3.4e38 0 0\nv 1e-45 0 1e-45\nv inf 0 0\nf 1 2 3\nf 2 3 4\nf 1 3 4\n",
    // a long polygon and repeated indices
    "v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nv -1 1 0\nv -1 0 0\nf 1 2 3 4 5 6 1 2 3 4 5 6\nf 1 1 1\n",
    // other statements the parser must skip
    "mtllib x.mtl\nusemtl red\ng grp\ns off\nl 1 2\np 1\nvp 0.5\nv 0 0 0\nv 0 0 1\nv 0 1 0\nf 1 2 3\n",
};

std::string mutate(const std::string& s) {
    std::string m = s;
    const int edits = 1 + static_cast<int>(rnd() % 8);
    static const char kAlpha[] = "0123456789 -+./eEnaif#vtn\n\r\t/";
    for (int e = 0; e < edits; ++e) {
        const size_t pos = m.empty() ? 0 : rnd() % (m.size() + 1);
        switch (rnd() % 5) {
            case 0:  // insert
                m.insert(m.begin() + static_cast<long>(pos), kAlpha[rnd() % (sizeof kAlpha - 1)]);
                break;
            case 1:  // delete
                if (pos < m.size()) m.erase(pos, 1 + rnd() % 4);
                break;
            case 2:  // replace
                if (pos < m.size()) m[pos] = static_cast<char>(rnd() % 256);
                break;
            case 3:  // duplicate a slice
                if (pos < m.size()) m.insert(pos, m.substr(pos, 1 + rnd() % 24));
                break;
            default:  // a huge index or number
                m.insert(pos, (rnd() & 1) ? " 2147483647 " : " -99999999999999999999 ");
        }
    }
    return m;
}

int g_loaded = 0, g_rejected = 0, g_built = 0;

// rt_upload_scene's host half: serialise the reference tree, then build the accelerator over it.
void build_everything(rts_scene* s, int max_depth) {
    if (rts_build_bvh(s, max_depth) < 0) return;
    int S = 0, N = 0, I = 0;
    if (rts_counts(s, &S, &N, &I) < 0) return;
    std::vector<FlatShape> shapes(S > 0 ? S : 1);
    std::vector<FlatNode> nodes(N > 0 ? N : 1);
    std::vector<int> idx(I > 0 ? I : 1);
    FlatCamera cam;
    FlatLight light;
    if (rts_serialize(s, shapes.data(), nodes.data(), idx.data(), &cam, &light) < 0) return;
    int leaves = 0, max_leaf = 0, depth = 0, stack = 0;
    rts_bvh_stats(s, &leaves, &max_leaf, &depth, &stack);
    if (N > 0) {
        rta::AccelHost A;
        if (rta::build_accel(shapes.data(), S, nodes.data(), N, idx.data(), I, 8, 64, A)) ++g_built;
    }
}

void parse_one(const std::string& text) {
    rts_scene* s = rts_new();
    const float origin[3] = {0.f, 0.f, -30.f};
    const int rc = rts_parse_obj(s, text.data(), static_cast<long>(text.size()), origin, nullptr,
                                 static_cast<int>(rnd() & 1));
    if (rc < 0) {
        ++g_rejected;
    } else {
        ++g_loaded;
        build_everything(s, 1 + static_cast<int>(rnd() % 25));
    }
    rts_free(s);
}

float rval() {
    switch (rnd() % 16) {
        case 0: return 0.f;
        case 1: return NAN;
        case 2: return (rnd() & 1) ? INFINITY : -INFINITY;
        case 3: return (rnd() & 1) ? 3.0e38f : -3.0e38f;
        case 4: return 1e-30f;
        default: return (static_cast<float>(rnd() % 20001) - 10000.f) * 0.01f;
    }
}

// Random shape soups with degenerate records: NaN/inf coordinates, zero-area
// and sliver triangles, +-Y walls (NaN basis), planes, zero/negative radii.
void soup_one() {
    rts_scene* s = rts_new();
    const int n = 1 + static_cast<int>(rnd() % 60);
    for (int i = 0; i < n; ++i) {
        float a[3] = {rval(), rval(), rval()}, b[3] = {rval(), rval(), rval()}, c[3] = {rval(), rval(), rval()};
        switch (rnd() % 6) {
            case 0: rts_add_sphere(s, a, rval(), nullptr); break;
            case 1: rts_add_plane(s, a, b, nullptr); break;
            case 2: {
                const float ny[3] = {0.f, (rnd() & 1) ? 1.f : -1.f, 0.f};
                rts_add_wall(s, a, rval(), rval(), (rnd() & 1) ? ny : b, nullptr);
                break;
            }
            case 3: {  // sliver: c on the segment ab
                float m[3] = {0.5f * (a[0] + b[0]), 0.5f * (a[1] + b[1]), 0.5f * (a[2] + b[2])};
                rts_add_triangle(s, a, b, m, static_cast<int>(rnd() & 1), nullptr);
                break;
            }
            default: rts_add_triangle(s, a, b, c, static_cast<int>(rnd() & 1), nullptr);
        }
    }
    build_everything(s, 1 + static_cast<int>(rnd() % 25));
    rts_free(s);
}

}  // namespace

int main(int argc, char** argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
    if (argc > 2) g_state ^= std::strtoull(argv[2], nullptr, 10) * 0x2545F4914F6CDD1Dull;
    for (const char* seed : kSeeds) parse_one(seed);
    parse_one(std::string());
    parse_one(std::string(1 << 16, 'v'));
    for (int i = 0; i < iters; ++i) parse_one(mutate(kSeeds[rnd() % (sizeof kSeeds / sizeof *kSeeds)]));
    for (int i = 0; i < iters / 4; ++i) soup_one();
    // the benchmark scenes through the same host path
    for (int cfg = 1; cfg <= 3; ++cfg)
        for (int variant = 0; variant <= (cfg == 3 ? 1 : 0); ++variant) {
            rts_scene* s = rts_new();
            if (rts_generate(s, cfg, variant, 16.f / 9.f) < 0) return 3;
            build_everything(s, cfg == 2 ? 15 : 25);
            rts_free(s);
        }
    // image dump: both formats, tight and padded pitch; bad arguments rejected
    std::vector<float> img(7 * 5 * 4 + 16, 0.5f);
    img[3] = NAN;
    img[6] = INFINITY;
    int bad = 0;
    bad += rts_write_image("/tmp/fuzz_host.ppm", img.data(), 7, 5, 7 * 16, RTS_IMAGE_PPM) != 0;
    bad += rts_write_image("/tmp/fuzz_host.pfm", img.data(), 6, 5, 7 * 16, RTS_IMAGE_PFM) != 0;
    bad += rts_write_image("/tmp/fuzz_host.ppm", img.data(), 7, 5, 7 * 15, RTS_IMAGE_PPM) == 0;
    bad += rts_write_image("/tmp/fuzz_host.ppm", img.data(), 0, 5, 7 * 16, RTS_IMAGE_PPM) == 0;
    std::remove("/tmp/fuzz_host.ppm");
    std::remove("/tmp/fuzz_host.pfm");
    std::printf("loaded %d, rejected %d, accelerators built %d, image checks failed %d\n", g_loaded, g_rejected,
                g_built, bad);
    return bad ? 1 : 0;
}

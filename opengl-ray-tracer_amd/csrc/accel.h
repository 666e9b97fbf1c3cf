// accel.h — host-side builder of the exact-result accelerator (librtamd.so).
//
// The reference tests every shape of every leaf whose box a ray enters
// (gpu_shader.comp:399-421) and keeps the nearest INNER hit, the first one in
// walk order on a tie. Its spatial-midpoint tree collapses into leaves of
// thousands of shapes, so most of the work is those scans.
// The accelerator keeps the reference's result bit for bit while skipping
// shapes that provably cannot win:
//
//   * the set of shapes a ray may hit is still decided by the reference's own
//     nodes and exact box test (which leaves a lane enters never changes);
//   * inside a large leaf, shapes are grouped under a local BVH whose boxes
//     are *conservative*: each contains every point the reference test can
//     return as an INNER hit for that shape, padded well beyond float error.
//     Shapes without such a bound (planes, walls with a ±Y normal whose basis
//     is NaN, triangles whose stored plane is steep to their vertices' plane
//     or that are too thin to bound their barycentric error) are tested
//     always (accel_bound.h, classify);
//   * a lane skips a local box only if its entry distance exceeds the lane's
//     best hit by a relative margin, and every candidate carries its rank in
//     the reference walk ("seq"), so the winner is the lexicographic minimum
//     of (distance, seq): exactly the reference's strict-< first-wins rule.
#pragma once

#include <cstdint>
#include <functional>
#include <vector>

#include "../../include/rt_flat.h"
#include "accel_bound.h"

namespace rta {

// Scene tree (build_scene_tree): one SAH tree over the shapes of every
// reference leaf, for rays whose slab values cannot be NaN (finite origin,
// finite non-zero 1/d). When every child box of the reference tree lies inside
// its parent's box, such a ray passes the exact test (gpu_shader.comp:364-377)
// of every ancestor of a leaf whose own box it passes: per axis the rounded
// slab values of the child lie between the parent's (rounding is monotone),
// so tmin only grows and tmax only shrinks going up. The reference therefore
// tests a leaf's shapes iff the ray passes that leaf's own box, and the tree
// above the leaves may be any tree. Each scene-tree leaf ("item") holds shapes
// of ONE reference leaf and carries that leaf's exact box, tested before its
// shapes; the inner boxes are the conservative shape bounds, as in the local
// BVHs. Unbounded shapes (planes, ...) sit in a separate subtree over their
// leaves' padded exact boxes, which bound where the ray may be when the leaf
// is entered but not where it hits: those nodes have cone threshold kNoPrune
// (never culled by cone or distance; entered at parameter 0).
struct SceneTree {
    // binary nodes: inner a = left, b = right | axis << 30; leaf a = -(start+1), b = count
    std::vector<Box3> box;
    std::vector<int> a, b;
    std::vector<int> item_of;   // per node: item id of a leaf, -1 for inner
    std::vector<int> item_ref;  // per item: its reference leaf
    std::vector<int> item_start, item_count;  // per item: prim range (AccelHost prims)
    std::vector<int> wchild, wsub;            // wide collapse (as AccelHost)
    std::vector<char> wpair;                  // per record (as AccelHost)
    int wroot = -1;             // wide root, -1: no scene tree for this scene
    int max_stack = 0;          // the lane walk's stack bound over it
    int height = 0;             // binary height
    int nested = 0;             // the reference tree's boxes nest (the condition above)
};

struct AccelHost {
    // prims: the shapes in the order the accelerated kernel reads them.
    std::vector<int> prim_shape;  // shape index per prim slot
    std::vector<int> prim_seq;    // rank in the reference walk
    // Per top-level (reference) node: content box + flags, and for leaves
    // the plain-scan range [plain_start, +plain_count) and the local root.
    std::vector<Box3> content;
    std::vector<int> flags;       // bit0-1 order axis, bit2 swap, bit3 bounded
    std::vector<int> plain_start, plain_count, local_root;
    // Local BVH nodes: box; inner: left, right | axis<<30; leaf: -(start+1), count.
    std::vector<Box3> lbox;
    std::vector<int> la, lb;
    // Back-face cone per local node: every shape below has an INNER-capable
    // normal within the cone, so a ray with dot(axis, d) < thr*|d| cannot get
    // an INNER hit there (np = N.d > 0 is required, gpu_shader.comp:206,278,294).
    // thr = -sin(angle + margin), or -4 (never culls).
    std::vector<float> lcone;     // 4 per local node: axis.xyz, thr
    // 4-wide collapse of the local trees (build_wide): each wide node holds up
    // to kWide binary nodes (their boxes and cones are tested at the wide node),
    // wchild = binary node index or -1, wsub = wide node of an inner child or -1.
    // wroot = wide node of each reference leaf's local root (-1: none, or a leaf).
    std::vector<int> wchild, wsub, wroot;
    // Per record of kWide children: 1 if it and the next record are ONE node of up to
    // 2 kWide children (kWideKids = 8, barycentric accelerators): the walk tests both
    // records' children at one step (rt_kernels.hip, the kPair bit of the node's code).
    std::vector<char> wpair;
    int max_stack = 0;            // worst-case wave stack entries
    // Largest |coordinate| of any bounded shape box, and the largest |coordinate|
    // of a ray origin the bounds are built for (kOriginRel * (scene_mag + 1)).
    // Rays from farther away take the always-enter mode of the padded tests
    // (accel_math.h); a camera farther away skips the accelerator for the
    // frame (rt_kernels.hip, launch()).
    float scene_mag = 0.f, origin_lim = 0.f;
    int always_prims = 0, bounded_prims = 0, local_leaves = 0;
    // Scene tree; its prims follow the local ones in prim_shape / prim_seq,
    // its cones are in st_cone (4 per binary node, as lcone).
    SceneTree st;
    std::vector<float> st_cone;
    // Built for the Moller-Trumbore triangle test (build_accel mt): static triangle
    // boxes (classify_mt_tight), grown per ray by the MT error bound (lmt below,
    // accel_math.h mt_pad / mt_slab); no back-face culling, and the cones of lcone
    // are GRAZING cones: axis and s = 2 sin(psi/2) over the triangle normals below,
    // either orientation (s = 2: any direction). Reference-node content boxes are
    // not used (flags bit 3 clear) and no scene tree is built.
    bool mt = false;
    // MT per-ray padding (accel_bound.h, mt_pad): per local node the worst-case
    // triangle constants below it, kMtPadF floats each (MtPad order), and the
    // centre Z the origin distance |o - Z| is measured from.
    std::vector<float> lmt;
    float mt_z[3] = {0.f, 0.f, 0.f};
    // Per shape, its class and conservative box (classify with origin_lim) as built, then
    // as prepare_animation last classified it (shapes written since the build): the refit's
    // fixed slot boxes reuse them (rt_kernels.hip prepare_animation; classifying 100k
    // shapes again took ~40 ms of a config-5 refit setup).
    std::vector<int> shape_cls;
    std::vector<Box3> shape_box;
};

// Builds the accelerator for a validated reference tree (see check_tree).
// leaf_threshold: leaves with more shapes than this get a local BVH.
bool build_accel(const FlatShape* shapes, int S, const FlatNode* nodes, int N, const int* idx, int I,
                 int leaf_threshold, int stack_cap, AccelHost& out, bool mt = false);

// Back-face cones of the local nodes (fills A.lcone; grazing cones when A.mt).
void build_cones(const FlatShape* shapes, AccelHost& A);

// fn(i0, i1) over [0, n) in contiguous chunks on the build threads (RTA_BUILD_THREADS,
// at most 16), each of at least min_per_thread items; the calling thread takes the
// first chunk. Exceptions reach the caller after every chunk ended.
void parallel_for(int n, int min_per_thread, const std::function<void(int, int)>& fn);

constexpr int kWide = 4;  // children per wide record (one 128-byte record of the barycentric accelerator)
// Children per wide node of the barycentric accelerators: 8 = two consecutive records
// tested at one step (half as many... log8 instead of log4 dependent node steps per
// descent), or 4. Moller-Trumbore accelerators stay at kWide.
#ifndef RT_WIDE8
#define RT_WIDE8 0
#endif
constexpr int kWideKids = RT_WIDE8 ? 2 * kWide : kWide;
// Cone threshold of a scene-tree node without a distance bound (SceneTree).
constexpr float kNoPrune = -8.0f;
// Stack entries the lane walk keeps per lane in LDS (6 B each: code + bf16
// entry parameter): 26 x 64 lanes x 6 B fits 16 waves per CU in 160 KB. The
// wide collapse stays within it wherever the binary tree allows.
#ifndef RT_LANE_STACK
#define RT_LANE_STACK 26
#endif
constexpr int kLaneStack = RT_LANE_STACK;

}  // namespace rta

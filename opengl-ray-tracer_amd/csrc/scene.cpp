// scene.cpp — host scene library: shapes, spatial-midpoint BVH, serialisers,
// benchmark scene generators. Product code (librtscene.so), C ABI in
// include/rt_scene.h.
//
// This restates the CPU half of the reference's hot path. Every rule that
// changes a serialised byte follows the reference exactly (citations inline):
// the tree must be the reference's tree, because traversal order decides ties
// and the spatial-midpoint builder decides which shapes a ray ever tests
// (SURVEY §8(a) A12). Build with -ffp-contract=off so every float matches
// the reference's IEEE sequence.
#include "../../include/rt_scene.h"

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

namespace {

struct V3 {
    float x = 0.f, y = 0.f, z = 0.f;  // glm 0.9.8 default ctor zero-initialises
    V3() = default;
    V3(float a, float b, float c) : x(a), y(b), z(c) {}
    explicit V3(const float* p) : x(p[0]), y(p[1]), z(p[2]) {}
    float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};
inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 operator-(V3 a) { return {-a.x, -a.y, -a.z}; }
inline V3 operator*(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline V3 operator*(float s, V3 a) { return {s * a.x, s * a.y, s * a.z}; }
inline V3 operator/(V3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
inline V3 operator+(V3 a, float s) { return {a.x + s, a.y + s, a.z + s}; }
inline V3 operator-(V3 a, float s) { return {a.x - s, a.y - s, a.z - s}; }
// glm semantics (glm/glm/detail/func_geometric.inl): dot = (x+y)+z, normalize =
// v * (1/sqrt(dot)), cross as written there.
inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3 cross(V3 a, V3 b) {
    return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y};
}
inline V3 normalize(V3 v) { return v * (1.0f / std::sqrt(dot(v, v))); }
inline float vmin(float a, float b) { return (b < a) ? b : a; }  // glm::min
inline float vmax(float a, float b) { return (a < b) ? b : a; }  // glm::max
inline rt_vec3 flat(V3 v) { return rt_vec3{v.x, v.y, v.z}; }

const float kDegToRad = static_cast<float>(0.01745329251994329576923690768489);   // glm::radians
const float kRadToDeg = static_cast<float>(57.295779513082320876798154814105);    // glm::degrees

// Material() defaults: the constructor's, not the in-class initialisers
// (src/material.hpp:23 overrides :13-16).
FlatMaterial default_material() {
    FlatMaterial m;
    std::memset(&m, 0, sizeof m);
    m.color = rt_vec3{1.f, 1.f, 1.f};
    m.fresnelStrength = 1.f;
    m.ambientStrength = 0.4f;
    m.diffuseStrength = 1.f;
    m.specularStrength = 0.5f;
    m.shininess = 32;
    return m;
}

// One tagged record instead of the reference's virtual Shape hierarchy.
struct Prim {
    int kind = RT_SPHERE;
    FlatMaterial mat = default_material();
    V3 p0, p1, p2;      // sphere centre | plane point | wall start | triangle a,b,c
    float radius = 0.f; // sphere
    V3 normal;          // plane/wall/triangle m_normal
    float d = 0.f;      // plane/wall/triangle d
    float width = 0.f, height = 0.f;  // wall

    // Plane(normal, point) (src/shapes/plane.hpp:28-33).
    void set_plane(V3 n, V3 point) {
        normal = normalize(n);
        d = -dot(normal, point);
    }
    // Wall::end() (src/shapes/wall.hpp:16-31): a different tangent basis from
    // the one the wall intersection uses.
    V3 wall_end() const {
        V3 t1;
        if (std::fabs(normal.x) > std::fabs(normal.y))
            t1 = normalize(V3(-normal.z, 0.f, normal.x));
        else
            t1 = normalize(V3(0.f, -normal.z, normal.y));
        V3 t2 = normalize(cross(normal, t1));
        return p0 + (width * t1) + (height * t2);
    }
    // Centre used by split() (src/main.cpp:1127-1140); a plane keeps the
    // zero-initialised vec3.
    V3 split_centre() const {
        switch (kind) {
            case RT_SPHERE: return p0;
            case RT_WALL: return (p0 + wall_end()) * 0.5f;
            case RT_TRIANGLE: return (p0 + p1 + p2) / 3.0f;
            default: return V3();
        }
    }
};

// BoundingBox (src/BoundingBox.hpp:7-95).
struct Box {
    V3 lo{INFINITY, INFINITY, INFINITY};
    V3 hi{-INFINITY, -INFINITY, -INFINITY};
    void grow(V3 p) {
        lo = V3(vmin(lo.x, p.x), vmin(lo.y, p.y), vmin(lo.z, p.z));
        hi = V3(vmax(hi.x, p.x), vmax(hi.y, p.y), vmax(hi.z, p.z));
    }
    // growToInclude(unique_ptr<Shape>&) dispatch (:87-95): planes add nothing.
    void grow(const Prim& s) {
        switch (s.kind) {
            case RT_SPHERE:
                grow(s.p0 + s.radius);
                grow(s.p0 - s.radius);
                break;
            case RT_WALL:
                grow(s.p0);
                grow(s.wall_end());
                break;
            case RT_TRIANGLE:
                // Only the x components are checked (:52-64).
                if (std::isfinite(s.p0.x) && std::isfinite(s.p1.x) && std::isfinite(s.p2.x)) {
                    grow(s.p0);
                    grow(s.p1);
                    grow(s.p2);
                } else {
                    std::fprintf(stderr, "rtscene: triangle with non-finite vertices left out of its box\n");
                }
                break;
            default:
                break;
        }
    }
    V3 centre() const { return (lo + hi) * 0.5f; }
};

struct TreeNode {
    Box box;
    int left = -1, right = -1;
    std::vector<int> prims;
};

struct Cam {
    V3 position, front{0.f, 0.f, -1.f}, up, right, world_up{0.f, 1.f, 0.f};
    float yaw = -90.f, pitch = 0.f, fov = 60.f, aspect = 1.f;
    Cam() { update(); }
    // updateCameraVectors (src/camera.hpp:152-163).
    void update() {
        V3 f(std::cos(yaw * kDegToRad) * std::cos(pitch * kDegToRad), std::sin(pitch * kDegToRad),
             std::sin(yaw * kDegToRad) * std::cos(pitch * kDegToRad));
        front = normalize(f);
        right = normalize(cross(front, world_up));
        up = normalize(cross(right, front));
    }
    // LookAt (src/camera.hpp:139-148).
    void look_at(V3 target) {
        V3 dir = normalize(target - position);
        pitch = std::asin(dir.y) * kRadToDeg;
        yaw = std::atan2(dir.z, dir.x) * kRadToDeg;
        update();
    }
};

}  // namespace

struct rts_scene {
    std::vector<Prim> prims;
    std::vector<TreeNode> nodes;  // post-order, root last (src/main.cpp:1163-1190)
    Cam cam;
    V3 light_pos, light_color{1.f, 1.f, 1.f};

    int add(const Prim& p) {
        prims.push_back(p);
        return static_cast<int>(prims.size()) - 1;
    }

    // split (src/main.cpp:1111-1173).
    void split(TreeNode& parent, int depth) {
        if (depth <= 0) {
            parent.left = parent.right = -1;
            return;
        }
        V3 size = parent.box.hi - parent.box.lo;
        int axis = size.x > vmax(size.y, size.z) ? 0 : (size.y > size.z ? 1 : 2);
        float split_pos = parent.box.centre()[axis];

        TreeNode lnode, rnode;
        for (int idx : parent.prims) {
            const Prim& s = prims[idx];
            TreeNode& side = (s.split_centre()[axis] < split_pos) ? lnode : rnode;
            side.box.grow(s);
            side.prims.push_back(idx);
        }
        if (lnode.prims.empty() || rnode.prims.empty()) {
            parent.left = parent.right = -1;
            return;
        }
        split(lnode, depth - 1);
        split(rnode, depth - 1);
        nodes.push_back(std::move(lnode));
        parent.left = static_cast<int>(nodes.size()) - 1;
        nodes.push_back(std::move(rnode));
        parent.right = static_cast<int>(nodes.size()) - 1;
    }

    // buildBVH (src/main.cpp:1175-1193).
    void build(int max_depth) {
        nodes.clear();
        TreeNode root;
        for (int i = 0; i < static_cast<int>(prims.size()); ++i) {
            root.box.grow(prims[i]);
            root.prims.push_back(i);
        }
        split(root, max_depth);
        nodes.push_back(std::move(root));
    }

    int index_count() const {
        int n = 0;
        for (const auto& nd : nodes)
            if (nd.left == -1) n += static_cast<int>(nd.prims.size());
        return n;
    }

    // serializeShape (src/main.cpp:994-1066); fields the type does not use stay 0.
    void serialize_shape(const Prim& s, FlatShape& out) const {
        std::memset(&out, 0, sizeof out);
        out.type = s.kind;
        out.material = s.mat;
        switch (s.kind) {
            case RT_SPHERE:
                out.sphereCenter = flat(s.p0);
                out.sphereRadius = s.radius;
                break;
            case RT_WALL:
                out.planeNormal = flat(s.normal);
                out.planeD = s.d;
                out.wallStart = flat(s.p0);
                out.wallWidth = s.width;
                out.wallHeight = s.height;
                break;
            case RT_TRIANGLE:
                out.planeNormal = flat(s.normal);
                out.planeD = s.d;
                out.triP1 = flat(s.p0);
                out.triP2 = flat(s.p1);
                out.triP3 = flat(s.p2);
                break;
            default:  // plane
                out.planeNormal = flat(s.normal);
                out.planeD = s.d;
                break;
        }
    }
};

namespace {

FlatMaterial mat_or_default(const FlatMaterial* m) { return m ? *m : default_material(); }

Prim make_triangle(V3 a, V3 b, V3 c) {
    // Triangle(p1,p2,p3) : Plane(get_normal(p1,p2,p3), p1) (src/shapes/triangle.hpp:46-47,84-93).
    Prim t;
    t.kind = RT_TRIANGLE;
    t.p0 = a;
    t.p1 = b;
    t.p2 = c;
    V3 A = b - a, B = c - a;
    V3 n(A.y * B.z - A.z * B.y, A.z * B.x - A.x * B.z, A.x * B.y - A.y * B.x);
    t.set_plane(n, a);
    return t;
}

void invert(Prim& t) {  // Triangle::invert_normal (src/shapes/triangle.hpp:95-98)
    t.normal = -t.normal;
    t.d = -dot(t.normal, t.p0);
}

int add_mesh(rts_scene* s, const float* v, int nv, const unsigned* idx, int ni, const float* origin,
             const FlatMaterial* mat, bool oriented) {
    if (!s || (!v && nv > 0) || (!idx && ni > 0) || nv < 0 || ni < 0 || ni % 3 != 0) return -1;
    for (int i = 0; i < ni; ++i)
        if (idx[i] >= static_cast<unsigned>(nv)) return -1;
    V3 org = origin ? V3(origin) : V3();
    // Mesh::center (src/mesh.hpp:51-61): the origin is counted n+1 times.
    V3 centre = org;
    for (int i = 0; i < nv; ++i) centre = centre + (org + V3(v + 3 * i));
    centre = centre / static_cast<float>(nv);
    int first = static_cast<int>(s->prims.size());
    FlatMaterial m = mat_or_default(mat);
    for (int i = 0; i < ni; i += 3) {
        V3 a = V3(v + 3 * idx[i]) + org, b = V3(v + 3 * idx[i + 1]) + org, c = V3(v + 3 * idx[i + 2]) + org;
        Prim t = make_triangle(a, b, c);
        // mesh2triangles flips triangles "facing the centre" (src/mesh.hpp:178-184).
        // generateScene1/2 rebuild each triangle from its vertices
        // (src/main.cpp:654,671,763), which drops that flip: oriented=false.
        if (oriented && dot(t.normal, centre) > 0.0f) invert(t);
        t.mat = m;
        s->add(t);
    }
    return first;
}

// ---------------------------------------------------------------------------
// Benchmark scene stand-ins. The reference's meshes are not in
// the repository (.gitignore:78), so meshes are generated procedurally with the
// published triangle counts; every other constant is the reference scene's.

// Deterministic uniform float in [lo, hi): 24 random bits of std::mt19937
// (a standardised engine), so every libstdc++ gives the same scene.
struct Rng {
    std::mt19937 g;
    explicit Rng(unsigned seed) : g(seed) {}
    float u01() { return static_cast<float>(g() >> 8) * (1.0f / 16777216.0f); }
    float uni(float lo, float hi) { return lo + (hi - lo) * u01(); }
};

struct MeshBuf {
    std::vector<float> v;
    std::vector<unsigned> i;
    unsigned vert(V3 p) {
        v.push_back(p.x);
        v.push_back(p.y);
        v.push_back(p.z);
        return static_cast<unsigned>(v.size() / 3 - 1);
    }
    void tri(unsigned a, unsigned b, unsigned c) {
        i.push_back(a);
        i.push_back(b);
        i.push_back(c);
    }
};

// Closed latitude/longitude surface around the y axis: pole fans plus quads;
// 2*slices*(stacks-1) triangles, outward counter-clockwise winding (as an OBJ
// export would have). `radius(theta, phi)` scales a unit sphere per vertex.
template <class F>
MeshBuf lat_long(int slices, int stacks, V3 semi, F radius) {
    MeshBuf m;
    const float pi = 3.14159265358979f;
    unsigned top = m.vert(V3(0.f, -semi.y * radius(0.f, 0.f), 0.f));
    std::vector<unsigned> ring_start;
    for (int st = 1; st < stacks; ++st) {
        float th = pi * static_cast<float>(st) / static_cast<float>(stacks);
        ring_start.push_back(static_cast<unsigned>(m.v.size() / 3));
        for (int sl = 0; sl < slices; ++sl) {
            float ph = 2.f * pi * static_cast<float>(sl) / static_cast<float>(slices);
            float r = radius(th, ph);
            m.vert(V3(semi.x * r * std::sin(th) * std::cos(ph), -semi.y * r * std::cos(th),
                      semi.z * r * std::sin(th) * std::sin(ph)));
        }
    }
    unsigned bottom = m.vert(V3(0.f, semi.y * radius(pi, 0.f), 0.f));
    auto at = [&](int ring, int sl) { return ring_start[ring] + static_cast<unsigned>(sl % slices); };
    for (int sl = 0; sl < slices; ++sl) m.tri(top, at(0, sl + 1), at(0, sl));
    for (int r = 0; r + 1 < stacks - 1; ++r)
        for (int sl = 0; sl < slices; ++sl) {
            m.tri(at(r, sl), at(r, sl + 1), at(r + 1, sl + 1));
            m.tri(at(r, sl), at(r + 1, sl + 1), at(r + 1, sl));
        }
    for (int sl = 0; sl < slices; ++sl) m.tri(bottom, at(stacks - 2, sl), at(stacks - 2, sl + 1));
    return m;
}

// Wheel: cylinder around the z axis, `seg` segments, 4*seg triangles.
MeshBuf wheel(V3 c, float r, float half_w, int seg) {
    MeshBuf m;
    const float pi = 3.14159265358979f;
    unsigned cf = m.vert(V3(c.x, c.y, c.z + half_w)), cb = m.vert(V3(c.x, c.y, c.z - half_w));
    unsigned f0 = static_cast<unsigned>(m.v.size() / 3);
    for (int k = 0; k < seg; ++k) {
        float a = 2.f * pi * static_cast<float>(k) / static_cast<float>(seg);
        m.vert(V3(c.x + r * std::cos(a), c.y + r * std::sin(a), c.z + half_w));
        m.vert(V3(c.x + r * std::cos(a), c.y + r * std::sin(a), c.z - half_w));
    }
    auto F = [&](int k) { return f0 + 2u * static_cast<unsigned>(k % seg); };
    auto B = [&](int k) { return f0 + 2u * static_cast<unsigned>(k % seg) + 1u; };
    for (int k = 0; k < seg; ++k) {
        m.tri(cf, F(k), F(k + 1));
        m.tri(cb, B(k + 1), B(k));
        m.tri(F(k), B(k), B(k + 1));
        m.tri(F(k), B(k + 1), F(k + 1));
    }
    return m;
}

FlatMaterial material(V3 color, float fresnel, float ambient, float diffuse, float specular) {
    FlatMaterial m = default_material();
    m.color = flat(color);
    m.fresnelStrength = fresnel;
    m.ambientStrength = ambient;
    m.diffuseStrength = diffuse;
    m.specularStrength = specular;
    return m;
}

const unsigned kSeed = 20250620u;

// Spheres of generateScene1 (src/main.cpp:594-623), in order.
void scene1_spheres(rts_scene* s) {
    const float c0[3] = {0.f, 10.f, -8.f}, c1[3] = {12.f, 10.f, -8.f}, c2[3] = {20.f, 7.5f, -8.f},
                c3[3] = {0.f, 23.f, -8.f};
    FlatMaterial m0 = material(V3(0.f, 0.37f, 0.f), 0.f, 0.2f, 1.f, 0.1f);
    FlatMaterial m1 = material(V3(0.58f, 0.18f, 0.48f), 0.f, 0.f, 0.5f, 0.f);
    FlatMaterial m2 = material(V3(0.8f, 0.2f, 0.8f), 1.f, 0.06f, 0.06f, 0.5f);
    FlatMaterial m3 = material(V3(0.f, 0.37f, 0.f), 0.f, 0.f, 0.5f, 0.f);
    rts_add_sphere(s, c0, 5.f, &m0);
    rts_add_sphere(s, c1, 4.f, &m1);
    rts_add_sphere(s, c2, 2.5f, &m2);
    rts_add_sphere(s, c3, 1.5f, &m3);
}

// Config 1: the spheres above + one Plane(normal (0,1,0), point (0,25,0)).
void gen_spheres(rts_scene* s, float aspect) {
    scene1_spheres(s);
    const float n[3] = {0.f, 1.f, 0.f}, p[3] = {0.f, 25.f, 0.f};
    rts_add_plane(s, n, p, nullptr);
    const float cam[3] = {30.f, -5.f, 40.f}, lp[3] = {0.f, -14.f, 0.f}, white[3] = {1.f, 1.f, 1.f};
    const float tgt[3] = {0.f, 10.f, -8.f};
    rts_set_camera(s, cam, 60.f, aspect);
    rts_set_light(s, lp, white, 50.f);
    rts_camera_look_at(s, tgt);
    s->build(15);
}

// Config 2: generateScene1 (src/main.cpp:583-716) with procedural "monkey" blobs.
void gen_monkey(rts_scene* s, float aspect) {
    Rng rng(kSeed);
    const float cam[3] = {30.f, -5.f, 40.f}, lp[3] = {0.f, -14.f, 0.f}, white[3] = {1.f, 1.f, 1.f};
    rts_set_camera(s, cam, 60.f, aspect);
    rts_set_light(s, lp, white, 50.f);
    scene1_spheres(s);
    // mirror wall (:625-630)
    const float ws[3] = {-15.f, 23.f, 10.f}, wn[3] = {-1.f, 0.2f, 0.f};
    FlatMaterial mw = material(V3(1.f, 1.f, 1.f), 1.f, 0.1f, 0.f, 1.f);
    rts_add_wall(s, ws, 30.f, 20.f, wn, &mw);
    // inverted triangle (:632-643)
    const float p1[3] = {-15.f, 20.f, 25.f}, p2[3] = {-12.f, 20.f, 10.f}, p3[3] = {-15.f, 0.f, 20.f};
    FlatMaterial mt = material(V3(0.19f, 0.66f, 0.32f), 1.f, 0.06f, 0.06f, 0.5f);
    rts_add_triangle(s, p1, p2, p3, 1, &mt);
    // "monkey.obj" stand-in: 968 triangles at (0,0,-30); "lowpolymonkey.obj": 240 at (50,0,-30).
    auto bumpy = [](float th, float ph) { return 1.f + 0.12f * std::sin(3.f * th) * std::cos(2.f * ph); };
    MeshBuf big = lat_long(22, 23, V3(8.f, 7.f, 6.f), bumpy);
    MeshBuf low = lat_long(12, 11, V3(8.f, 7.f, 6.f), bumpy);
    const float o1[3] = {0.f, 0.f, -30.f}, o2[3] = {50.f, 0.f, -30.f};
    FlatMaterial mm1 = material(V3(179.f / 255, 165.f / 255, 61.f / 255), 1.f, 0.2f, 0.8f, 0.1f);
    FlatMaterial mm2 = material(V3(0.f, 1.f, 0.9f), 1.f, 0.2f, 0.8f, 0.f);
    rts_add_mesh(s, big.v.data(), static_cast<int>(big.v.size() / 3), big.i.data(),
                 static_cast<int>(big.i.size()), o1, &mm1);
    rts_add_mesh(s, low.v.data(), static_cast<int>(low.v.size() / 3), low.i.data(),
                 static_cast<int>(low.i.size()), o2, &mm2);
    // 25 random spheres (:685-696)
    for (int i = 0; i < 25; ++i) {
        float x = rng.uni(-40.f, 40.f), z = rng.uni(-40.f, 40.f);
        FlatMaterial m = default_material();
        m.color.x = rng.u01();
        m.color.y = rng.u01();
        m.color.z = rng.u01();
        const float c[3] = {x, 23.f, z};
        rts_add_sphere(s, c, 1.5f, &m);
    }
    // floor (:699-701)
    const float fs[3] = {-100.f, 25.f, -100.f}, fn[3] = {0.f, 1.f, 0.f};
    FlatMaterial mf = default_material();
    mf.color = rt_vec3{0.65f, 0.17f, 0.35f};
    mf.specularStrength = 0.f;
    rts_add_wall(s, fs, 210.f, 210.f, fn, &mf);
    const float tgt[3] = {0.f, 10.f, -8.f};
    rts_camera_look_at(s, tgt);
    s->build(15);
}

// Config 3: generateScene2 (src/main.cpp:718-804) with a procedural car: body
// (3,380 triangles), four wheels (160 each), road (2 triangles, or 222 strips
// for variant 1): 4,022 triangles, then 100 spheres.
void gen_car(rts_scene* s, int variant, float aspect) {
    Rng rng(kSeed);
    const float cam[3] = {0.f, -10.f, 40.f}, lp[3] = {14.8f, -17.f, 17.f}, white[3] = {1.f, 1.f, 1.f};
    rts_set_camera(s, cam, 60.f, aspect);
    rts_set_light(s, lp, white, 26.f);
    const float origin[3] = {0.f, 0.f, 0.f};
    // +y points down the screen in the reference (row 0 = +Up, shown at the
    // bottom of the GL texture), so the car stands on y = 0 at negative y.
    auto body_r = [](float th, float ph) {
        // cabin bump on the upper half, flattened floor
        float bump = 1.f + 0.35f * std::fmax(0.f, -std::cos(th)) * std::exp(-2.f * std::cos(ph) * std::cos(ph));
        return bump;
    };
    MeshBuf body = lat_long(65, 27, V3(9.f, 1.8f, 3.6f), body_r);
    for (size_t k = 1; k < body.v.size(); k += 3) body.v[k] -= 3.4f;
    std::vector<MeshBuf> meshes;
    meshes.push_back(body);
    const float wx = 5.6f, wz = 3.7f, wr = 1.6f;
    meshes.push_back(wheel(V3(-wx, -wr, wz), wr, 0.45f, 40));
    meshes.push_back(wheel(V3(wx, -wr, wz), wr, 0.45f, 40));
    meshes.push_back(wheel(V3(-wx, -wr, -wz), wr, 0.45f, 40));
    meshes.push_back(wheel(V3(wx, -wr, -wz), wr, 0.45f, 40));
    MeshBuf road;
    if (variant == 1) {
        // 111 strips across x, two triangles each
        const int strips = 111;
        for (int k = 0; k <= strips; ++k) {
            float x = -55.f + 110.f * static_cast<float>(k) / static_cast<float>(strips);
            road.vert(V3(x, 0.f, -20.f));
            road.vert(V3(x, 0.f, 20.f));
        }
        for (unsigned k = 0; k < static_cast<unsigned>(strips); ++k) {
            unsigned a = 2 * k, b = 2 * k + 1, c = 2 * k + 2, d = 2 * k + 3;
            road.tri(a, b, d);  // normal (0,+1,0): INNER for rays heading +y
            road.tri(a, d, c);
        }
    } else {
        unsigned a = road.vert(V3(-55.f, 0.f, -20.f)), b = road.vert(V3(55.f, 0.f, -20.f)),
                 c = road.vert(V3(55.f, 0.f, 20.f)), d = road.vert(V3(-55.f, 0.f, 20.f));
        road.tri(a, c, b);  // normal (0,+1,0)
        road.tri(a, d, c);
    }
    meshes.push_back(road);
    for (size_t i = 0; i < meshes.size(); ++i) {
        FlatMaterial m = default_material();  // (:733-752)
        if (i == 0) {
            m.color = rt_vec3{19.f / 255, 7.f / 255, 92.f / 255};
            m.specularStrength = 0.f;
        } else if (i <= 4) {
            m.color = rt_vec3{0.2f, 0.2f, 0.2f};
            m.specularStrength = 0.f;
        } else {
            m.color = rt_vec3{0.f, 0.f, 0.f};
            m.specularStrength = 0.25f;
        }
        const MeshBuf& mb = meshes[i];
        rts_add_mesh(s, mb.v.data(), static_cast<int>(mb.v.size() / 3), mb.i.data(),
                     static_cast<int>(mb.i.size()), origin, &m);
    }
    // 100 background spheres (:788-795)
    for (int i = 0; i < 100; ++i) {
        float x = rng.uni(-30.f, 30.f), y = rng.uni(-15.f, 0.f);
        FlatMaterial m = default_material();
        m.color.x = rng.u01();
        m.color.y = rng.u01();
        m.color.z = rng.u01();
        const float c[3] = {x, y, -10.f};
        rts_add_sphere(s, c, 1.5f, &m);
    }
    rts_camera_look_at(s, origin);
    s->build(25);
}

// Config 5: 100,000 random triangles, centres U(-20,20)^3, vertices at
// centre + U(-0.5,0.5)^3, seed 7, default materials, buildBVH(25).
void gen_random(rts_scene* s, float aspect) {
    Rng rng(7u);
    const float cam[3] = {0.f, -10.f, 60.f}, lp[3] = {0.f, -40.f, 40.f}, white[3] = {1.f, 1.f, 1.f};
    rts_set_camera(s, cam, 60.f, aspect);
    rts_set_light(s, lp, white, 60.f);
    s->prims.reserve(100000);
    for (int i = 0; i < 100000; ++i) {
        V3 c(rng.uni(-20.f, 20.f), rng.uni(-20.f, 20.f), rng.uni(-20.f, 20.f));
        V3 v[3];
        for (int k = 0; k < 3; ++k)
            v[k] = c + V3(rng.uni(-0.5f, 0.5f), rng.uni(-0.5f, 0.5f), rng.uni(-0.5f, 0.5f));
        Prim t = make_triangle(v[0], v[1], v[2]);
        s->add(t);
    }
    const float origin[3] = {0.f, 0.f, 0.f};
    rts_camera_look_at(s, origin);
    s->build(25);
}

// The reference's default scene (`int SCENE = 3`, src/main.cpp:46): generateScene3
// (:1196-1229) -- Camera() at (0,-10,40) with the window's aspect, the scene-2 light,
// ONE Triangle((0,0,0), (5,0,0), (2.5,-5,0)) with the Material() defaults, LookAt
// the origin. It never calls buildBVH: no nodes and no bvhIndices are serialised,
// so the GLSL's BVH branch would start from bvhNodes[-1] (gpu_shader.comp:386).
void gen_triangle(rts_scene* s, float aspect) {
    const float cam[3] = {0.f, -10.f, 40.f}, lp[3] = {14.8f, -17.f, 17.f}, white[3] = {1.f, 1.f, 1.f};
    rts_set_camera(s, cam, 60.f, aspect);  // Camera() default fov (src/camera.hpp:50)
    rts_set_light(s, lp, white, 26.f);
    const float a[3] = {0.f, 0.f, 0.f}, b[3] = {5.f, 0.f, 0.f}, c[3] = {2.5f, -5.f, 0.f};
    rts_add_triangle(s, a, b, c, 0, nullptr);
    rts_camera_look_at(s, a);
}

}  // namespace

extern "C" {

rts_scene* rts_new(void) { return new (std::nothrow) rts_scene(); }
void rts_free(rts_scene* s) { delete s; }
int rts_clear(rts_scene* s) {
    if (!s) return -1;
    *s = rts_scene();
    return 0;
}

int rts_add_sphere(rts_scene* s, const float* center, float radius, const FlatMaterial* mat) {
    if (!s || !center) return -1;
    Prim p;  // Sphere(center, radius) (src/shapes/sphere.hpp:28-33)
    p.kind = RT_SPHERE;
    p.p0 = V3(center);
    p.radius = radius;
    p.mat = mat_or_default(mat);
    return s->add(p);
}

int rts_add_plane(rts_scene* s, const float* normal, const float* point, const FlatMaterial* mat) {
    if (!s || !normal || !point) return -1;
    Prim p;
    p.kind = RT_PLANE;
    p.p0 = V3(point);
    p.set_plane(V3(normal), V3(point));
    p.mat = mat_or_default(mat);
    return s->add(p);
}

int rts_add_wall(rts_scene* s, const float* start, float width, float height, const float* normal,
                 const FlatMaterial* mat) {
    if (!s || !start || !normal) return -1;
    Prim p;  // Wall(s, w, h, normal) : Plane(normal, s) (src/shapes/wall.hpp:37-40)
    p.kind = RT_WALL;
    p.p0 = V3(start);
    p.width = width;
    p.height = height;
    p.set_plane(V3(normal), V3(start));
    p.mat = mat_or_default(mat);
    return s->add(p);
}

int rts_add_triangle(rts_scene* s, const float* a, const float* b, const float* c, int inv,
                     const FlatMaterial* mat) {
    if (!s || !a || !b || !c) return -1;
    Prim t = make_triangle(V3(a), V3(b), V3(c));
    if (inv) invert(t);
    t.mat = mat_or_default(mat);
    return s->add(t);
}

int rts_add_mesh(rts_scene* s, const float* v, int nv, const unsigned* idx, int ni, const float* origin,
                 const FlatMaterial* mat) {
    return add_mesh(s, v, nv, idx, ni, origin, mat, false);
}

int rts_add_mesh_oriented(rts_scene* s, const float* v, int nv, const unsigned* idx, int ni,
                          const float* origin, const FlatMaterial* mat) {
    return add_mesh(s, v, nv, idx, ni, origin, mat, true);
}

// ---------------------------------------------------------------------------
// Wavefront OBJ ingestion (replaces assimp's loader,
// src/model.hpp:49-168). Vertex positions ("v x y z [w]") and faces
// ("f a b c ...", each corner "i", "i/t", "i//n" or "i/t/n"; negative indices
// count back from the last vertex read) are kept; texture coordinates, normals,
// groups, objects and materials are ignored, as they do not reach the ray
// tracer's FlatShape records. A face of k corners becomes the fan
// (0,1,2), (0,2,3), ..., (0,k-2,k-1), aiProcess_Triangulate's split of a convex
// polygon. The whole file is one mesh: Mesh::mesh2triangles with `origin`
// added to every vertex (src/mesh.hpp:163-189), and the normal flip applied
// only if `oriented` (generateScene1/2 drop it, see add_mesh).
namespace {

int parse_obj(rts_scene* s, const char* text, size_t len, const float* origin, const FlatMaterial* mat, bool oriented) {
    std::vector<float> v;
    std::vector<unsigned> idx;
    std::vector<long> face;
    size_t pos = 0;
    int line_no = 0;
    while (pos < len) {
        size_t end = pos;
        while (end < len && text[end] != '\n') ++end;
        std::string line(text + pos, end - pos);
        pos = end + 1;
        ++line_no;
        if (!line.empty() && line.back() == '\r') line.pop_back();
        const char* c = line.c_str();
        while (*c == ' ' || *c == '\t') ++c;
        if (c[0] == 'v' && (c[1] == ' ' || c[1] == '\t')) {
            char* e = nullptr;
            float xyz[3];
            const char* q = c + 2;
            for (int k = 0; k < 3; ++k) {
                errno = 0;
                xyz[k] = std::strtof(q, &e);
                if (e == q || errno == ERANGE) return -3;
                q = e;
            }
            v.insert(v.end(), xyz, xyz + 3);
        } else if (c[0] == 'f' && (c[1] == ' ' || c[1] == '\t')) {
            face.clear();
            const char* q = c + 2;
            const long nv = static_cast<long>(v.size() / 3);
            for (;;) {
                while (*q == ' ' || *q == '\t') ++q;
                if (!*q) break;
                char* e = nullptr;
                const long i = std::strtol(q, &e, 10);
                if (e == q) return -3;
                const long r = i > 0 ? i - 1 : nv + i;  // 1-based, or relative to the last vertex
                if (i == 0 || r < 0 || r >= nv) return -3;
                face.push_back(r);
                q = e;
                while (*q && *q != ' ' && *q != '\t') ++q;  // skip "/t/n"
            }
            if (face.size() < 3) return -3;
            for (size_t k = 1; k + 1 < face.size(); ++k) {
                idx.push_back(static_cast<unsigned>(face[0]));
                idx.push_back(static_cast<unsigned>(face[k]));
                idx.push_back(static_cast<unsigned>(face[k + 1]));
            }
        }
    }
    if (idx.empty()) return 0;
    const int first = add_mesh(s, v.data(), static_cast<int>(v.size() / 3), idx.data(), static_cast<int>(idx.size()),
                               origin, mat, oriented);
    return first < 0 ? first : static_cast<int>(idx.size() / 3);
}

}  // namespace

int rts_parse_obj(rts_scene* s, const char* text, long len, const float* origin, const FlatMaterial* mat,
                  int oriented) {
    if (!s || (!text && len > 0) || len < 0) return -1;
    return parse_obj(s, text, static_cast<size_t>(len), origin, mat, oriented != 0);
}

int rts_load_obj(rts_scene* s, const char* path, const float* origin, const FlatMaterial* mat, int oriented) {
    if (!s || !path) return -1;
    FILE* f = std::fopen(path, "rb");
    if (!f) return -2;
    std::string text;
    char buf[1 << 16];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) text.append(buf, n);
    const bool err = std::ferror(f) != 0;
    std::fclose(f);
    if (err) return -2;
    return parse_obj(s, text.data(), text.size(), origin, mat, oriented != 0);
}

// ---------------------------------------------------------------------------
// Image dump (replaces the screen quad, src/main.cpp:476-501,
// shader.frag, which shows the RGBA32F texture's rgb). Rows are written in
// image order, row 0 first = NDC y +1, the top of the camera's view.
// RTS_IMAGE_PPM: binary P6, each channel clamped to [0, 1] and rounded to 8 bits.
// RTS_IMAGE_PFM: colour PFM ("PF"), the float rgb exactly; PFM stores the
// bottom row first, so the file's first row is image row h-1.
int rts_write_image(const char* path, const float* rgba, int w, int h, long pitch_bytes, int format) {
    if (!path || !rgba || w <= 0 || h <= 0 || pitch_bytes < 16L * w || (format != RTS_IMAGE_PPM && format != RTS_IMAGE_PFM))
        return -1;
    FILE* f = std::fopen(path, "wb");
    if (!f) return -2;
    bool ok = true;
    auto row = [&](int y) { return reinterpret_cast<const float*>(reinterpret_cast<const char*>(rgba) + y * pitch_bytes); };
    if (format == RTS_IMAGE_PPM) {
        ok = std::fprintf(f, "P6\n%d %d\n255\n", w, h) > 0;
        std::vector<unsigned char> line(3 * static_cast<size_t>(w));
        for (int y = 0; y < h && ok; ++y) {
            const float* r = row(y);
            for (int x = 0; x < w; ++x)
                for (int k = 0; k < 3; ++k) {
                    float c = r[4 * x + k];
                    c = c > 0.f ? (c < 1.f ? c : 1.f) : 0.f;  // NaN -> 0
                    line[3 * x + k] = static_cast<unsigned char>(std::lround(c * 255.f));
                }
            ok = std::fwrite(line.data(), 1, line.size(), f) == line.size();
        }
    } else {
        ok = std::fprintf(f, "PF\n%d %d\n-1.0\n", w, h) > 0;  // negative scale: little endian
        std::vector<float> line(3 * static_cast<size_t>(w));
        for (int y = h - 1; y >= 0 && ok; --y) {
            const float* r = row(y);
            for (int x = 0; x < w; ++x)
                for (int k = 0; k < 3; ++k) line[3 * x + k] = r[4 * x + k];
            ok = std::fwrite(line.data(), sizeof(float), line.size(), f) == line.size();
        }
    }
    ok = (std::fclose(f) == 0) && ok;
    return ok ? 0 : -2;
}

int rts_set_camera(rts_scene* s, const float* position, float fov_deg, float aspect) {
    if (!s || !position) return -1;
    s->cam = Cam();
    s->cam.position = V3(position);
    s->cam.fov = fov_deg;
    s->cam.aspect = aspect;
    return 0;
}

int rts_camera_look_at(rts_scene* s, const float* target) {
    if (!s || !target) return -1;
    s->cam.look_at(V3(target));
    return 0;
}

int rts_set_light(rts_scene* s, const float* position, const float* color, float intensity) {
    if (!s || !position) return -1;
    s->light_pos = V3(position);
    V3 base = color ? V3(color) : V3(1.f, 1.f, 1.f);
    s->light_color = intensity * base;  // Light::updateColor (src/light.hpp:32-35)
    return 0;
}

int rts_build_bvh(rts_scene* s, int max_depth) {
    if (!s) return -1;
    s->build(max_depth);
    return 0;
}

int rts_counts(const rts_scene* s, int* ns, int* nn, int* ni) {
    if (!s) return -1;
    if (ns) *ns = static_cast<int>(s->prims.size());
    if (nn) *nn = static_cast<int>(s->nodes.size());
    if (ni) *ni = s->index_count();
    return 0;
}

int rts_serialize(const rts_scene* s, FlatShape* shapes, FlatNode* nodes, int* indices, FlatCamera* camera,
                  FlatLight* light) {
    if (!s) return -1;
    if (shapes)
        for (size_t i = 0; i < s->prims.size(); ++i) s->serialize_shape(s->prims[i], shapes[i]);
    // serializeBVH (src/main.cpp:955-979): startShapeIdx = running index count,
    // numShapes = the node's list length (also for inner nodes).
    if (nodes || indices) {
        int cursor = 0;
        for (size_t k = 0; k < s->nodes.size(); ++k) {
            const TreeNode& nd = s->nodes[k];
            if (nodes) {
                FlatNode& f = nodes[k];
                std::memset(&f, 0, sizeof f);
                f.boundsMin = flat(nd.box.lo);
                f.boundsMax = flat(nd.box.hi);
                f.leftChild = nd.left;
                f.rightChild = nd.right;
                f.startShapeIdx = cursor;
                f.numShapes = static_cast<int>(nd.prims.size());
            }
            if (nd.left == -1) {
                for (int idx : nd.prims) {
                    if (indices) indices[cursor] = idx;
                    ++cursor;
                }
            }
        }
    }
    if (camera) {  // serializeCamera (src/main.cpp:806-816)
        std::memset(camera, 0, sizeof *camera);
        camera->Position = flat(s->cam.position);
        camera->aspectRatio = s->cam.aspect;
        camera->Front = flat(s->cam.front);
        camera->Up = flat(s->cam.up);
        camera->Right = flat(s->cam.right);
        camera->fov = s->cam.fov;
    }
    if (light) {  // serializeLight (src/main.cpp:818-823)
        std::memset(light, 0, sizeof *light);
        light->position = flat(s->light_pos);
        light->color = flat(s->light_color);
    }
    return 0;
}

int rts_bvh_stats(const rts_scene* s, int* leaves, int* max_leaf, int* depth, int* max_stack) {
    if (!s) return -1;
    int nl = 0, ml = 0, dp = 0, ms = 0;
    const int n = static_cast<int>(s->nodes.size());
    if (n > 0) {
        // The reference walk with every box hit: push root; pop; inner pushes left, right.
        std::vector<std::pair<int, int>> st;
        st.push_back({n - 1, 1});
        ms = 1;
        while (!st.empty()) {
            auto [k, d] = st.back();
            st.pop_back();
            const TreeNode& nd = s->nodes[k];
            dp = d > dp ? d : dp;
            if (nd.left == -1) {
                ++nl;
                int sz = static_cast<int>(nd.prims.size());
                ml = sz > ml ? sz : ml;
            } else {
                st.push_back({nd.left, d + 1});
                st.push_back({nd.right, d + 1});
                ms = static_cast<int>(st.size()) > ms ? static_cast<int>(st.size()) : ms;
            }
        }
    }
    if (leaves) *leaves = nl;
    if (max_leaf) *max_leaf = ml;
    if (depth) *depth = dp;
    if (max_stack) *max_stack = ms;
    return 0;
}

// updateBVH (src/main.cpp:1068-1077) on the serialised arrays. A node's shape set
// is the shapes of the leaves below it; split() hands every child its parent's
// list filtered in order, so every list is in increasing shape index, and a node
// grows by its animated shapes in that order (growToInclude keeps the first of
// equal values, so the order can decide the sign of a zero).
int rts_update_bvh(const FlatShape* shapes, int S, FlatNode* nodes, int N, const int* idx, int I, const int* ids,
                   int count) {
    if (S < 0 || N < 0 || I < 0 || count < 0 || (S > 0 && !shapes) || (N > 0 && !nodes) || (I > 0 && !idx) ||
        (count > 0 && !ids))
        return -1;
    if (N == 0 || count == 0) return 0;
    std::vector<char> animated(static_cast<size_t>(S), 0);
    for (int j = 0; j < count; ++j) {
        if (ids[j] < 0 || ids[j] >= S) return -1;
        animated[ids[j]] = 1;
    }
    // the nodes above each node (split()'s trees: one parent each; any others are kept too)
    std::vector<int> parent(static_cast<size_t>(N), -1);
    std::vector<std::pair<int, int>> extra;  // (child, another parent)
    for (int k = 0; k < N; ++k) {
        const FlatNode& nd = nodes[k];
        if (nd.leftChild == -1) continue;
        if (nd.leftChild < 0 || nd.leftChild >= N || nd.rightChild < 0 || nd.rightChild >= N) return -1;
        for (int ch : {nd.leftChild, nd.rightChild}) {
            if (parent[ch] < 0) parent[ch] = k;
            else if (parent[ch] != k) extra.push_back({ch, k});
        }
    }
    // (shape, leaf) for every animated shape a leaf lists, in shape order
    std::vector<std::pair<int, int>> occ;
    for (int k = 0; k < N; ++k) {
        const FlatNode& nd = nodes[k];
        if (nd.leftChild != -1 || nd.numShapes <= 0) continue;
        if (nd.startShapeIdx < 0 || nd.startShapeIdx > I - nd.numShapes) return -1;
        for (int j = nd.startShapeIdx; j < nd.startShapeIdx + nd.numShapes; ++j) {
            if (idx[j] < 0 || idx[j] >= S) return -1;
            if (animated[idx[j]]) occ.push_back({idx[j], k});
        }
    }
    std::sort(occ.begin(), occ.end());
    std::vector<int> stamp(static_cast<size_t>(N), -1), todo;
    for (size_t q = 0; q < occ.size();) {
        const int a = occ[q].first;
        const FlatShape& f = shapes[a];
        Prim p;
        p.kind = f.type;
        p.radius = f.sphereRadius;
        p.normal = V3(&f.planeNormal.x);
        p.width = f.wallWidth;
        p.height = f.wallHeight;
        p.p0 = f.type == RT_SPHERE ? V3(&f.sphereCenter.x) : f.type == RT_WALL ? V3(&f.wallStart.x) : V3(&f.triP1.x);
        p.p1 = V3(&f.triP2.x);
        p.p2 = V3(&f.triP3.x);
        todo.clear();
        for (; q < occ.size() && occ[q].first == a; ++q)
            if (stamp[occ[q].second] != a) {
                stamp[occ[q].second] = a;
                todo.push_back(occ[q].second);
            }
        while (!todo.empty()) {  // each node listing shape a grows once by it
            const int k = todo.back();
            todo.pop_back();
            Box b;
            b.lo = V3(&nodes[k].boundsMin.x);
            b.hi = V3(&nodes[k].boundsMax.x);
            b.grow(p);
            nodes[k].boundsMin = flat(b.lo);
            nodes[k].boundsMax = flat(b.hi);
            auto up = [&](int u) {
                if (u >= 0 && stamp[u] != a) {
                    stamp[u] = a;
                    todo.push_back(u);
                }
            };
            up(parent[k]);
            for (const auto& e : extra)
                if (e.first == k) up(e.second);
        }
    }
    return 0;
}

int rts_generate(rts_scene* s, int config, int variant, float aspect) {
    if (!s) return -1;
    *s = rts_scene();
    switch (config) {
        case RTS_CONFIG_SPHERES: gen_spheres(s, aspect); break;
        case RTS_CONFIG_MONKEY: gen_monkey(s, aspect); break;
        case RTS_CONFIG_CAR: gen_car(s, variant, aspect); break;
        case RTS_CONFIG_RANDOM: gen_random(s, aspect); break;
        case RTS_CONFIG_TRIANGLE: gen_triangle(s, aspect); break;
        default: return -1;
    }
    return 0;
}

}  // extern "C"

// ref_harness.cpp — TEST INFRASTRUCTURE ONLY (oracle pinning).
//
// Compiles the reference's own header-only CPU classes where they lie under
// /root/reference (nothing is copied into this repository) and exposes them
// through a small C ABI, so tests/golden/make_golden.py can record known-answer
// vectors from the reference itself:
//   src/shapes/sphere.hpp  Sphere::get_intersection (:41-60)
//   src/shapes/plane.hpp   Plane::Plane (:28-33), Plane::get_intersection (:44-57)
//   src/shapes/wall.hpp    Wall::Wall (:37-40), Wall::end (:16-31),
//                          Wall::get_intersection (:46-68)
//   src/light.hpp          Light::Light / updateColor (:22-35)
//   src/material.hpp       Material::Material defaults (:23)
//   src/flatStructures.hpp the SSBO record sizes and offsets (:7-106)
// triangle.hpp, camera.hpp, BoundingBox.hpp and main.cpp need Embree, glad or
// GLFW, which the image lacks; they are not built ("Oracle").
// Built by oracle/Makefile into oracle/_ref/ (git-ignored) only when the
// reference tree is present.
#include <glm/glm.hpp>

#include <cstddef>
#include <cstring>

#include "src/light.hpp"
#include "src/material.hpp"
#include "src/shapes/plane.hpp"
#include "src/shapes/sphere.hpp"
#include "src/shapes/wall.hpp"

namespace {
glm::vec3 v(const float* p) { return glm::vec3(p[0], p[1], p[2]); }
void put(float* out, glm::vec3 a) {
    out[0] = a.x;
    out[1] = a.y;
    out[2] = a.z;
}
int run(const Shape& s, const float* o, const float* d, float* hit) {
    Intersection it = s.get_intersection(Ray(v(o), v(d)));
    put(hit, it.hit_point);
    return static_cast<int>(it.intersect_type);
}
}  // namespace

extern "C" {

// Sizes then offsets, in a fixed order (see make_golden.py LAYOUT_FIELDS).
int ref_layout(long* out, int cap) {
    const long vals[] = {
        (long)sizeof(FlatMaterial), (long)sizeof(FlatShape), (long)sizeof(FlatCamera), (long)sizeof(FlatLight),
        (long)sizeof(FlatNode),
        (long)offsetof(FlatMaterial, color), (long)offsetof(FlatMaterial, fresnelStrength),
        (long)offsetof(FlatMaterial, ambientStrength), (long)offsetof(FlatMaterial, diffuseStrength),
        (long)offsetof(FlatMaterial, specularStrength), (long)offsetof(FlatMaterial, shininess),
        (long)offsetof(FlatShape, type), (long)offsetof(FlatShape, material), (long)offsetof(FlatShape, sphereCenter),
        (long)offsetof(FlatShape, sphereRadius), (long)offsetof(FlatShape, planeNormal), (long)offsetof(FlatShape, planeD),
        (long)offsetof(FlatShape, wallStart), (long)offsetof(FlatShape, wallWidth), (long)offsetof(FlatShape, wallHeight),
        (long)offsetof(FlatShape, triP1), (long)offsetof(FlatShape, triP2), (long)offsetof(FlatShape, triP3),
        (long)offsetof(FlatCamera, Position), (long)offsetof(FlatCamera, aspectRatio), (long)offsetof(FlatCamera, Front),
        (long)offsetof(FlatCamera, Up), (long)offsetof(FlatCamera, Right), (long)offsetof(FlatCamera, fov),
        (long)offsetof(FlatLight, position), (long)offsetof(FlatLight, color),
        (long)offsetof(FlatNode, boundsMin), (long)offsetof(FlatNode, boundsMax), (long)offsetof(FlatNode, leftChild),
        (long)offsetof(FlatNode, rightChild), (long)offsetof(FlatNode, startShapeIdx), (long)offsetof(FlatNode, numShapes),
    };
    const int n = static_cast<int>(sizeof vals / sizeof vals[0]);
    for (int i = 0; i < n && i < cap; ++i) out[i] = vals[i];
    return n;
}

int ref_sphere_isect(const float* c, float r, const float* o, const float* d, float* hit) {
    Sphere s(v(c), r);
    return run(s, o, d, hit);
}

// Plane(normal, point): returns the stored m_normal and d too.
int ref_plane_isect(const float* n, const float* p, const float* o, const float* d, float* hit, float* nd) {
    Plane s(v(n), v(p));
    put(nd, s.m_normal);
    nd[3] = s.d;
    return run(s, o, d, hit);
}

int ref_wall_isect(const float* start, float w, float h, const float* n, const float* o, const float* d, float* hit,
                   float* nd) {
    Wall s(v(start), w, h, v(n));
    put(nd, s.m_normal);
    nd[3] = s.d;
    return run(s, o, d, hit);
}

int ref_wall_end(const float* start, float w, float h, const float* n, float* end) {
    Wall s(v(start), w, h, v(n));
    put(end, s.end());
    return 0;
}

int ref_light_color(const float* pos, const float* c, float intensity, float* color) {
    Light l(v(pos), v(c), intensity);
    put(color, l.color);
    return 0;
}

// Material() defaults: color.xyz, fresnel, ambient, diffuse, specular, shininess.
int ref_material_default(float* out) {
    Material m;
    put(out, m.color);
    out[3] = m.fresnelStrength;
    out[4] = m.ambientStrength;
    out[5] = m.diffuseStrength;
    out[6] = m.specularStrength;
    out[7] = static_cast<float>(m.shininess);
    return 0;
}

}  // extern "C"

/*
 * rt_flat.h — the byte layout of the scene records handed to the renderer.
 *
 * These are the reference's shader-storage records (std430 blocks), restated as
 * plain C so that an existing host can hand the very same arrays to the HIP
 * renderer that it used to hand to glBufferData:
 *
 *   FlatMaterial  32 B   src/flatStructures.hpp:7-20   ≡ gpu_shader.comp:29-37
 *   FlatShape    192 B   src/flatStructures.hpp:22-53  ≡ gpu_shader.comp:39-63
 *   FlatCamera    80 B   src/flatStructures.hpp:55-70  ≡ gpu_shader.comp:4-19 (std430 view 96 B: tail pad)
 *   FlatLight     32 B   src/flatStructures.hpp:72-78  ≡ gpu_shader.comp:21-27
 *   FlatNode      48 B   src/flatStructures.hpp:94-106 ≡ gpu_shader.comp:74-86
 *
 * Every size and field offset is pinned by static assertions below and, in
 * tests/test_oracle_golden.py (test_layout_matches_reference_header), against the offsets printed by the reference header
 * itself (compiled from /root/reference by oracle/Makefile, fixture
 * tests/golden/ref_layout.json).
 *
 * Shape type tags follow serializeShape (src/main.cpp:994-1066):
 *   0 sphere, 1 plane, 2 wall, 3 triangle.
 */
#ifndef RT_FLAT_H
#define RT_FLAT_H

#include <stddef.h>

#ifdef __cplusplus
#define RT_ALIGN16 alignas(16)
extern "C" {
#else
#define RT_ALIGN16 _Alignas(16)
#endif

typedef struct rt_vec3 { float x, y, z; } rt_vec3;

enum rt_shape_type { RT_SPHERE = 0, RT_PLANE = 1, RT_WALL = 2, RT_TRIANGLE = 3 };

typedef struct FlatMaterial {
    RT_ALIGN16 rt_vec3 color;   /* @0  */
    float fresnelStrength;      /* @12 */
    float ambientStrength;      /* @16 */
    float diffuseStrength;      /* @20 */
    float specularStrength;     /* @24 */
    int   shininess;            /* @28 (int in the reference, promoted by pow) */
} FlatMaterial;

typedef struct FlatShape {
    int type;                          /* @0   */
    RT_ALIGN16 rt_vec3 padding;        /* @16  */
    FlatMaterial material;             /* @32  */
    RT_ALIGN16 rt_vec3 sphereCenter;   /* @64  */
    float sphereRadius;                /* @76  */
    RT_ALIGN16 rt_vec3 planeNormal;    /* @80  */
    float planeD;                      /* @92  */
    RT_ALIGN16 rt_vec3 wallStart;      /* @96  */
    float wallWidth;                   /* @108 */
    float wallHeight;                  /* @112 */
    RT_ALIGN16 rt_vec3 padding1;       /* @128 */
    RT_ALIGN16 rt_vec3 triP1;          /* @144 */
    float padding2;                    /* @156 */
    RT_ALIGN16 rt_vec3 triP2;          /* @160 */
    float padding3;                    /* @172 */
    RT_ALIGN16 rt_vec3 triP3;          /* @176 */
    float padding4;                    /* @188 */
} FlatShape;

typedef struct FlatCamera {
    rt_vec3 Position;    /* @0  */
    float aspectRatio;   /* @12 */
    rt_vec3 Front;       /* @16 */
    float padding2;      /* @28 */
    rt_vec3 Up;          /* @32 */
    float padding3;      /* @44 */
    rt_vec3 Right;       /* @48 */
    float padding4;      /* @60 */
    float fov;           /* @64, degrees */
    rt_vec3 padding5;    /* @68 */
} FlatCamera;

typedef struct FlatLight {
    rt_vec3 position;    /* @0  */
    float padding1;      /* @12 */
    rt_vec3 color;       /* @16, = intensity * baseColor (src/light.hpp:32-35) */
    float padding2;      /* @28 */
} FlatLight;

typedef struct FlatNode {
    RT_ALIGN16 rt_vec3 boundsMin;  /* @0  */
    float padding1;                /* @12 */
    RT_ALIGN16 rt_vec3 boundsMax;  /* @16 */
    float padding2;                /* @28 */
    int leftChild;                 /* @32, -1 marks a leaf (gpu_shader.comp:399) */
    int rightChild;                /* @36 */
    int startShapeIdx;             /* @40, first slot in bvhIndices */
    int numShapes;                 /* @44 */
} FlatNode;

#ifdef __cplusplus
}
#define RT_STATIC_ASSERT(c, m) static_assert(c, m)
#else
#define RT_STATIC_ASSERT(c, m) _Static_assert(c, m)
#endif

RT_STATIC_ASSERT(sizeof(FlatMaterial) == 32, "FlatMaterial must be 32 B");
RT_STATIC_ASSERT(sizeof(FlatShape) == 192, "FlatShape must be 192 B");
RT_STATIC_ASSERT(sizeof(FlatCamera) == 80, "FlatCamera must be 80 B");
RT_STATIC_ASSERT(sizeof(FlatLight) == 32, "FlatLight must be 32 B");
RT_STATIC_ASSERT(sizeof(FlatNode) == 48, "FlatNode must be 48 B");
RT_STATIC_ASSERT(offsetof(FlatShape, material) == 32, "FlatShape.material");
RT_STATIC_ASSERT(offsetof(FlatShape, sphereCenter) == 64, "FlatShape.sphereCenter");
RT_STATIC_ASSERT(offsetof(FlatShape, sphereRadius) == 76, "FlatShape.sphereRadius");
RT_STATIC_ASSERT(offsetof(FlatShape, planeNormal) == 80, "FlatShape.planeNormal");
RT_STATIC_ASSERT(offsetof(FlatShape, planeD) == 92, "FlatShape.planeD");
RT_STATIC_ASSERT(offsetof(FlatShape, wallStart) == 96, "FlatShape.wallStart");
RT_STATIC_ASSERT(offsetof(FlatShape, wallWidth) == 108, "FlatShape.wallWidth");
RT_STATIC_ASSERT(offsetof(FlatShape, wallHeight) == 112, "FlatShape.wallHeight");
RT_STATIC_ASSERT(offsetof(FlatShape, triP1) == 144, "FlatShape.triP1");
RT_STATIC_ASSERT(offsetof(FlatShape, triP2) == 160, "FlatShape.triP2");
RT_STATIC_ASSERT(offsetof(FlatShape, triP3) == 176, "FlatShape.triP3");
RT_STATIC_ASSERT(offsetof(FlatNode, leftChild) == 32, "FlatNode.leftChild");
RT_STATIC_ASSERT(offsetof(FlatNode, numShapes) == 44, "FlatNode.numShapes");
RT_STATIC_ASSERT(offsetof(FlatCamera, fov) == 64, "FlatCamera.fov");
RT_STATIC_ASSERT(offsetof(FlatLight, color) == 16, "FlatLight.color");

#endif /* RT_FLAT_H */

/*
 * rt_scene.h — C ABI of the host scene library (librtscene.so).
 *
 * The CPU side of the reference's hot path, restated in C++: the shape set
 * (src/shapes/{sphere,plane,wall,triangle}.hpp), Material/Light/Camera (src/material.hpp, src/light.hpp,
 * src/camera.hpp), the spatial-midpoint BVH builder (split/buildBVH,
 * src/main.cpp:1111-1193, src/BoundingBox.hpp) and the serialisers that fill
 * the Flat* records (serializeShape/serializeBVH/serializeCamera/serializeLight,
 * src/main.cpp:806-823,955-979,994-1066). The arrays it produces are the same
 * bytes the reference uploads with glBufferData, and are what rt_upload_scene
 * (rt_api.h) consumes.
 *
 * Vectors are passed as `const float*` triples. Functions return 0 or a
 * negative status (same codes as rt_api.h); adders return the new shape index.
 */
#ifndef RT_SCENE_H
#define RT_SCENE_H

#include "rt_flat.h"

#ifdef __cplusplus
extern "C" {
#endif

struct rts_scene;

/* Benchmark configurations (BASELINE.json "configs"). */
enum rts_config {
    RTS_CONFIG_SPHERES = 1,   /* config 1: 4 spheres + 1 plane, 800x600 (CPU path)        */
    RTS_CONFIG_MONKEY = 2,    /* config 2: 1,240 shapes, 800x600, primary + shadow        */
    RTS_CONFIG_CAR = 3,       /* config 3/4: 4,022 triangles + 100 spheres                */
    RTS_CONFIG_RANDOM = 5,    /* config 5: 100k random triangles, deep BVH                */
    RTS_CONFIG_TRIANGLE = 6   /* the reference's default SCENE 3 (generateScene3): one
                                 triangle, no BVH built (0 nodes, 0 indices)               */
};

struct rts_scene* rts_new(void);
void rts_free(struct rts_scene* s);
int rts_clear(struct rts_scene* s);

/* Shapes. `mat` may be NULL for the Material() defaults (src/material.hpp:23). */
int rts_add_sphere(struct rts_scene* s, const float* center, float radius, const FlatMaterial* mat);
int rts_add_plane(struct rts_scene* s, const float* normal, const float* point, const FlatMaterial* mat);
int rts_add_wall(struct rts_scene* s, const float* start, float width, float height,
                 const float* normal, const FlatMaterial* mat);
/* invert != 0 applies Triangle::invert_normal (src/shapes/triangle.hpp:95-98). */
int rts_add_triangle(struct rts_scene* s, const float* a, const float* b, const float* c,
                     int invert, const FlatMaterial* mat);
/* Mesh → triangles the way generateScene1/2 add them (src/main.cpp:648-681,760-768):
 * vertices (xyz triples) + origin, one Triangle per index triple. Returns the
 * index of the first triangle added. */
int rts_add_mesh(struct rts_scene* s, const float* vertices, int num_vertices,
                 const unsigned* indices, int num_indices, const float* origin,
                 const FlatMaterial* mat);
/* Mesh::mesh2triangles normal-orientation rule (src/mesh.hpp:163-189), for
 * callers that keep the oriented triangles (the reference scenes do not). */
int rts_add_mesh_oriented(struct rts_scene* s, const float* vertices, int num_vertices,
                          const unsigned* indices, int num_indices, const float* origin,
                          const FlatMaterial* mat);

/* Wavefront OBJ ingestion, replacing assimp (src/model.hpp:49-168): vertex
 * positions and faces (polygons split as a fan from their first corner, as
 * aiProcess_Triangulate does for convex faces) become one mesh, added like
 * rts_add_mesh (oriented != 0: like rts_add_mesh_oriented). Returns the number
 * of triangles added, -1 invalid argument, -2 I/O error, -3 malformed file. */
int rts_load_obj(struct rts_scene* s, const char* path, const float* origin, const FlatMaterial* mat,
                 int oriented);
int rts_parse_obj(struct rts_scene* s, const char* text, long len, const float* origin,
                  const FlatMaterial* mat, int oriented);

/* Image dump, replacing the screen quad (src/main.cpp:476-501, shaders/shader.frag):
 * an RGBA32F image (row 0 = NDC y +1, pitch in bytes) written as binary PPM
 * (rgb clamped to [0,1], 8 bits) or colour PFM (float rgb, exact). 0 or -1
 * (invalid argument) / -2 (I/O error). */
enum { RTS_IMAGE_PPM = 0, RTS_IMAGE_PFM = 1 };
int rts_write_image(const char* path, const float* rgba, int width, int height, long pitch_bytes, int format);

/* Camera() then Position/aspect/fov, and Camera::LookAt (src/camera.hpp:124-163). */
int rts_set_camera(struct rts_scene* s, const float* position, float fov_deg, float aspect);
int rts_camera_look_at(struct rts_scene* s, const float* target);
/* Light(pos, color, intensity) (src/light.hpp:22-35). */
int rts_set_light(struct rts_scene* s, const float* position, const float* color, float intensity);

/* buildBVH(maxDepth) (src/main.cpp:1175-1193). Replaces any previous tree. */
int rts_build_bvh(struct rts_scene* s, int max_depth);

/* updateBVH (src/main.cpp:1068-1077) on serialised arrays, for a host that keeps
 * the reference's own per-frame upload (rt_update_nodes): every node whose shape
 * set lists one of the shapes ids[0..count) (a leaf listing it in bvhIndices, and
 * every node above that leaf) grows to include that shape's current record
 * (growToInclude, src/BoundingBox.hpp:44-95), in the order the reference grows
 * them. Grow-only; nodes are updated in place. 0, or -1 on bad arguments. */
int rts_update_bvh(const FlatShape* shapes, int num_shapes, FlatNode* nodes, int num_nodes, const int* indices,
                   int num_indices, const int* ids, int count);

/* Sizes of the serialised arrays: shapes, nodes, bvhIndices. */
int rts_counts(const struct rts_scene* s, int* num_shapes, int* num_nodes, int* num_indices);

/* serializeScene (src/main.cpp:825-846): fills caller arrays sized by rts_counts.
 * Any pointer may be NULL to skip that part. Unused fields are zero. */
int rts_serialize(const struct rts_scene* s, FlatShape* shapes, FlatNode* nodes, int* indices,
                  FlatCamera* camera, FlatLight* light);

/* Tree statistics: leaves, largest leaf, tree depth, the reference traversal's
 * worst-case stack need (all boxes hit). */
int rts_bvh_stats(const struct rts_scene* s, int* leaves, int* max_leaf, int* depth, int* max_stack);

/* Fill the scene with benchmark configuration `config` (rts_config) at aspect
 * width/height. variant 0 = the primary stand-in; for RTS_CONFIG_CAR variant 1
 * = tessellated road. Builds the BVH with the reference's depth for that scene.
 * Fixed seed: identical output on every machine. */
int rts_generate(struct rts_scene* s, int config, int variant, float aspect);

#ifdef __cplusplus
}
#endif

#endif /* RT_SCENE_H */

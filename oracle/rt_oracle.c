/*
 * rt_oracle.c — CPU ORACLE for the MI355X ray tracer.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker / the timed CPU baseline. The product
 * (librtamd.so, librtscene.so) never links or calls it.
 *
 * What it restates, line by line (paths relative to the reference repo):
 *   - src/shaders/gpu_shader.comp (the GLSL hot path): getRay :155-168,
 *     get_intersection :242-328 with the barycentric :196-240 and
 *     Moller-Trumbore :170-195 triangle tests, getNormalFromShape :64-71,
 *     phong :331-361, rayIntersectsAABB :364-377, intersectScene2 :380-430,
 *     main :433-624 (BVH branch :446-520, brute-force branch :523-620).
 *   - cpuRayTracer src/main.cpp:848-894 with the CPU phong :553-581 and the
 *     shape classes src/shapes/{sphere,plane,wall,triangle}.hpp (the CPU
 *     baseline of BASELINE.md; triangles use BARYCENTRIC).
 *   - the BVH builder split/buildBVH/serializeBVH src/main.cpp:955-979,
 *     1111-1193 with BoundingBox src/BoundingBox.hpp:34-95, working from the
 *     serialised FlatShape records, so the product's builder can be checked
 *     byte for byte against an independent restatement.
 *   - glm semantics (glm/glm/detail/func_geometric.inl:94,114,
 *     func_exponential.inl:132, func_common.inl:143-152): dot = (x+y)+z,
 *     normalize = v*(1/sqrt(v.v)), reflect = I - N*dot(N,I)*2, mix = x+a*(y-x).
 *
 * Pinning: the sphere/plane/wall intersection, Wall::end, Plane/Triangle
 * normals and the Flat* layouts are checked against the reference's own
 * headers compiled from /root/reference (oracle/ref_harness.cpp ->
 * tests/golden/ref_*.json). The GLSL whole-frame semantics have no reference
 * test or golden image; they are pinned through those
 * primitives plus this restatement.
 *
 * Build: -O2 -ffp-contract=off, no fast-math (see oracle/Makefile).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>
#include <stddef.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/rt_flat.h"
#include "../include/rt_api.h"

typedef struct { float x, y, z; } v3;
typedef struct { v3 o, d; } ray_t;

static inline v3 mk(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 fv(rt_vec3 a) { return mk(a.x, a.y, a.z); }
static inline v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 neg(v3 a) { return mk(-a.x, -a.y, -a.z); }
static inline v3 muls(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
static inline v3 smul(float s, v3 a) { return mk(s * a.x, s * a.y, s * a.z); }
static inline v3 mulv(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 divs(v3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
static inline float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline v3 cross(v3 a, v3 b) {
    return mk(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
static inline float length3(v3 a) { return sqrtf(dot(a, a)); }
static inline v3 normalize3(v3 a) { return muls(a, 1.0f / sqrtf(dot(a, a))); }
static inline float distance3(v3 a, v3 b) { return length3(sub(b, a)); }
static inline v3 reflect3(v3 i, v3 n) { return sub(i, muls(muls(n, dot(n, i)), 2.0f)); }
static inline v3 mix3(v3 x, v3 y, float a) { return add(x, smul(a, sub(y, x))); }
static inline float fmaxg(float a, float b) { return (a < b) ? b : a; }  /* GLSL/glm max */
static inline float fming(float a, float b) { return (b < a) ? b : a; }  /* GLSL/glm min */

enum { NONE = 0, INNER = 1, OUTER = 2 };
typedef struct { int type; v3 hit; } isect_t;

/* ------------------------------------------------------------------------ */
/* GLSL primitives                                                           */

/* getRay (gpu_shader.comp:155-168). */
static ray_t get_ray(const FlatCamera* cam, float ndcX, float ndcY) {
    float h = 2.0f * tanf((cam->fov / 2.0f) * 0.01745329251994329576923690768489f);
    float w = h * cam->aspectRatio;
    v3 pos = fv(cam->Position);
    v3 p = add(add(add(pos, fv(cam->Front)), smul(ndcX * w / 2.0f, fv(cam->Right))),
               smul(ndcY * h / 2.0f, fv(cam->Up)));
    ray_t r;
    r.o = pos;
    r.d = normalize3(sub(p, pos));
    return r;
}

/* getIntersectionTriangle_MollerTrumbore (:170-195). */
static isect_t tri_mt(const FlatShape* s, ray_t r) {
    isect_t it = {NONE, {0, 0, 0}};
    v3 p1 = fv(s->triP1);
    v3 e1 = sub(fv(s->triP2), p1), e2 = sub(fv(s->triP3), p1);
    v3 h = cross(r.d, e2);
    float a = dot(e1, h);
    if (fabsf(a) < 1e-5f) return it;
    float f = 1.0f / a;
    v3 sv = sub(r.o, p1);
    float u = f * dot(sv, h);
    if (u < 0 || u > 1) return it;
    v3 q = cross(sv, e1);
    float v = f * dot(r.d, q);
    if (v < 0 || u + v > 1) return it;
    float t = f * dot(e2, q);
    if (t > 0) {
        it.type = INNER;
        it.hit = add(r.o, smul(t, r.d));
    }
    return it;
}

/* getIntersectionTriangle_Barycentric (:196-240). */
static isect_t tri_bary(const FlatShape* s, ray_t r) {
    isect_t it = {NONE, {0, 0, 0}};
    v3 n = fv(s->planeNormal);
    float np = dot(n, r.d);
    if (np == 0) return it;
    float t = -(s->planeD + dot(n, r.o)) / np;
    if (t > 0) {
        it.type = (np > 0) ? INNER : OUTER;
        it.hit = add(r.o, smul(t, r.d));
        if (np <= 0) return it;
    } else {
        return it;
    }
    v3 p1 = fv(s->triP1);
    v3 e1 = sub(fv(s->triP2), p1), e2 = sub(fv(s->triP3), p1), tp = sub(it.hit, p1);
    float d00 = dot(e1, e1), d01 = dot(e1, e2), d11 = dot(e2, e2);
    float d20 = dot(tp, e1), d21 = dot(tp, e2);
    float denom = d00 * d11 - d01 * d01;
    float v = (d11 * d20 - d01 * d21) / denom;
    float w = (d00 * d21 - d01 * d20) / denom;
    float u = 1.0f - v - w;
    if (u < 0 || v < 0 || w < 0) it.type = NONE;
    return it;
}

/* get_intersection (:242-328). */
static isect_t get_isect(const FlatShape* s, ray_t r, int use_mt) {
    isect_t it = {NONE, {0, 0, 0}};
    if (s->type == RT_SPHERE) {
        v3 c = fv(s->sphereCenter);
        v3 oc = sub(r.o, c);
        float aa = dot(r.d, r.d);
        float bb = 2 * (dot(r.d, oc));
        float cc = dot(oc, oc) - s->sphereRadius * s->sphereRadius;
        float D = bb * bb - 4 * aa * cc;
        if (D > 0) {
            float sD = sqrtf(D);
            float t1 = (-bb - sD) / (2 * aa);
            if (t1 > 0) {
                it.type = INNER;
                it.hit = add(r.o, smul(t1, r.d));
                return it;
            }
            float t2 = (-bb + sD) / (2 * aa);
            if (t2 > 0) {
                it.type = OUTER;
                return it;
            }
        }
    } else if (s->type == RT_PLANE) {
        v3 n = fv(s->planeNormal);
        float np = dot(n, r.d);
        if (np == 0) return it;
        float t = -(s->planeD + dot(n, r.o)) / np;
        if (t > 0) {
            it.type = (np > 0) ? INNER : OUTER;
            if (np <= 0) return it;
            it.hit = add(r.o, smul(t, r.d));
        } else {
            return it;
        }
    } else if (s->type == RT_WALL) {
        v3 n = fv(s->planeNormal);
        float np = dot(n, r.d);
        if (np == 0) return it;
        float t = -(s->planeD + dot(n, r.o)) / np;
        if (t > 0) {
            it.type = (np > 0) ? INNER : OUTER;
            if (np <= 0) return it;
            it.hit = add(r.o, smul(t, r.d));
        } else {
            return it;
        }
        v3 u = normalize3(cross(n, mk(0, 1, 0)));
        if (length3(u) < 1e-5f) u = normalize3(cross(n, mk(1, 0, 0)));
        v3 v = normalize3(cross(n, u));
        v3 lp = sub(it.hit, fv(s->wallStart));
        float up = dot(lp, u), vp = dot(lp, v);
        if (up < 0 || up > s->wallWidth || vp < 0 || vp > s->wallHeight) it.type = NONE;
    } else if (s->type == RT_TRIANGLE) {
        it = use_mt ? tri_mt(s, r) : tri_bary(s, r);
    }
    return it;
}

/* getNormalFromShape (:64-71); other type values have no return in GLSL. */
static v3 shape_normal(const FlatShape* s, v3 p) {
    if (s->type == RT_SPHERE) return normalize3(sub(p, fv(s->sphereCenter)));
    return fv(s->planeNormal);
}

/* phong (:331-361). pow(float, int) promotes the int; shininess 0 follows C powf. */
static v3 phong_gpu(v3 p, v3 n, v3 view, const FlatLight* L, const FlatMaterial* m) {
    v3 lpos = fv(L->position);
    float dl = distance3(lpos, p);
    v3 lc = divs(fv(L->color), dl);
    v3 amb = smul(m->ambientStrength, lc);
    v3 ldir = normalize3(sub(lpos, p));
    float diff = fmaxg(dot(n, ldir), 0.0f);
    v3 dif = smul(m->diffuseStrength * diff, lc);
    v3 spc = mk(0, 0, 0);
    if (diff > 0.f) {
        v3 rd = reflect3(neg(ldir), n);
        float sp = powf(fmaxg(dot(view, rd), 0.0f), (float)m->shininess);
        spc = smul(m->specularStrength * sp, lc);
    }
    return mulv(add(add(amb, dif), spc), fv(m->color));
}

/* rayIntersectsAABB (:364-377). */
static int ray_aabb(ray_t r, v3 bmin, v3 bmax) {
    v3 inv = mk(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);
    v3 t0 = mulv(sub(bmin, r.o), inv), t1 = mulv(sub(bmax, r.o), inv);
    v3 lo = mk(fming(t0.x, t1.x), fming(t0.y, t1.y), fming(t0.z, t1.z));
    v3 hi = mk(fmaxg(t0.x, t1.x), fmaxg(t0.y, t1.y), fmaxg(t0.z, t1.z));
    float tmin = fmaxg(fmaxg(lo.x, lo.y), lo.z);
    float tmax = fming(fming(hi.x, hi.y), hi.z);
    return tmax >= tmin && tmax > 0.0f;
}

typedef struct {
    const FlatShape* shapes; int S;
    const FlatNode* nodes; int N;
    const int* idx; int I;
    const FlatCamera* cam; const FlatLight* light;
    rt_params p;
} scene_t;

typedef struct { int type; v3 hit, normal; const FlatMaterial* mat; } hit_t;

/* intersectScene2 (:380-430): closest INNER hit by distance, strict <, from a
 * stack walk that pushes left then right (right popped first), no ordering,
 * no pruning. Stack of 64 as in :384; deeper trees are UB in GLSL and are
 * reported as a miss here. */
static hit_t intersect_scene2(const scene_t* sc, ray_t r, rt_stats* st) {
    hit_t h;
    h.type = NONE;
    h.mat = NULL;
    h.hit = h.normal = mk(0, 0, 0);
    if (sc->N <= 0) return h;
    int stack[64];
    int sp = 0;
    stack[sp++] = sc->N - 1;
    float closest = 1e20f;
    while (sp > 0) {
        int k = stack[--sp];
        const FlatNode* nd = &sc->nodes[k];
        if (st) st->node_visits++;
        if (!ray_aabb(r, fv(nd->boundsMin), fv(nd->boundsMax))) continue;
        if (nd->leftChild == -1) {
            for (int i = 0; i < nd->numShapes; i++) {
                int si = sc->idx[nd->startShapeIdx + i];
                const FlatShape* s = &sc->shapes[si];
                if (st && s->type >= 0 && s->type < 4) st->bvh_tests[s->type]++;
                isect_t it = get_isect(s, r, sc->p.useMollerTrumbore);
                if (it.type == INNER) {
                    float dist = distance3(r.o, it.hit);
                    if (dist < closest) {
                        closest = dist;
                        h.type = INNER;
                        h.hit = it.hit;
                        h.normal = shape_normal(s, it.hit);
                        h.mat = &s->material;
                        if (st) st->closest_updates++;
                    }
                }
            }
        } else {
            if (sp + 2 > 64) { h.type = NONE; return h; }
            stack[sp++] = nd->leftChild;
            stack[sp++] = nd->rightChild;
        }
    }
    return h;
}

/* main (:433-624) for one pixel. */
static void shade_pixel(const scene_t* sc, int x, int y, float* out, rt_stats* st) {
    float fx = (float)x, fy = (float)y;
    v3 bg = mix3(mk(0.05f, 0.07f, 0.1f), mk(0.5f, 0.7f, 1.0f), fy / sc->p.resY);
    float val[4] = {bg.x, bg.y, bg.z, 1.0f};
    ray_t ray = get_ray(sc->cam, 2.0f * fx / sc->p.resX - 1.0f, 1.0f - 2.0f * fy / sc->p.resY);
    const FlatLight* L = sc->light;
    v3 lpos = fv(L->position);
    v3 acc = mk(0, 0, 0), att = mk(1, 1, 1);
    if (st) st->pixels++;
    if (sc->p.useBVH) {
        for (int depth = 0; depth < sc->p.maxBounces; ++depth) {
            if (st) st->closest_rays++;
            hit_t hit = intersect_scene2(sc, ray, st);
            if (hit.type != INNER) {
                acc = add(acc, mulv(att, bg));
                break;
            }
            if (st) st->hits++;
            v3 hp = hit.hit, hn = hit.normal;
            const FlatMaterial* m = hit.mat;
            v3 hc = fv(m->color);
            int shadow = 0;
            ray_t sr;
            sr.o = add(hp, muls(hn, 1e-3f));
            sr.d = normalize3(sub(lpos, hp));
            if (st) st->shadow_rays++;
            hit_t sh = intersect_scene2(sc, sr, st);
            if (sh.type != NONE) {
                float ld = distance3(lpos, hp);
                float hd = distance3(sr.o, sh.hit);
                if (hd < ld) shadow = 1;
            }
            v3 pc = phong_gpu(hp, hn, ray.d, L, m);
            if (shadow) pc = muls(pc, 0.3f);
            acc = add(acc, mulv(att, pc));
            if (m->specularStrength > 0) {
                v3 rd = reflect3(ray.d, hn);
                ray.o = add(hp, muls(hn, 1e-3f));
                ray.d = rd;
                if (sc->p.useFresnel) {
                    float fr = powf(1.0f - fmaxg(dot(neg(ray.d), hn), 0.0f), 5.0f);
                    fr = fming(fmaxg(fr, 0.0f), 0.8f);
                    float rw = m->fresnelStrength * fr;
                    float mw = 1.0f - rw;
                    att = mulv(att, mix3(hc, mk(1, 1, 1), rw));
                    acc = add(acc, mulv(smul(mw, hc), pc));
                } else {
                    att = muls(att, m->specularStrength);
                }
            } else {
                break;
            }
        }
        val[0] = acc.x; val[1] = acc.y; val[2] = acc.z;
    } else {
        for (int depth = 0; depth < sc->p.maxBounces; ++depth) {
            float closest = 1e20f;
            int hit_any = 0;
            v3 hc = bg, hp = mk(0, 0, 0), hn = mk(0, 0, 0);
            const FlatMaterial* m = NULL;
            if (st) st->closest_rays++;
            for (int i = 0; i < sc->S; ++i) {
                const FlatShape* s = &sc->shapes[i];
                if (st && s->type >= 0 && s->type < 4) st->brute_tests[s->type]++;
                isect_t it = get_isect(s, ray, sc->p.useMollerTrumbore);
                if (it.type == INNER) {
                    float dist = distance3(ray.o, it.hit);
                    if (dist < closest) {
                        closest = dist;
                        hit_any = 1;
                        hp = it.hit;
                        hn = shape_normal(s, hp);
                        m = &s->material;
                        hc = fv(s->material.color);
                        if (st) st->closest_updates++;
                    }
                }
            }
            if (!hit_any) {
                acc = add(acc, mulv(att, bg));
                break;
            }
            if (st) st->hits++;
            int shadow = 0;
            ray_t sr;
            sr.o = add(hp, muls(hn, 1e-5f));
            sr.d = normalize3(sub(lpos, hp));
            if (st) st->shadow_rays++;
            for (int i = 0; i < sc->S; ++i) {
                const FlatShape* s = &sc->shapes[i];
                if (st && s->type >= 0 && s->type < 4) st->brute_tests[s->type]++;
                isect_t it = get_isect(s, sr, sc->p.useMollerTrumbore);
                if (it.type == INNER) {
                    float ld = distance3(lpos, hp);
                    float hd = distance3(sr.o, it.hit);
                    if (hd < ld) { shadow = 1; break; }
                }
            }
            v3 pc = phong_gpu(hp, hn, ray.d, L, m);
            if (shadow) pc = muls(pc, 0.3f);
            acc = add(acc, mulv(att, pc));
            if (m->specularStrength > 0) {
                v3 rd = reflect3(ray.d, hn);
                ray.o = add(hp, muls(hn, 1e-3f));
                ray.d = rd;
                if (sc->p.useFresnel) {
                    float fr = powf(1.0f - fmaxg(dot(neg(ray.d), hn), 0.0f), 5.0f);
                    fr = fming(fmaxg(fr, 0.0f), 0.8f);
                    float rw = m->fresnelStrength * fr;
                    float mw = 1.0f - rw;
                    att = mulv(att, mix3(hc, mk(1, 1, 1), rw));
                    acc = add(acc, mulv(smul(mw, hc), pc));
                } else {
                    att = muls(att, m->specularStrength);
                }
            } else {
                break;
            }
        }
        val[0] = acc.x; val[1] = acc.y; val[2] = acc.z;
    }
    out[0] = val[0]; out[1] = val[1]; out[2] = val[2]; out[3] = val[3];
}

static void stats_add(rt_stats* a, const rt_stats* b) {
    a->pixels += b->pixels; a->closest_rays += b->closest_rays; a->shadow_rays += b->shadow_rays;
    a->node_visits += b->node_visits; a->closest_updates += b->closest_updates; a->hits += b->hits;
    for (int i = 0; i < 4; ++i) { a->bvh_tests[i] += b->bvh_tests[i]; a->brute_tests[i] += b->brute_tests[i]; }
}

/* Row mapping shared with rt_dispatch_rows (include/rt_api.h). */
static int image_row(int y0, int stripe, int step, int r) {
    return y0 + (r / stripe) * stripe * step + (r % stripe);
}

/* Renders output rows [0, out_rows) of the stripe mapping into `out` (packed,
 * width*4 floats per row). Rows mapping to y >= height are left untouched.
 * stats may be NULL. threads <= 0 uses the OpenMP default. Returns 0. */
int orc_render(const FlatShape* shapes, int S, const FlatNode* nodes, int N, const int* idx, int I,
               const FlatCamera* cam, const FlatLight* light, const rt_params* p,
               int width, int height, int y0, int stripe, int step, int out_rows,
               float* out, rt_stats* stats, int threads) {
    if (!cam || !light || !p || !out || width <= 0 || height <= 0 || stripe <= 0 || step <= 0) return -1;
    scene_t sc = {shapes, S, nodes, N, idx, I, cam, light, *p};
    rt_stats total;
    memset(&total, 0, sizeof total);
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
#pragma omp parallel
    {
        rt_stats local;
        memset(&local, 0, sizeof local);
#pragma omp for schedule(dynamic, 1)
        for (int r = 0; r < out_rows; ++r) {
            int y = image_row(y0, stripe, step, r);
            if (y >= height) continue;
            for (int x = 0; x < width; ++x)
                shade_pixel(&sc, x, y, out + ((size_t)r * width + x) * 4, stats ? &local : NULL);
        }
        if (stats) {
#pragma omp critical
            stats_add(&total, &local);
        }
    }
    if (stats) *stats = total;
    return 0;
}

/* ------------------------------------------------------------------------ */
/* cpuRayTracer (src/main.cpp:848-894): brute force, primary rays only, black */
/* background, CPU phong without attenuation (:553-581).                      */

static v3 phong_cpu(v3 p, v3 n, v3 view, v3 color, v3 lpos, v3 lcol, const FlatMaterial* m) {
    v3 amb = smul(m->ambientStrength, lcol);
    v3 ldir = normalize3(sub(lpos, p));
    float diff = fmaxg(dot(n, ldir), 0.0f);
    v3 dif = smul(m->diffuseStrength * diff, lcol);
    v3 spc = mk(0, 0, 0);
    if (diff > 0.f) {
        v3 rd = reflect3(neg(ldir), n);
        /* glm::pow -> std::pow(float, int) -> double pow (glm func_exponential.inl:68) */
        float sp = (float)pow((double)fmaxg(dot(view, rd), 0.0f), (double)m->shininess);
        spc = smul(m->specularStrength * sp, lcol);
    }
    return mulv(add(add(amb, dif), spc), color);
}

/* The shape classes' get_intersection: same INNER set as the GLSL functions
 * (sphere.hpp:41-60, plane.hpp:44-57, wall.hpp:46-68 with the 1e-4 fallback
 * threshold, triangle.hpp:100-131 BARYCENTRIC). Only INNER is used by
 * cpuRayTracer, so the GLSL routine's INNER results are reused and the wall
 * threshold is the only difference (never reached by a unit normal). */
static isect_t get_isect_cpu(const FlatShape* s, ray_t r) {
    if (s->type == RT_WALL) {
        isect_t it = {NONE, {0, 0, 0}};
        v3 n = fv(s->planeNormal);
        float np = dot(n, r.d);
        if (np == 0) return it;
        float t = -(s->planeD + dot(n, r.o)) / np;
        if (!(t > 0)) return it;
        it.type = (np > 0) ? INNER : OUTER;
        it.hit = add(r.o, smul(t, r.d));
        v3 u = normalize3(cross(n, mk(0, 1, 0)));
        if (length3(u) < 1e-4f) u = normalize3(cross(n, mk(1, 0, 0)));
        v3 v = normalize3(cross(n, u));
        v3 lp = sub(it.hit, fv(s->wallStart));
        float up = dot(lp, u), vp = dot(lp, v);
        if (up < 0 || up > s->wallWidth || vp < 0 || vp > s->wallHeight) it.type = NONE;
        return it;
    }
    return get_isect(s, r, 0);
}

int orc_cpu_raytracer(const FlatShape* shapes, int S, const FlatCamera* cam, const FlatLight* light,
                      int width, int height, int y0, int y1, float* out, int threads) {
    if (!cam || !light || !out || width <= 0 || height <= 0 || y0 < 0 || y1 > height || y0 > y1) return -1;
    v3 lpos = fv(light->position), lcol = fv(light->color);
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
#pragma omp parallel for schedule(dynamic, 1)
    for (int y = y0; y < y1; ++y) {
        for (int x = 0; x < width; ++x) {
            ray_t r;
            /* Camera::GetRay (src/camera.hpp:124-137) == GLSL getRay. */
            r = get_ray(cam, 2.f * (float)x / (float)width - 1, 1.f - 2.f * (float)y / (float)height);
            v3 color = mk(0, 0, 0);
            float closest = FLT_MAX;
            float* px = out + ((size_t)(y - y0) * width + x) * 4;
            for (int i = 0; i < S; ++i) {
                const FlatShape* s = &shapes[i];
                isect_t it = get_isect_cpu(s, r);
                if (it.type == INNER) {
                    float dist = distance3(r.o, it.hit);
                    if (dist < closest) {
                        closest = dist;
                        color = phong_cpu(it.hit, shape_normal(s, it.hit), r.d, fv(s->material.color),
                                          lpos, lcol, &s->material);
                    }
                }
                px[0] = color.x; px[1] = color.y; px[2] = color.z; px[3] = 1.f;
            }
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* BVH builder from serialised shapes (split/buildBVH src/main.cpp:1111-1193, */
/* BoundingBox src/BoundingBox.hpp:34-95, Wall::end src/shapes/wall.hpp:16-31). */

typedef struct { v3 lo, hi; } box_t;
typedef struct { box_t box; int left, right; int* list; int n; } bnode_t;
typedef struct { bnode_t* v; int n, cap; const FlatShape* shapes; int failed; } builder_t;

static box_t box_empty(void) { box_t b = {{INFINITY, INFINITY, INFINITY}, {-INFINITY, -INFINITY, -INFINITY}}; return b; }
static void box_pt(box_t* b, v3 p) {
    b->lo = mk(fming(b->lo.x, p.x), fming(b->lo.y, p.y), fming(b->lo.z, p.z));
    b->hi = mk(fmaxg(b->hi.x, p.x), fmaxg(b->hi.y, p.y), fmaxg(b->hi.z, p.z));
}
static v3 wall_end(const FlatShape* s) {
    v3 n = fv(s->planeNormal), t1;
    if (fabsf(n.x) > fabsf(n.y)) t1 = normalize3(mk(-n.z, 0, n.x));
    else t1 = normalize3(mk(0, -n.z, n.y));
    v3 t2 = normalize3(cross(n, t1));
    return add(add(fv(s->wallStart), smul(s->wallWidth, t1)), smul(s->wallHeight, t2));
}
static void box_shape(box_t* b, const FlatShape* s) {
    if (s->type == RT_SPHERE) {
        v3 c = fv(s->sphereCenter);
        float r = s->sphereRadius;
        box_pt(b, mk(c.x + r, c.y + r, c.z + r));
        box_pt(b, mk(c.x - r, c.y - r, c.z - r));
    } else if (s->type == RT_WALL) {
        box_pt(b, fv(s->wallStart));
        box_pt(b, wall_end(s));
    } else if (s->type == RT_TRIANGLE) {
        if (isfinite(s->triP1.x) && isfinite(s->triP2.x) && isfinite(s->triP3.x)) {
            box_pt(b, fv(s->triP1));
            box_pt(b, fv(s->triP2));
            box_pt(b, fv(s->triP3));
        }
    }
}
static v3 split_centre(const FlatShape* s) {
    if (s->type == RT_SPHERE) return fv(s->sphereCenter);
    if (s->type == RT_WALL) return muls(add(fv(s->wallStart), wall_end(s)), 0.5f);
    if (s->type == RT_TRIANGLE) return divs(add(add(fv(s->triP1), fv(s->triP2)), fv(s->triP3)), 3.0f);
    return mk(0, 0, 0);
}
static float comp(v3 v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); }

static int push_node(builder_t* B, bnode_t nd) {
    if (B->n == B->cap) {
        int cap = B->cap ? 2 * B->cap : 64;
        bnode_t* nv = (bnode_t*)realloc(B->v, (size_t)cap * sizeof(bnode_t));
        if (!nv) { B->failed = 1; free(nd.list); return -1; }
        B->v = nv;
        B->cap = cap;
    }
    B->v[B->n] = nd;
    return B->n++;
}

static void split_node(builder_t* B, bnode_t* parent, int depth) {
    if (depth <= 0 || B->failed) { parent->left = parent->right = -1; return; }
    v3 size = sub(parent->box.hi, parent->box.lo);
    int axis = size.x > fmaxg(size.y, size.z) ? 0 : (size.y > size.z ? 1 : 2);
    float pos = comp(muls(add(parent->box.lo, parent->box.hi), 0.5f), axis);
    bnode_t L = {box_empty(), -1, -1, (int*)malloc(sizeof(int) * (size_t)(parent->n ? parent->n : 1)), 0};
    bnode_t R = {box_empty(), -1, -1, (int*)malloc(sizeof(int) * (size_t)(parent->n ? parent->n : 1)), 0};
    if (!L.list || !R.list) { B->failed = 1; free(L.list); free(R.list); return; }
    for (int i = 0; i < parent->n; ++i) {
        int k = parent->list[i];
        const FlatShape* s = &B->shapes[k];
        bnode_t* side = (comp(split_centre(s), axis) < pos) ? &L : &R;
        box_shape(&side->box, s);
        side->list[side->n++] = k;
    }
    if (L.n == 0 || R.n == 0) {
        parent->left = parent->right = -1;
        free(L.list); free(R.list);
        return;
    }
    split_node(B, &L, depth - 1);
    split_node(B, &R, depth - 1);
    parent->left = push_node(B, L);
    parent->right = push_node(B, R);
}

/* Builds the reference tree over shapes[0..S) and serialises it like
 * serializeBVH (src/main.cpp:955-979). Writes at most node_cap nodes and
 * idx_cap indices; *out_n / *out_i receive the full sizes. Returns 0, or -1
 * on allocation failure / when a capacity is too small. */
int orc_build_bvh(const FlatShape* shapes, int S, int max_depth, FlatNode* nodes, int node_cap,
                  int* idx, int idx_cap, int* out_n, int* out_i) {
    builder_t B = {NULL, 0, 0, shapes, 0};
    bnode_t root = {box_empty(), -1, -1, (int*)malloc(sizeof(int) * (size_t)(S > 0 ? S : 1)), 0};
    if (!root.list) return -1;
    for (int i = 0; i < S; ++i) {
        box_shape(&root.box, &shapes[i]);
        root.list[root.n++] = i;
    }
    split_node(&B, &root, max_depth);
    push_node(&B, root);
    int rc = B.failed ? -1 : 0;
    int cursor = 0;
    for (int k = 0; k < B.n; ++k) {
        bnode_t* nd = &B.v[k];
        if (k < node_cap && nodes) {
            FlatNode* f = &nodes[k];
            memset(f, 0, sizeof *f);
            f->boundsMin.x = nd->box.lo.x; f->boundsMin.y = nd->box.lo.y; f->boundsMin.z = nd->box.lo.z;
            f->boundsMax.x = nd->box.hi.x; f->boundsMax.y = nd->box.hi.y; f->boundsMax.z = nd->box.hi.z;
            f->leftChild = nd->left;
            f->rightChild = nd->right;
            f->startShapeIdx = cursor;
            f->numShapes = nd->n;
        }
        if (nd->left == -1)
            for (int i = 0; i < nd->n; ++i) {
                if (idx && cursor < idx_cap) idx[cursor] = nd->list[i];
                ++cursor;
            }
        free(nd->list);
    }
    if (out_n) *out_n = B.n;
    if (out_i) *out_i = cursor;
    if (B.n > node_cap || cursor > idx_cap) rc = -1;
    free(B.v);
    return rc;
}

/* updateBVH (src/main.cpp:1068-1077) on the serialised tree: every node whose
 * shapesIndices list an animated shape grows to include the shape's current
 * geometry (BoundingBox::growToInclude, src/BoundingBox.hpp:44-95; grow-only).
 * The reference keeps shapesIndices on inner nodes too: the union of its
 * children's (split, src/main.cpp:1128-1144), i.e. every shape of the leaves
 * below. This restatement derives that set from the flat tree: node k lists
 * shape a iff a leaf reachable from k lists it. Boxes in nodes[] grow in place. */
static int lists_shape(const FlatNode* nodes, const int* idx, int k, int a, signed char* memo, int depth) {
    if (memo[k] >= 0) return memo[k];
    int r = 0;
    const FlatNode* n = &nodes[k];
    if (n->leftChild == -1) {
        for (int i = 0; i < n->numShapes && !r; ++i) r = idx[n->startShapeIdx + i] == a;
    } else if (depth < 4096) {
        r = lists_shape(nodes, idx, n->leftChild, a, memo, depth + 1) |
            lists_shape(nodes, idx, n->rightChild, a, memo, depth + 1);
    }
    memo[k] = (signed char)r;
    return r;
}

int orc_update_bvh(const FlatShape* shapes, int S, FlatNode* nodes, int N, const int* idx, int I, const int* ids,
                   int count) {
    (void)I;
    signed char* memo = (signed char*)malloc((size_t)(N > 0 ? N : 1));
    if (!memo) return -1;
    for (int j = 0; j < count; ++j) {
        const int a = ids[j];
        if (a < 0 || a >= S) { free(memo); return -2; }
        memset(memo, -1, (size_t)(N > 0 ? N : 1));
        for (int k = 0; k < N; ++k) {
            if (!lists_shape(nodes, idx, k, a, memo, 0)) continue;
            box_t b = {fv(nodes[k].boundsMin), fv(nodes[k].boundsMax)};
            box_shape(&b, &shapes[a]);
            nodes[k].boundsMin.x = b.lo.x; nodes[k].boundsMin.y = b.lo.y; nodes[k].boundsMin.z = b.lo.z;
            nodes[k].boundsMax.x = b.hi.x; nodes[k].boundsMax.y = b.hi.y; nodes[k].boundsMax.z = b.hi.z;
        }
    }
    free(memo);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* Known-answer helpers for tests/                                           */

/* GLSL get_intersection for one shape and ray; returns the type, fills hit. */
int orc_intersect(const FlatShape* s, const float* o, const float* d, int use_mt, float* hit) {
    ray_t r;
    r.o = mk(o[0], o[1], o[2]);
    r.d = mk(d[0], d[1], d[2]);
    isect_t it = get_isect(s, r, use_mt);
    if (hit) { hit[0] = it.hit.x; hit[1] = it.hit.y; hit[2] = it.hit.z; }
    return it.type;
}

/* CPU-class get_intersection (cpuRayTracer's view), INNER/NONE/OUTER. */
int orc_intersect_cpu(const FlatShape* s, const float* o, const float* d, float* hit) {
    ray_t r;
    r.o = mk(o[0], o[1], o[2]);
    r.d = mk(d[0], d[1], d[2]);
    isect_t it = get_isect_cpu(s, r);
    if (hit) { hit[0] = it.hit.x; hit[1] = it.hit.y; hit[2] = it.hit.z; }
    return it.type;
}

/* getRay for one pixel: origin and direction. */
int orc_get_ray(const FlatCamera* cam, float ndcX, float ndcY, float* o, float* d) {
    ray_t r = get_ray(cam, ndcX, ndcY);
    o[0] = r.o.x; o[1] = r.o.y; o[2] = r.o.z;
    d[0] = r.d.x; d[1] = r.d.y; d[2] = r.d.z;
    return 0;
}

/* rayIntersectsAABB. */
int orc_ray_aabb(const float* o, const float* d, const float* bmin, const float* bmax) {
    ray_t r;
    r.o = mk(o[0], o[1], o[2]);
    r.d = mk(d[0], d[1], d[2]);
    return ray_aabb(r, mk(bmin[0], bmin[1], bmin[2]), mk(bmax[0], bmax[1], bmax[2]));
}

/* Wall::end (used by the builder). */
int orc_wall_end(const FlatShape* s, float* e) {
    v3 v = wall_end(s);
    e[0] = v.x; e[1] = v.y; e[2] = v.z;
    return 0;
}

/* Closest-hit (shape index or -1, distance) and shadow query (any INNER hit
 * nearer than lim) of the reference walk for arbitrary rays: the checker for
 * tests/native/accel_check.cpp. */
int orc_trace_rays_mt(const FlatShape* shapes, int S, const FlatNode* nodes, int N, const int* idx, int I,
                      const float* o, const float* d, const float* lim, int R, int* out_shape, float* out_d,
                      int* out_shadow, int use_mt);

int orc_trace_rays(const FlatShape* shapes, int S, const FlatNode* nodes, int N, const int* idx, int I,
                   const float* o, const float* d, const float* lim, int R, int* out_shape, float* out_d,
                   int* out_shadow) {
    return orc_trace_rays_mt(shapes, S, nodes, N, idx, I, o, d, lim, R, out_shape, out_d, out_shadow, 0);
}

/* The same with the Moller-Trumbore triangle test when use_mt (useMollerTrumbore). */
int orc_trace_rays_mt(const FlatShape* shapes, int S, const FlatNode* nodes, int N, const int* idx, int I,
                      const float* o, const float* d, const float* lim, int R, int* out_shape, float* out_d,
                      int* out_shadow, int use_mt) {
    rt_params p = {1, 1, 1, 1, 0, use_mt ? 1 : 0};
    scene_t sc = {shapes, S, nodes, N, idx, I, NULL, NULL, p};
#pragma omp parallel for schedule(dynamic, 64)
    for (int i = 0; i < R; ++i) {
        ray_t r;
        r.o = mk(o[3 * i], o[3 * i + 1], o[3 * i + 2]);
        r.d = mk(d[3 * i], d[3 * i + 1], d[3 * i + 2]);
        hit_t h = intersect_scene2(&sc, r, NULL);
        out_shape[i] = -1;
        out_d[i] = 1e20f;
        if (h.type == INNER) {
            out_shape[i] = (int)((const FlatShape*)((const char*)h.mat - offsetof(FlatShape, material)) - shapes);
            out_d[i] = distance3(r.o, h.hit);
        }
        float best = 1e20f;
        (void)best;
        out_shadow[i] = (h.type == INNER && distance3(r.o, h.hit) < lim[i]) ? 1 : 0;
    }
    return 0;
}

/* Every ray the BVH branch of main() traces for pixel (x, y): kind 0 =
 * closest-hit (primary/reflection), 1 = shadow; with the shadow query's
 * limit (min(light distance, 1e20)). Returns the ray count (<= cap).
 * Diagnostics for tests/tools only. */
int orc_pixel_rays(const FlatShape* shapes, int S, const FlatNode* nodes, int N, const int* idx, int I,
                   const FlatCamera* cam, const FlatLight* light, const rt_params* p, int x, int y,
                   float* o, float* d, float* lim, int* kind, int cap) {
    scene_t sc = {shapes, S, nodes, N, idx, I, cam, light, *p};
    int n = 0;
    float fx = (float)x, fy = (float)y;
    ray_t ray = get_ray(cam, 2.0f * fx / p->resX - 1.0f, 1.0f - 2.0f * fy / p->resY);
    v3 lpos = fv(light->position);
    for (int depth = 0; depth < p->maxBounces && n < cap; ++depth) {
        o[3 * n] = ray.o.x; o[3 * n + 1] = ray.o.y; o[3 * n + 2] = ray.o.z;
        d[3 * n] = ray.d.x; d[3 * n + 1] = ray.d.y; d[3 * n + 2] = ray.d.z;
        lim[n] = 1e20f; kind[n] = 0; ++n;
        hit_t hit = intersect_scene2(&sc, ray, NULL);
        if (hit.type != INNER || n >= cap) break;
        ray_t sr;
        sr.o = add(hit.hit, muls(hit.normal, 1e-3f));
        sr.d = normalize3(sub(lpos, hit.hit));
        o[3 * n] = sr.o.x; o[3 * n + 1] = sr.o.y; o[3 * n + 2] = sr.o.z;
        d[3 * n] = sr.d.x; d[3 * n + 1] = sr.d.y; d[3 * n + 2] = sr.d.z;
        lim[n] = fming(distance3(lpos, hit.hit), 1e20f); kind[n] = 1; ++n;
        if (!(hit.mat->specularStrength > 0)) break;
        v3 rd = reflect3(ray.d, hit.normal);
        ray.o = add(hit.hit, muls(hit.normal, 1e-3f));
        ray.d = rd;
    }
    return n;
}

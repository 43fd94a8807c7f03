/*
 * ort_oracle.c -- TEST INFRASTRUCTURE ONLY: CPU restatement of the reference's GPU path.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * (as the checker / the timed CPU baseline); the product (libort.so) never does.
 *
 * The reference has no CPU ray tracer: all tracing lives in
 * shaders/octree_fragment_shader.glsl, whose own build (GLFW window, Windows-only) cannot run
 * here.  This file restates that shader line by line in plain C over the
 * reference's buffer layout (SSBO bindings 0-6, glsl:20-46), with the canonical builtins of
 * include/ort_math.h.  Pinning: the octree input is byte-for-byte the
 * reference's own src/octree.cpp's (oracle/_ref/ref_octree, tests/golden); the pixels are
 * checked against the reference's own shaders run by the image's Mesa llvmpipe
 * (oracle/glsl_run.c, tests/golden/glsl, tests/test_glsl_parity.py): with GLSL's
 * implementation-defined builtins set to the canonical ones of include/ort_math.h
 * (oracle/glsl_canonical_builtins.glsl), this file's frames are BIT-IDENTICAL to the shader's
 * (18 frames, multi-bounce, depth-9/10 trees and the full C2 and C3 bench frames included; the
 * canonical prelude also reads the pixel centre from gl_FragCoord, exact, where llvmpipe's
 * interpolated FragCoord varying misses it by an ulp at some frame sizes); with llvmpipe's own builtins
 * within 1e-6 on >= 99.99 % of a primary-ray frame's pixels.

 * Differences from the GLSL, all forced: node offsets are int32 instead of float-in-
 * vec4.w; FragCoord is exactly (px+0.5, py+0.5) (vertex_shader.glsl:15);
 * the traversal order for the impossible zero sign vector is the identity.
 *
 * Build: gcc -O3 -ffp-contract=off -fopenmp -fPIC -shared (oracle/Makefile).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/ort_math.h"
#include "ort_oracle.h"

#define MAXFLOAT_F 3.402823466e+38f
#define PI_F ((float)3.14159265359)
#define LAMBERT 0
#define METAL 1
#define DIELECTRIC 2

typedef struct { float x, y, z; } vec3;
typedef struct { vec3 origin, direction; } Ray;
typedef struct {
    float t;
    vec3 point, normal;
    int materialType;
    vec3 albedo;
    float fuzz, refractionIndex;
} IntersectInfo;
typedef struct {
    vec3 origin, lowerLeftCorner, horizontal, vertical, u, v, w;
    float lensRadius;
} Camera;

typedef struct {
    const oracle_scene* sc;
    const oracle_params* pr;
    ort_rng randState;
    uint64_t* counts; /* ORACLE_COUNT_N, may be NULL */
} Ctx;

static vec3 v3(float x, float y, float z) { vec3 r = {x, y, z}; return r; }
static float dot3(vec3 a, vec3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static vec3 normalize3(vec3 v) { float s = 1.0f / sqrtf(dot3(v, v)); return v3(v.x * s, v.y * s, v.z * s); }
static vec3 cross3(vec3 x, vec3 y) { return v3(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y); }
static vec3 reflect3(vec3 I, vec3 N) {
    float k = 2.0f * dot3(N, I);
    return v3(I.x - k * N.x, I.y - k * N.y, I.z - k * N.z);
}
static void cnt(Ctx* c, int k, uint64_t v) { if (c->counts) c->counts[k] += v; }

/* rand2D glsl:89-101 lives in ort_math.h (ort_rand2D) */
static float rand2D(Ctx* c) { return ort_rand2D(&c->randState); }

/* glsl:104-147 */
static vec3 random_in_unit_disk(Ctx* c) {
    float spx = 2.0f * rand2D(c) - 1.0f;
    float spy = 2.0f * rand2D(c) - 1.0f;
    float r, phi;
    if (spx > -spy) {
        if (spx > spy) { r = spx; phi = spy / spx; }
        else { r = spy; phi = 2.0f - spx / spy; }
    } else {
        if (spx < spy) { r = -spx; phi = 4.0f + spy / spx; }
        else {
            r = -spy;
            if (spy != 0.0f) phi = 6.0f - spx / spy;
            else phi = 0.0f;
        }
    }
    phi *= PI_F / 4.0f;
    return v3(r * ort_cosf(phi), r * ort_sinf(phi), 0.0f);
}
/* glsl:149-159 */
static vec3 random_in_unit_sphere(Ctx* c) {
    float z = 2.0f * rand2D(c) - 1.0f;
    float phi = 2.0f * PI_F * rand2D(c);
    float r = ort_powf(rand2D(c), 1.0f / 3.0f);
    float sqrt1minz2 = sqrtf(1.0f - z * z);
    return v3(r * sqrt1minz2 * ort_cosf(phi), r * sqrt1minz2 * ort_sinf(phi), r * z);
}
/* glsl:161-173 */
static vec3 random_cosine_direction(Ctx* c) {
    float r1 = rand2D(c);
    float r2 = rand2D(c);
    float phi = 2.0f * PI_F * r1;
    float sqrt_r2 = sqrtf(r2);
    float x = ort_cosf(phi) * sqrt_r2;
    float y = ort_sinf(phi) * sqrt_r2;
    float z = sqrtf(1.0f - r2);
    return v3(x, y, z);
}

/* glsl:176-202 (view is column-major: GLSL viewMatrix[c][r] == view[4c+r]) */
static Camera Camera_initFromViewMatrix(const float* view, const float* position, float fovDegrees, float aspect) {
    Camera cam;
    cam.origin = v3(position[0], position[1], position[2]);
    vec3 wn = normalize3(v3(view[0 * 4 + 2], view[1 * 4 + 2], view[2 * 4 + 2]));
    cam.w = v3(-wn.x, -wn.y, -wn.z);
    cam.u = normalize3(v3(view[0 * 4 + 0], view[1 * 4 + 0], view[2 * 4 + 0]));
    cam.v = normalize3(v3(view[0 * 4 + 1], view[1 * 4 + 1], view[2 * 4 + 1]));
    float aperture = 0.1f;
    cam.lensRadius = aperture / 2.0f;
    float distToFocus = 10.0f;
    float theta = fovDegrees * PI_F / 180.0f;
    float halfHeight = ort_tanf(theta / 2.0f);
    float halfWidth = aspect * halfHeight;
    float a = halfWidth * distToFocus, b = halfHeight * distToFocus;
    cam.lowerLeftCorner = v3(((cam.origin.x - a * cam.u.x) - b * cam.v.x) - distToFocus * cam.w.x,
                             ((cam.origin.y - a * cam.u.y) - b * cam.v.y) - distToFocus * cam.w.y,
                             ((cam.origin.z - a * cam.u.z) - b * cam.v.z) - distToFocus * cam.w.z);
    float h2 = 2.0f * halfWidth * distToFocus, v2 = 2.0f * halfHeight * distToFocus;
    cam.horizontal = v3(h2 * cam.u.x, h2 * cam.u.y, h2 * cam.u.z);
    cam.vertical = v3(v2 * cam.v.x, v2 * cam.v.y, v2 * cam.v.z);
    return cam;
}

/* glsl:205-221 */
static Ray Camera_getRay(Ctx* c, const Camera* cam, float s, float t) {
    float W = (float)c->pr->width, H = (float)c->pr->height;
    float pixelRadius = 0.5f / ort_maxf(W, H);
    float jitterX = pixelRadius * (rand2D(c) - 0.5f);
    float jitterY = pixelRadius * (rand2D(c) - 0.5f);
    vec3 d = random_in_unit_disk(c);
    vec3 rd = v3(cam->lensRadius * d.x, cam->lensRadius * d.y, cam->lensRadius * d.z);
    vec3 offset = v3(cam->u.x * rd.x + cam->v.x * rd.y, cam->u.y * rd.x + cam->v.y * rd.y,
                     cam->u.z * rd.x + cam->v.z * rd.y);
    Ray ray;
    ray.origin = v3(cam->origin.x + offset.x, cam->origin.y + offset.y, cam->origin.z + offset.z);
    float a = s + jitterX, b = t + jitterY;
    ray.direction = normalize3(v3(
        (((cam->lowerLeftCorner.x + a * cam->horizontal.x) + b * cam->vertical.x) - cam->origin.x) - offset.x,
        (((cam->lowerLeftCorner.y + a * cam->horizontal.y) + b * cam->vertical.y) - cam->origin.y) - offset.y,
        (((cam->lowerLeftCorner.z + a * cam->horizontal.z) + b * cam->vertical.z) - cam->origin.z) - offset.z));
    return ray;
}

/* glsl:224-273 */
static int Sphere_hit(Ctx* c, int sphereIdx, Ray ray, float t_min, float t_max, IntersectInfo* rec) {
    const float* s = c->sc->sphere_center_radius + 4 * (size_t)sphereIdx;
    vec3 center = v3(s[0], s[1], s[2]);
    float radius = s[3];
    vec3 oc = v3(ray.origin.x - center.x, ray.origin.y - center.y, ray.origin.z - center.z);
    float a = dot3(ray.direction, ray.direction);
    float half_b = dot3(oc, ray.direction);
    float cc = dot3(oc, oc) - radius * radius;
    float discriminant = half_b * half_b - a * cc;
    if (discriminant > 0.0f) {
        float sqrtd = sqrtf(discriminant);
        for (int root = 0; root < 2; ++root) {
            float temp = root == 0 ? (-half_b - sqrtd) / a : (-half_b + sqrtd) / a;
            if (temp < t_max && temp > t_min) {
                rec->t = temp;
                rec->point = v3(ray.origin.x + temp * ray.direction.x, ray.origin.y + temp * ray.direction.y,
                                ray.origin.z + temp * ray.direction.z);
                rec->normal = v3((rec->point.x - center.x) / radius, (rec->point.y - center.y) / radius,
                                 (rec->point.z - center.z) / radius);
                const float* m = c->sc->sphere_mat_albedo + 4 * (size_t)sphereIdx;
                rec->materialType = (int)m[0];
                rec->albedo = v3(m[1], m[2], m[3]);
                const float* m2 = c->sc->sphere_fuzz_ri + 4 * (size_t)sphereIdx;
                rec->fuzz = m2[0];
                rec->refractionIndex = m2[1];
                cnt(c, ORACLE_COUNT_ACCEPTED_HITS, 1);
                return 1;
            }
        }
    }
    return 0;
}

/* glsl:276-288 */
static int rayBoxIntersection(Ray ray, vec3 boxMin, vec3 boxMax, float* tmin, float* tmax) {
    vec3 invDir = v3(1.0f / ray.direction.x, 1.0f / ray.direction.y, 1.0f / ray.direction.z);
    vec3 tbot = v3(invDir.x * (boxMin.x - ray.origin.x), invDir.y * (boxMin.y - ray.origin.y),
                   invDir.z * (boxMin.z - ray.origin.z));
    vec3 ttop = v3(invDir.x * (boxMax.x - ray.origin.x), invDir.y * (boxMax.y - ray.origin.y),
                   invDir.z * (boxMax.z - ray.origin.z));
    vec3 tmin3 = v3(ort_minf(tbot.x, ttop.x), ort_minf(tbot.y, ttop.y), ort_minf(tbot.z, ttop.z));
    vec3 tmax3 = v3(ort_maxf(tbot.x, ttop.x), ort_maxf(tbot.y, ttop.y), ort_maxf(tbot.z, ttop.z));
    *tmin = ort_maxf(ort_maxf(tmin3.x, tmin3.y), tmin3.z);
    *tmax = ort_minf(ort_minf(tmax3.x, tmax3.y), tmax3.z);
    return *tmax >= *tmin;
}

static int cmpv(int x, int y, int z, int a, int b, int cc) { return x == a && y == b && z == cc; }

/* glsl:341-447 */
static void traversal_order(vec3 d, int order[8]) {
    int cx = 0, cy = 0, cz = 0;
    if (d.x < 0.0f) cx = -1; else if (d.x > 0.0f) cx = 1;
    if (d.y < 0.0f) cy = -1; else if (d.y > 0.0f) cy = 1;
    if (d.z < 0.0f) cz = -1; else if (d.z > 0.0f) cz = 1;
    static const int T[8][8] = {
        {0, 1, 2, 3, 4, 5, 6, 7}, /* cyan */
        {2, 0, 3, 1, 6, 4, 7, 5}, /* yellow */
        {3, 1, 2, 0, 7, 5, 6, 4}, /* red */
        {1, 0, 3, 2, 5, 4, 7, 6}, /* dark purple */
        {4, 5, 6, 7, 0, 1, 2, 3}, /* blue */
        {6, 4, 7, 5, 2, 0, 3, 1}, /* purple */
        {7, 5, 6, 4, 3, 1, 2, 0}, /* green */
        {5, 4, 7, 6, 1, 0, 3, 2}, /* black */
    };
    int k;
    if (cmpv(cx, cy, cz, 1, 1, 1)) k = 0;
    else if (cmpv(cx, cy, cz, -1, 1, 1) || cmpv(cx, cy, cz, -1, 1, 0) || cmpv(cx, cy, cz, 0, 1, 0) ||
             cmpv(cx, cy, cz, 0, 1, 1)) k = 1;
    else if (cmpv(cx, cy, cz, -1, -1, 1) || cmpv(cx, cy, cz, -1, 0, 1) || cmpv(cx, cy, cz, 0, 0, 1) ||
             cmpv(cx, cy, cz, 0, -1, 1) || cmpv(cx, cy, cz, -1, -1, 0) || cmpv(cx, cy, cz, 0, -1, 0) ||
             cmpv(cx, cy, cz, -1, 0, 0)) k = 2;
    else if (cmpv(cx, cy, cz, 1, -1, 1) || cmpv(cx, cy, cz, 1, 0, 1) || cmpv(cx, cy, cz, 1, -1, 0) ||
             cmpv(cx, cy, cz, 1, 0, 0)) k = 3;
    else if (cmpv(cx, cy, cz, 1, 1, -1) || cmpv(cx, cy, cz, 1, 0, -1) || cmpv(cx, cy, cz, 0, 1, -1) ||
             cmpv(cx, cy, cz, 1, 1, 0)) k = 4;
    else if (cmpv(cx, cy, cz, -1, 1, -1)) k = 5;
    else if (cmpv(cx, cy, cz, -1, -1, -1) || cmpv(cx, cy, cz, -1, 0, -1) || cmpv(cx, cy, cz, 0, -1, -1) ||
             cmpv(cx, cy, cz, 0, 0, -1)) k = 6;
    else if (cmpv(cx, cy, cz, 1, -1, -1)) k = 7;
    else k = 0; /* zero vector: uninitialised in the GLSL */
    memcpy(order, T[k], sizeof(T[k]));
}

/* glsl:290-481 */
static int traverseOctree(Ctx* c, Ray ray, float t_min, float t_max, IntersectInfo* rec) {
    const oracle_scene* S = c->sc;
    enum { MAX_STACK = 200 };
    int nodeStack[MAX_STACK];
    float tminStack[MAX_STACK];
    float tmaxStack[MAX_STACK];
    int stackPtr = 0;
    nodeStack[0] = 0;
    tminStack[0] = t_min;
    tmaxStack[0] = t_max;
    int hit_anything = 0;
    float closest_so_far = t_max;
    float childTMin, childTMax;
    vec3 nodeMin = v3(S->node_min[0], S->node_min[1], S->node_min[2]);
    vec3 nodeMax = v3(S->node_max[0], S->node_max[1], S->node_max[2]);
    if (!rayBoxIntersection(ray, nodeMin, nodeMax, &childTMin, &childTMax)) return 0;
    int order[8];
    traversal_order(ray.direction, order); /* depends on the ray only; hoisted */
    while (stackPtr >= 0) {
        int nodeIdx = nodeStack[stackPtr];
        float node_tmin = tminStack[stackPtr];
        float node_tmax = tmaxStack[stackPtr--];
        (void)node_tmax;
        cnt(c, ORACLE_COUNT_NODES_POPPED, 1);
        int childrenOffset = S->children_offset[nodeIdx];
        int objectsOffset = S->objects_offset[nodeIdx];
        int objectCount = S->object_count[nodeIdx];
        if (childrenOffset == -1) {
            for (int i = 0; i < objectCount; i++) {
                IntersectInfo temp_rec;
                cnt(c, ORACLE_COUNT_LEAF_OBJECTS, 1);
                if (Sphere_hit(c, S->object_indices[objectsOffset + i], ray, node_tmin, closest_so_far, &temp_rec)) {
                    hit_anything = 1;
                    closest_so_far = temp_rec.t;
                    *rec = temp_rec;
                    stackPtr = -1;
                }
            }
        } else {
            for (int i = 7; i >= 0; i--) {
                int octant = order[i];
                int childIdx = childrenOffset + octant;
                if (childIdx >= S->n_nodes) continue;
                cnt(c, ORACLE_COUNT_CHILD_RECORDS, 1);
                vec3 childMin = v3(S->node_min[3 * (size_t)childIdx], S->node_min[3 * (size_t)childIdx + 1],
                                   S->node_min[3 * (size_t)childIdx + 2]);
                vec3 childMax = v3(S->node_max[3 * (size_t)childIdx], S->node_max[3 * (size_t)childIdx + 1],
                                   S->node_max[3 * (size_t)childIdx + 2]);
                if (!rayBoxIntersection(ray, childMin, childMax, &childTMin, &childTMax) ||
                    childTMax < node_tmin || childTMin > closest_so_far ||
                    (S->children_offset[childIdx] == -1 && S->objects_offset[childIdx] == -1))
                    continue;
                if (stackPtr < MAX_STACK - 1) {
                    stackPtr++;
                    nodeStack[stackPtr] = childIdx;
                    tminStack[stackPtr] = ort_maxf(childTMin, node_tmin);
                    tmaxStack[stackPtr] = ort_minf(childTMax, closest_so_far);
                }
            }
        }
    }
    return hit_anything;
}

/* glsl:484-498 */
static int bruteForceIntersect(Ctx* c, Ray ray, float t_min, float t_max, IntersectInfo* rec) {
    IntersectInfo temp_rec;
    int hit_anything = 0;
    float closest_so_far = t_max;
    for (int i = 0; i < c->sc->n_spheres; i++) {
        cnt(c, ORACLE_COUNT_LEAF_OBJECTS, 1);
        if (Sphere_hit(c, i, ray, t_min, closest_so_far, &temp_rec)) {
            hit_anything = 1;
            closest_so_far = temp_rec.t;
            *rec = temp_rec;
        }
    }
    return hit_anything;
}

/* glsl:500-506 */
static int intersectScene(Ctx* c, Ray ray, float t_min, float t_max, IntersectInfo* rec) {
    cnt(c, ORACLE_COUNT_TRAVERSALS, 1);
    if (c->pr->use_octree == 1) return traverseOctree(c, ray, t_min, t_max, rec);
    return bruteForceIntersect(c, ray, t_min, t_max, rec);
}

/* glsl:508-517 */
static int refractVec(vec3 v, vec3 n, float ni_over_nt, vec3* refracted) {
    vec3 uv = normalize3(v);
    float dt = dot3(uv, n);
    float discriminant = 1.0f - ni_over_nt * ni_over_nt * (1.0f - dt * dt);
    if (discriminant > 0.0f) {
        float s = sqrtf(discriminant);
        *refracted = v3(ni_over_nt * (uv.x - n.x * dt) - n.x * s, ni_over_nt * (uv.y - n.y * dt) - n.y * s,
                        ni_over_nt * (uv.z - n.z * dt) - n.z * s);
        return 1;
    }
    return 0;
}
/* glsl:519-523 */
static float schlick(float cosine, float refractionIndex) {
    float r0 = (1.0f - refractionIndex) / (1.0f + refractionIndex);
    r0 = r0 * r0;
    return r0 + (1.0f - r0) * ort_powf(1.0f - cosine, 5.0f);
}

/* glsl:525-589 */
static int Material_bsdf(Ctx* c, IntersectInfo isect, Ray wo, Ray* wi, vec3* attenuation) {
    wi->origin = isect.point;
    switch (isect.materialType) {
        case LAMBERT: {
            vec3 local_dir = random_cosine_direction(c);
            vec3 w = isect.normal;
            vec3 u = normalize3(cross3((fabsf(w.x) > 0.1f ? v3(0, 1, 0) : v3(1, 0, 0)), w));
            vec3 v = cross3(w, u);
            wi->direction = normalize3(v3((local_dir.x * u.x + local_dir.y * v.x) + local_dir.z * w.x,
                                          (local_dir.x * u.y + local_dir.y * v.y) + local_dir.z * w.y,
                                          (local_dir.x * u.z + local_dir.y * v.z) + local_dir.z * w.z));
            *attenuation = isect.albedo;
            return 1;
        }
        case METAL: {
            float fuzz = isect.fuzz;
            vec3 reflected = reflect3(normalize3(wo.direction), isect.normal);
            vec3 rs = random_in_unit_sphere(c);
            wi->direction = v3(reflected.x + fuzz * rs.x, reflected.y + fuzz * rs.y, reflected.z + fuzz * rs.z);
            *attenuation = isect.albedo;
            return dot3(wi->direction, isect.normal) > 0.0f;
        }
        case DIELECTRIC: {
            vec3 outward_normal;
            float ni_over_nt, cosine;
            float ri = isect.refractionIndex;
            *attenuation = v3(1.0f, 1.0f, 1.0f);
            if (dot3(wo.direction, isect.normal) > 0.0f) {
                outward_normal = v3(-isect.normal.x, -isect.normal.y, -isect.normal.z);
                ni_over_nt = ri;
                cosine = dot3(wo.direction, isect.normal) / sqrtf(dot3(wo.direction, wo.direction));
                cosine = sqrtf(1.0f - ri * ri * (1.0f - cosine * cosine));
            } else {
                outward_normal = isect.normal;
                ni_over_nt = 1.0f / ri;
                cosine = -dot3(wo.direction, isect.normal) / sqrtf(dot3(wo.direction, wo.direction));
            }
            float reflect_prob;
            vec3 refracted = v3(0, 0, 0);
            int can_refract = refractVec(wo.direction, outward_normal, ni_over_nt, &refracted);
            reflect_prob = can_refract ? schlick(cosine, ri) : 1.0f;
            if (rand2D(c) < reflect_prob) wi->direction = reflect3(wo.direction, isect.normal);
            else wi->direction = refracted;
            return 1;
        }
        default:
            return 0;
    }
}

/* glsl:592-595 */
static vec3 skyColor(Ray ray) {
    float t = 0.5f * (ray.direction.y + 1.0f);
    return v3((1.0f - t) * 1.0f + t * 0.5f, (1.0f - t) * 1.0f + t * 0.7f, (1.0f - t) * 1.0f + t * 1.0f);
}

/* glsl:597-633 */
static vec3 radiance(Ctx* c, Ray ray) {
    IntersectInfo rec;
    vec3 col = v3(1.0f, 1.0f, 1.0f);
    float importance = 1.0f;
    ray.direction = normalize3(ray.direction);
    for (int i = 0; i < c->pr->max_depth; i++) {
        if (importance < 0.01f) break;
        if (intersectScene(c, ray, 0.001f, MAXFLOAT_F, &rec)) {
            Ray wi;
            wi.direction = ray.direction;
            vec3 attenuation = v3(0, 0, 0);
            int wasScattered = Material_bsdf(c, rec, ray, &wi, &attenuation);
            ray.origin = wi.origin;
            ray.direction = wi.direction;
            if (wasScattered) col = v3(col.x * attenuation.x, col.y * attenuation.y, col.z * attenuation.z);
            else {
                col = v3(col.x * 0.0f, col.y * 0.0f, col.z * 0.0f);
                break;
            }
            importance *= ort_maxf(attenuation.x, ort_maxf(attenuation.y, attenuation.z));
        } else {
            vec3 s = skyColor(ray);
            col = v3(col.x * s.x, col.y * s.y, col.z * s.z);
            break;
        }
    }
    return col;
}

/* glsl:636-664 for one pixel; py = 0 is the bottom row */
static void shade(Ctx* c, const Camera* cam, int px, int py, float* out) {
    const oracle_params* P = c->pr;
    float fcx = (float)px + 0.5f, fcy = (float)py + 0.5f;
    float W = (float)P->width, H = (float)P->height;
    c->randState.x = fcx / W;
    c->randState.y = fcy / H;
    vec3 col = v3(0, 0, 0);
    for (int s = 0; s < P->num_samples; s++) {
        int sqrt_ns = (int)sqrtf((float)P->num_samples);
        int i = s % sqrt_ns;
        int j = s / sqrt_ns;
        float u = (fcx + ((float)i + rand2D(c)) / (float)sqrt_ns) / W;
        float v = (fcy + ((float)j + rand2D(c)) / (float)sqrt_ns) / H;
        Ray r = Camera_getRay(c, cam, u, v);
        vec3 rc = radiance(c, r);
        col = v3(col.x + rc.x, col.y + rc.y, col.z + rc.z);
    }
    float ns = (float)P->num_samples;
    col = v3(col.x / ns, col.y / ns, col.z / ns);
    float g = 1.0f / 2.2f;
    out[0] = ort_powf(col.x, g);
    out[1] = ort_powf(col.y, g);
    out[2] = ort_powf(col.z, g);
    cnt(c, ORACLE_COUNT_PIXELS, 1);
}

int oracle_render(const oracle_scene* sc, const oracle_params* pr, int x0, int y0, int tw, int th,
                  int band_height, int band_stride, float* out, uint64_t* counts, int nthreads) {
    if (!sc || !pr || !out || tw < 0 || th < 0) return 1;
    if (pr->use_octree == 1 && sc->n_nodes <= 0) return 2;
    Camera cam = Camera_initFromViewMatrix(pr->view, pr->camera_position, pr->camera_zoom,
                                           (float)pr->width / (float)pr->height);
    if (counts) memset(counts, 0, sizeof(uint64_t) * ORACLE_COUNT_N);
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    long long rows = th;
#pragma omp parallel
    {
        uint64_t local[ORACLE_COUNT_N];
        memset(local, 0, sizeof(local));
        Ctx c;
        c.sc = sc;
        c.pr = pr;
        c.counts = counts ? local : NULL;
#pragma omp for schedule(dynamic, 1)
        for (long long j = 0; j < rows; ++j) {
            int y = band_height > 0 ? y0 + (int)(j / band_height) * band_stride + (int)(j % band_height) : y0 + (int)j;
            for (int col = 0; col < tw; ++col) {
                float* o = out + 3 * ((size_t)j * (size_t)tw + (size_t)col);
                if (y >= pr->height) { o[0] = o[1] = o[2] = 0.0f; continue; }
                shade(&c, &cam, x0 + col, y, o);
            }
        }
        if (counts) {
#pragma omp critical
            for (int k = 0; k < ORACLE_COUNT_N; ++k) counts[k] += local[k];
        }
    }
    return 0;
}

int oracle_camera(const oracle_params* pr, float* out22) {
    Camera cam = Camera_initFromViewMatrix(pr->view, pr->camera_position, pr->camera_zoom,
                                           (float)pr->width / (float)pr->height);
    memcpy(out22, &cam, sizeof(float) * 22);
    return 0;
}

float oracle_sin(float x) { return ort_sinf(x); }
float oracle_cos(float x) { return ort_cosf(x); }
float oracle_pow(float x, float y) { return ort_powf(x, y); }
float oracle_tan(float x) { return ort_tanf(x); }
void oracle_rand_sequence(float sx, float sy, int n, float* out) {
    ort_rng st = {sx, sy};
    for (int i = 0; i < n; ++i) out[i] = ort_rand2D(&st);
}
void oracle_traversal_order(float dx, float dy, float dz, int* order8) { traversal_order(v3(dx, dy, dz), order8); }
/* intersectScene(ray, 0.001, MAXFLOAT) for given rays (rays[6 i] = origin, direction):
 * out[2 i] = 1 if it hit, out[2 i + 1] = bits of the hit t */
void oracle_trace_rays(const oracle_scene* sc, const float* rays, int n, int* out) {
    oracle_params pr;
    memset(&pr, 0, sizeof(pr));
    pr.use_octree = 1;
    Ctx c;
    c.sc = sc;
    c.pr = &pr;
    c.counts = NULL;
    for (int i = 0; i < n; ++i) {
        Ray r;
        r.origin = v3(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]);
        r.direction = v3(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
        IntersectInfo rec;
        memset(&rec, 0, sizeof(rec));
        const int hit = intersectScene(&c, r, 0.001f, MAXFLOAT_F, &rec);
        out[2 * i] = hit ? 1 : 0;
        memcpy(&out[2 * i + 1], &rec.t, 4);
    }
}

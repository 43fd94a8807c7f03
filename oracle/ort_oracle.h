/* ort_oracle.h -- TEST INFRASTRUCTURE ONLY (see ort_oracle.c). */
#ifndef ORT_ORACLE_H
#define ORT_ORACLE_H
#include <stdint.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* reference-layout scene: SSBO bindings 0-6 (glsl:20-46), offsets as int32 */
typedef struct oracle_scene {
    const float* sphere_center_radius; /* 4 per sphere */
    const float* sphere_mat_albedo;    /* 4 per sphere */
    const float* sphere_fuzz_ri;       /* 4 per sphere */
    int n_spheres;
    const float* node_min; /* 3 per node */
    const float* node_max; /* 3 per node */
    const int* children_offset;
    const int* objects_offset;
    const int* object_count;
    int n_nodes;
    const int* object_indices;
    long long n_indices;
} oracle_scene;

/* the uniforms; same layout as ort_params in include/ort.h */
typedef struct oracle_params {
    int width, height, num_samples, max_depth, use_octree;
    float view[16];
    float camera_position[3];
    float camera_zoom;
} oracle_params;

#define ORACLE_COUNT_NODES_POPPED 0
#define ORACLE_COUNT_CHILD_RECORDS 1
#define ORACLE_COUNT_LEAF_OBJECTS 2
#define ORACLE_COUNT_ACCEPTED_HITS 3
#define ORACLE_COUNT_PIXELS 4
#define ORACLE_COUNT_TRAVERSALS 5
#define ORACLE_COUNT_N 6

int oracle_render(const oracle_scene* sc, const oracle_params* pr, int x0, int y0, int tw, int th,
                  int band_height, int band_stride, float* out, uint64_t* counts, int nthreads);
int oracle_camera(const oracle_params* pr, float* out22);
float oracle_sin(float x);
float oracle_cos(float x);
float oracle_pow(float x, float y);
float oracle_tan(float x);
void oracle_rand_sequence(float sx, float sy, int n, float* out);
void oracle_traversal_order(float dx, float dy, float dz, int* order8);
void oracle_trace_rays(const oracle_scene* sc, const float* rays, int n, int* out);

#endif

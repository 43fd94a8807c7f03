// ort_internal.h -- internal declarations shared by the host .cpp files and the .hip file.
#pragma once
#include <cstdint>
#include <string>

#include "../../include/ort.h"

namespace ort {
void set_thread_error(const std::string& msg);
const char* thread_error();
}  // namespace ort

// The ort_debug_* entry points below exist in the analysis library only (Makefile `analysis`,
// -DORT_ANALYSIS=1: octreeraytracer_amd/lib/libort_analysis.so); libort.so exports include/ort.h.
extern "C" {
// TEST-ONLY: run the kernel's per-pixel code (render_core.h, compact or explicit layout)
// on the host CPU, single-threaded, for CPU-side validation of the traversal logic
// against the independent oracle.  Never called by ort_render (which has no CPU path).
int ort_debug_emulate_render(const float* sphere_center_radius, const float* sphere_mat_albedo,
                             const float* sphere_fuzz_ri, int32_t n_spheres, const float* node_min,
                             const float* node_max, const int32_t* children_offset,
                             const int32_t* objects_offset, const int32_t* object_count, int32_t n_nodes,
                             const int32_t* object_indices, int64_t n_indices, int32_t layout,
                             const ort_params* params, const ort_tile* tile, float* rgb_out, uint64_t* counts);
// TEST-ONLY: the ort_group partition and assembly with an in-memory transport: each of the
// `world` band tiles rendered by ort_debug_emulate_render, then assembled by the device
// kernel's row map (group_map.h).  Full frame into rgb_out (host).
int ort_debug_group_emulate(const float* sphere_center_radius, const float* sphere_mat_albedo,
                            const float* sphere_fuzz_ri, int32_t n_spheres, const float* node_min,
                            const float* node_max, const int32_t* children_offset, const int32_t* objects_offset,
                            const int32_t* object_count, int32_t n_nodes, const int32_t* object_indices,
                            int64_t n_indices, int32_t world, const ort_params* params, float* rgb_out);
// TEST-ONLY: the fast walk's traversal order for direction-sign mask m = (d.z<0)<<2 |
// (d.x<0)<<1 | (d.y<0) (render_core.h rank_perm: order[r] = perm(r) ^ m) and its rank LUT
// rows (rank_lut_entry) for every child mask: lut256[cmask] (checked against the shader's
// tables, tests/golden/traversal_orders.json).
int ort_debug_fast_order(int32_t m, int32_t* order8, uint8_t* lut256);
// TEST-ONLY: the split walk (render_core.h traverse_split, the walk of ort_trace_split) of each
// ray run by `lanes` lanes one after another, level-`level` subtrees dealt round robin, merged by
// the lowest DFS position; out[4 i] = {hit entry (-1 none), t bits, position, summed steps}.
int ort_debug_split_rays(const float* sphere_center_radius, int32_t n_spheres, const float* node_min,
                         const float* node_max, const int32_t* children_offset, const int32_t* objects_offset,
                         const int32_t* object_count, int32_t n_nodes, const int32_t* object_indices,
                         int64_t n_indices, const float* rays, int32_t n_rays, int32_t level, int32_t lanes,
                         int32_t* out);
// TEST-ONLY: per ray (origin.xyz, direction.xyz in rays[6 i]) the fast walk where the kernels
// would take it (fast_prepare) and the exact walk (traverse_compact, literal GLSL min/max);
// out[5 i] = {fast taken, fast entry, fast t bits, exact entry, exact t bits}.  bounce != 0:
// the bounce walk (no inline leaf children, the rejected-sphere skip).
int ort_debug_trace_rays(const float* sphere_center_radius, int32_t n_spheres, const float* node_min,
                         const float* node_max, const int32_t* children_offset, const int32_t* objects_offset,
                         const int32_t* object_count, int32_t n_nodes, const int32_t* object_indices, int64_t n_indices,
                         const float* rays, int32_t n_rays, int32_t bounce, int32_t* out);
// ANALYSIS-ONLY: lane overlap of sampled 8x8 primary-ray blocks (tools/wave_stats.py).
int ort_debug_wave_stats(const float* sphere_center_radius, const float* sphere_mat_albedo,
                         const float* sphere_fuzz_ri, int32_t n_spheres, const float* node_min,
                         const float* node_max, const int32_t* children_offset, const int32_t* objects_offset,
                         const int32_t* object_count, int32_t n_nodes, const int32_t* object_indices,
                         int64_t n_indices, const ort_params* params, int32_t block_step, double* stats,
                         int32_t n_stats);
// ANALYSIS-ONLY: the per-step work of the fast walk (the kernel's own fast_step, inline leaf
// children) for the 64 lanes of sampled 8x8 primary-ray blocks (tools/walk_sim.py).
// lens[64 * w + l] = steps of lane l of sampled wave w (0: not a fast-walk lane); steps[] =
// the lanes' steps back to back, one uint16 each: objects tested (bits 0-7, saturated),
// leaf children tested (bits 8-11), bit 15 = the step's node has leaf children (LEAFKIDS).
// Returns the number of steps (or, if cap is too small, minus the number needed).
int ort_debug_bounce_walks(const float* sphere_center_radius, const float* sphere_mat_albedo,
                           const float* sphere_fuzz_ri, int32_t n_spheres, const float* node_min, const float* node_max,
                           const int32_t* children_offset, const int32_t* objects_offset, const int32_t* object_count,
                           int32_t n_nodes, const int32_t* object_indices, int64_t n_indices, const ort_params* params,
                           const ort_tile* tile, int32_t bounce, float* rays, int32_t* walks, int64_t cap,
                           int64_t* n_out);
int64_t ort_debug_walk_steps(const float* sphere_center_radius, const float* sphere_mat_albedo,
                             const float* sphere_fuzz_ri, int32_t n_spheres, const float* node_min,
                             const float* node_max, const int32_t* children_offset, const int32_t* objects_offset,
                             const int32_t* object_count, int32_t n_nodes, const int32_t* object_indices,
                             int64_t n_indices, const ort_params* params, int32_t block_step, int32_t* lens,
                             int64_t n_lens, uint16_t* steps, int64_t cap);
}

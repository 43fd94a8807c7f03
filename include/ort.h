/*
 * ort.h -- C ABI of the MI355X octree ray tracer (libort.so).
 *
 * This is the drop-in boundary that replaces the reference's OpenGL path:
 *
 *   reference (GL, Tiago27Cruz/OctreeRayTracer)                         this ABI
 *   ---------------------------------------------------------------------------------------
 *   Raytracer::initialize -> startGLFW/setupQuad/setupShader         ort_create
 *     (src/raytracer.cpp:32-60, src/main.cpp:60-102)
 *   Raytracer::setupBuffers: 7x glBufferData SSBOs + static uniforms ort_upload_scene /
 *     (src/raytracer.cpp:74-152; SSBO bindings glsl:20-46)             ort_upload_octree
 *   per-frame uniforms view/cameraPosition/cameraZoom + glDrawArrays ort_render
 *     (src/raytracer.cpp:491-499; uniforms glsl:13-18, 48-53)
 *   Raytracer::cleanupBuffers (src/raytracer.cpp:154-162)            ort_destroy
 *   (GL errors never checked; shader errors printed, shader.cpp:52-78) ort_last_error
 *
 * Conventions: every call returns an int status (ORT_OK == 0); no C++ exception crosses
 * the ABI.  The context owns all device memory; host arrays passed in are copied.  One
 * context per device; calls on one context are not thread-safe, different contexts may
 * be driven from different threads.  ort_render is synchronous when stream == NULL and
 * stream-ordered (asynchronous) otherwise.
 *
 * Deliberate deviation: node offsets are int32, not float as in the
 * reference's vec4.w packing (src/raytracer.cpp:98-99), which is exact only below 2^24.
 */
#ifndef ORT_H
#define ORT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORT_OK 0
#define ORT_ERR_INVALID_ARG 1
#define ORT_ERR_HIP 2
#define ORT_ERR_NO_SCENE 3
#define ORT_ERR_OUT_OF_MEMORY 4
#define ORT_ERR_UNSUPPORTED 5
#define ORT_ERR_INTERNAL 6
#define ORT_ERR_TIMEOUT 7     /* a bounded wait expired (ort_group_wait: the message names the slot and the
                                 ranks whose render or band send had not completed) */

typedef struct ort_ctx ort_ctx;

/* The shader's uniforms (glsl:13-18, 48-53).  view is column-major like glm::mat4
 * (view[4*col + row]); model/projection are unused by the reference shader. */
typedef struct ort_params {
    int32_t width, height;      /* iResolution.xy of the FULL frame (src/raytracer.cpp:150) */
    int32_t num_samples;        /* numSamples (src/config.h:20) */
    int32_t max_depth;          /* maxDepth: bounces per path (src/config.h:23, MAXRAYSDEPTH) */
    int32_t use_octree;         /* useOctree: 1 octree traversal, 0 brute force (glsl:500-506) */
    float view[16];             /* view matrix uniform */
    float camera_position[3];   /* cameraPosition uniform */
    float camera_zoom;          /* cameraZoom uniform: vertical field of view in degrees */
} ort_params;

/* Which pixels to render.  Output row j (0-based) is pixel row
 *     y = y0 + (j / band_height) * band_stride + (j % band_height)
 * (band_height <= 0 means one band: y = y0 + j).  Pixel rows are GL rows: y = 0 is the
 * BOTTOM row of the image.  Columns are x0 .. x0+width-1.  Rows with y >= height are
 * written as zeros.  The RNG seed and the camera always use the full-frame resolution,
 * so any tiling produces the same pixels as a full-frame render. */
typedef struct ort_tile {
    int32_t x0, width;
    int32_t y0, rows;
    int32_t band_height;
    int32_t band_stride;
} ort_tile;

/* Per-scene information after upload. */
typedef struct ort_scene_info {
    int32_t n_spheres;
    int32_t n_nodes;
    int64_t n_indices;
    int32_t layout;            /* ORT_LAYOUT_* actually selected */
    int32_t tree_depth;        /* deepest node level (root = 0) */
    int64_t device_bytes;      /* device memory held for the scene */
} ort_scene_info;

#define ORT_LAYOUT_COMPACT 0   /* 8-byte node records, boxes re-derived from per-axis split planes */
#define ORT_LAYOUT_EXPLICIT 1  /* reference record layout, boxes read from memory */

/* Options (ort_set_option). */
#define ORT_OPT_FORCE_LAYOUT 1     /* -1 auto (default), or ORT_LAYOUT_* */
#define ORT_OPT_EXACT_TRAVERSAL 2  /* 1: disable the sign-specialised fast walk (A/B testing; same pixels) */
#define ORT_OPT_REFILL 3           /* persistent trace: refill a wave when >= value of its 64 lanes idle (16) */
#define ORT_OPT_PERSISTENT 4       /* persistent trace kernel with per-lane ray refill: 0 off, 2 (default)
                                      bounce >= 1 traces only: their incoherent rays gain from
                                      refilling idle lanes (C5 -4.5 %); 1 (every trace) was removed in
                                      round 4 (C5 -19 %): ORT_ERR_UNSUPPORTED */
#define ORT_OPT_SORT_PATHS 6       /* order of the alive paths between bounces (coherence; same pixels):
                                      2 (default) radix-sort the compacted list by direction octant +
                                      origin cell + direction; the list's length stays on the device
                                      (the sort's size is the same bounce's length in the previous
                                      frame of the same shape + 1/64 + 1024, read back asynchronously;
                                      a longer list goes on unsorted): no host wait; 1 sort every
                                      slot's key; 0 slot order */
#define ORT_OPT_XCD_SWIZZLE 8      /* workgroup -> tile order (same pixels): 2 each XCD renders runs of
                                      consecutive raster tiles (about 1/15 of a tile row, a power of
                                      two: 16 at 3840 px); 1: each XCD renders 128x128-pixel
                                      super-tiles; 0: raster order (tile b on XCD b % 8); -1 (default):
                                      0 for one-tile workgroups on tiles of at most 1.5 M pixels (a
                                      C3 1/8 band at one frame in flight -3 %), 2 otherwise */
#define ORT_OPT_KID_SKIP 9         /* 1 (default): a lane skips one-sphere leaf children holding the sphere it
                                      last rejected at a tmin <= theirs (they cannot end the walk; same
                                      pixels, kid_table.h), a node's record and kid entry loaded together
                                      from the interleaved copy; 2: the skip with the record and kid
                                      entry from their own arrays (testing; same pixels); 0: walk them
                                      as the reference does */
#define ORT_OPT_SORT_BOUND 10      /* testing: > 0 forces the size of the list sort (SORT_PATHS 2) to this
                                      bound -- below the list's length the list goes on in append
                                      order (same pixels); 0 (default): the hint described above */
#define ORT_OPT_COST_ORDER 11      /* 1 (default): each workgroup of the camera-ray trace deals its 16x16
                                      pixels to its waves ordered by the walk steps each pixel's ray took
                                      in the previous frame of the same shape (rays of like cost share a
                                      wave; same pixels); 0: the fixed 8x8 block per wave */
#define ORT_OPT_HEAVY_FIRST 12     /* T > 0 (default 64): the sorted bounce lists (SORT_PATHS 2, persistent
                                      trace) order paths by the steps their walk at that bounce took in
                                      the previous frame of the same shape -- >= 4T first, then >= 2T,
                                      >= T, the rest, each class in coherence order -- so the longest
                                      walks start early rather than in the launch's drain tail.  After a
                                      camera move (the steps are stale) the classes come from the rays
                                      themselves instead: the distance to the root box's exit, within
                                      1.2 / 2.7 / 6.8 x its smallest extent.  Same pixels.  0: coherence
                                      order only */
#define ORT_OPT_HEAVY_PRIO 13      /* T > 0 (default 150): a wave of the camera-ray trace (cost order on)
                                      that holds a ray whose walk took >= T steps in the previous frame of
                                      the same shape runs at raised issue priority (s_setprio), so the
                                      frame's longest walks do not set its end -- while the camera stands
                                      still (after a move the steps are stale); 0: off.  Same pixels */
#define ORT_OPT_SPLIT_HEAVY 14     /* T > 0 (1 sample, cost order on): the camera rays whose walk took >= T
                                      steps in the previous frame of the same shape (up to 4096 a frame)
                                      are each walked by 8 lanes that deal the walk's subtrees of level
                                      ORT_OPT_SPLIT_LEVEL round robin (the first hit = the hit of the
                                      lowest such subtree in the walk's order), on a second stream beside
                                      the per-tile kernel: a small tile's frame no longer waits for its
                                      longest walks.  0: off.  -1 (default): T = 200 on tiles of at most
                                      2^21 pixels, off on larger ones (where the second stream costs more
                                      than the tail it cuts).  A caller that keeps several frames in
                                      flight should set 0: the next frames fill the tail (C3 1/8 band at
                                      3 in flight: 0.266 -> 0.227 ms/frame); pipelined groups do.
                                      Same pixels */
#define ORT_OPT_SPLIT_LEVEL 15     /* the level of those subtrees: 0 (default) = tree depth - 5 (at least 1) */
#define ORT_OPT_TILE_PAIRS 16      /* 1: a camera-ray workgroup renders two 16x16 tiles side by side, its 512
                                      pixels dealt to 8 blocks of 64 by last frame's walk steps and each
                                      wave walking a heavy and a light block (a workgroup keeps its LDS
                                      until its slowest wave ends); 0: a tile per workgroup; -1 (default):
                                      pairs on tiles of more than 2^21 pixels, or on any tile when
                                      ORT_OPT_SPLIT_HEAVY is 0 (on small tiles at one frame in flight the
                                      fewer, longer workgroups lengthen the frame's tail).  Same pixels */
#define ORT_OPT_DEBUG_FLAGS 18     /* analysis library only (libort_analysis.so, tools/ab_stream.py): 1 records
                                      no per-launch trace-timing events, 2 scans the heavy list at the start
                                      of each split frame; libort.so: ORT_ERR_UNSUPPORTED */
#define ORT_OPT_LAUNCH_TIMES 19    /* 1 (default): HIP events time every trace launch of a frame
                                      (ort_last_trace_ms, ort_trace_times_ms, ort_frame_trace_times_ms);
                                      0: only the frame's start and end are timed (ort_last_kernel_ms) --
                                      fewer event packets on the stream: a C3 1/8 band at one frame in
                                      flight 0.297 -> 0.291 ms; the per-launch queries then report
                                      no newer launch (ort_last_trace_ms: an error while none was ever
                                      timed).  Same pixels */
#define ORT_OPT_PIXEL_PATHS 20    /* whole-pixel paths: the frame in ONE launch, each lane stepping a pixel's
                                      samples and bounces in turn (the RNG state runs on from one sample to the
                                      next, glsl:640, so a pixel is a sequential chain) and taking the next
                                      pixel when done -- instead of the per-sample, per-bounce pipeline (trace,
                                      shade, list sort launches).  -1 (default): on for frames of more than one
                                      traversal per pixel on brute force, on trees of at most 2^19 nodes,
                                      2^23 with maxDepth 5-7 and 2^24 with maxDepth 8 or more (the
                                      reference's sweeps: launches and sorts dominate, more so the more
                                      bounces; larger trees keep the pipeline's sorted bounce rays); 0 off; 1 on wherever it applies (compact layout or brute
                                      force, maxDepth >= 1, not 1 sample x 1 bounce).  Same pixels */
#define ORT_OPT_PIXEL_LDS_SCENE 21 /* 1 (default): whole-pixel paths on scenes whose node records and leaf
                                      spheres fit 32 KB (depth <= 8) copy them into each workgroup's LDS and
                                      walk them there; 0: from global memory.  Same pixels */
#define ORT_OPT_PIXEL_HEAVY_FIRST 22 /* whole-pixel paths: the frame's 8x8 blocks taken in the order of the
                                      previous frame's cost (bounces per sample, 32 classes, heaviest first)
                                      when that frame had the same shape and scene, so the longest pixel
                                      chains start first and do not trail the frame; tile order otherwise.
                                      -1 (default): on for frames of 2 or more samples; 0 off; 1 on.  Same
                                      pixels (the order changes which lane traces a pixel, not its chain) */
#define ORT_OPT_PIXEL_SPECULATE 23 /* whole-pixel paths, 5+ samples: from the second frame of a shape on,
                                      a pixel's samples are traced as up to 4 chunks (of 4 or more
                                      samples) in parallel, chunk c
                                      starting from the RNG state chunk c-1 ended with in the previous
                                      frame (it only depends on how many draws the paths took); a pixel
                                      whose chunk ends in another state than last frame's has its later
                                      samples re-traced from the true state, and every pixel's samples
                                      are summed in order: same pixels, and a frame no longer waits for
                                      its longest pixel's chain.  -1 (default) and 1: on while the
                                      buffers (12 B per sample and path slot, 16 B per chunk) fit 8 GiB;
                                      0: off */
/* Retired option codes, reserved (ORT_ERR_UNSUPPORTED): options that lost to the defaults in
 * A/B and were removed -- 5 the wave-level packet walk (1.2-1.35x slower),
 * 7 the wave-level block queue (1/8 band 0.83 vs 0.61 ms), 17 longest-first workgroups
 * (C3 -25 %).  ORT_OPT_PERSISTENT value 1 is refused likewise (C5 -19 %). */
#define ORT_OPT_IS_RETIRED(o) ((o) == 5 || (o) == 7 || (o) == 17)

/* Traffic counters (ort_count_traffic), in the REFERENCE layout's terms. */
#define ORT_COUNT_NODES_POPPED 0
#define ORT_COUNT_CHILD_RECORDS 1
#define ORT_COUNT_LEAF_OBJECTS 2
#define ORT_COUNT_ACCEPTED_HITS 3
#define ORT_COUNT_PIXELS 4
#define ORT_COUNT_TRAVERSALS 5
#define ORT_COUNT_N 6

/* ---- device context ---------------------------------------------------------------- */
int ort_create(int device, ort_ctx** out);
int ort_destroy(ort_ctx* ctx);
/* Last error message for ctx (or of the calling thread when ctx == NULL). Never NULL. */
const char* ort_last_error(const ort_ctx* ctx);
int ort_set_option(ort_ctx* ctx, int option, int value);

/* Upload a scene in the reference's packing (src/raytracer.cpp:87-101), SoA:
 *   sphere_center_radius[4*i]  = center.xyz, radius          (SSBO binding 0)
 *   sphere_mat_albedo[4*i]     = float(materialType), albedo (SSBO binding 1)
 *   sphere_fuzz_ri[4*i]        = fuzz, refractionIndex, 0, 0 (SSBO binding 2)
 *   node_min[3*k], node_max[3*k], children_offset[k], objects_offset[k], object_count[k]
 *                                                            (SSBO bindings 3, 4, 5)
 *   object_indices[n_indices]                                (SSBO binding 6)
 * Replaces any previous scene on the context. */
int ort_upload_scene(ort_ctx* ctx,
                     const float* sphere_center_radius, const float* sphere_mat_albedo,
                     const float* sphere_fuzz_ri, int32_t n_spheres,
                     const float* node_min, const float* node_max,
                     const int32_t* children_offset, const int32_t* objects_offset,
                     const int32_t* object_count, int32_t n_nodes,
                     const int32_t* object_indices, int64_t n_indices);

/* Same, taking Octree::flattenedTree.data() directly (36-byte GPUOctreeNode records). */
int ort_upload_octree_nodes(ort_ctx* ctx,
                            const float* sphere_center_radius, const float* sphere_mat_albedo,
                            const float* sphere_fuzz_ri, int32_t n_spheres,
                            const void* gpu_octree_nodes, int32_t n_nodes,
                            const int32_t* object_indices, int64_t n_indices);

int ort_scene_get_info(const ort_ctx* ctx, ort_scene_info* info);

/* Build the octree ON THE GPU and make it ctx's scene: replaces Octree::build + setGPUData
 * (src/octree.cpp:47-95, 189-229, 231-242, 268-312) followed by ort_upload_scene, without the
 * host tree.  Same tree, byte for byte: root box from the sphere bounds, midpoint octants,
 * sphereIntersectsBox distribution, BFS numbering, objectIndices in BFS leaf order
 * (level-synchronous build, octreeraytracer_amd/csrc/gpu_build.hip).  n_spheres == 0 fails
 * with ORT_ERR_INVALID_ARG "Sphere list is empty" like the reference's std::invalid_argument.
 * keep_tree != 0 keeps the reference-layout arrays on the device for ort_scene_export_octree. */
int ort_build_scene(ort_ctx* ctx, const float* sphere_center_radius, const float* sphere_mat_albedo,
                    const float* sphere_fuzz_ri, int32_t n_spheres, int32_t max_depth, int32_t max_spheres_per_node,
                    int32_t keep_tree);
/* Copy the kept GPU-built tree to host arrays (sizes: ort_scene_get_info n_nodes x 3 floats /
 * n_nodes ints / n_indices ints): the Octree::flattenedTree fields and objectIndices. */
int ort_scene_export_octree(ort_ctx* ctx, float* node_min, float* node_max, int32_t* children_offset,
                            int32_t* objects_offset, int32_t* object_count, int32_t* object_indices);
/* Device time of the last ort_build_scene (HIP events; the reference's Octree::buildTime). */
int ort_last_build_ms(const ort_ctx* ctx, float* ms);

/* The context's own HIP stream (created non-blocking by ort_create), for callers that keep
   several frames in flight on several contexts: a frame rendered on each context's stream
   overlaps the tail of the previous frame (bench.py --inflight).  No reference counterpart. */
int ort_get_stream(const ort_ctx* ctx, void** stream);

/* Render the tile; rgb_out receives tile->rows * tile->width RGB float triples, row-major,
 * output row 0 first.  out_is_device != 0: rgb_out is a device pointer on ctx's device.
 * stream: a hipStream_t on ctx's device (stream-ordered, returns at once -- also for
 * multi-sample / multi-bounce frames: no step of the frame waits on the host; the first
 * frame of a new shape may allocate, and hipMalloc/hipFree synchronise the device), or NULL
 * for the context's own stream (then the call returns after the frame is complete).  The HIP
 * null stream has the NULL handle, so passing it also means "synchronous".  Two frames in
 * flight on one context must not overlap: render the next one on the same stream or wait. */
int ort_render(ort_ctx* ctx, const ort_params* params, const ort_tile* tile,
               float* rgb_out, int out_is_device, void* stream);

/* Duration in milliseconds of the last ort_render's kernels (the whole per-frame pipeline),
 * from HIP events recorded on its stream.  Only valid once that stream has passed the frame. */
int ort_last_kernel_ms(ort_ctx* ctx, float* ms);

/* Duration in milliseconds of the first trace kernel (camera rays + octree walk of bounce
 * 0, sample 0: the dominant kernel) of the last ort_render, from HIP events on its stream. */
int ort_last_trace_ms(ort_ctx* ctx, float* ms);

/* The same for the last n frames (at most 64), oldest first; returns how many were
 * written, or a negative ORT_ERR_* code. */
int ort_trace_times_ms(ort_ctx* ctx, int n, float* ms);

/* Per frame, the summed duration of ALL its trace kernels (every sample and bounce: camera
 * rays and the bounce >= 1 walks; at most the first 16 trace launches of a frame are timed),
 * last n frames (at most 64), oldest first; launches[i] (may be NULL) receives how many
 * launches frame i summed.  Returns how many frames were written, or a negative ORT_ERR_*.
 * Shading, path sorting and the deferred-ray exact walk are not included. */
int ort_frame_trace_times_ms(ort_ctx* ctx, int n, float* ms, int32_t* launches);

/* Run the counting variant of the kernel over the tile and return, summed over all
 * pixels, the reference-layout work counters ORT_COUNT_* (counts[ORT_COUNT_N]). */
int ort_count_traffic(ort_ctx* ctx, const ort_params* params, const ort_tile* tile, uint64_t* counts);

/* ---- several GPUs, one process --------------------------------------
 * The reference renders on one GL context; a caller of Raytracer::render() reaches the 8-GPU
 * configs through a group: one context per listed device (scene replicated), the frame cut
 * into 16-row bands dealt round-robin (rank r renders bands r, r+N, ...; every rank the same
 * number of rows), ONE exchange -- the bands gathered to devices[0] -- and a de-interleave
 * kernel there.  Pixels equal a single-context render bit for bit (they depend only on the
 * global pixel and the frame size).  Transports:
 *   ORT_GROUP_TRANSPORT_RCCL  ncclSend/ncclRecv fused in one ncclGroupStart/End over
 *                             communicators from ncclCommInitAll (RCCL over xGMI); devices
 *                             must be distinct; RCCL is dlopen'ed (RTLD_LOCAL) on demand.
 *   ORT_GROUP_TRANSPORT_COPY  hipMemcpyPeerAsync (testing; a device may be listed twice).
 * Calls on one group are not thread-safe. */
typedef struct ort_group ort_group;
#define ORT_GROUP_MAX_DEVICES 64
#define ORT_GROUP_MAX_INFLIGHT 4
#define ORT_GROUP_TRANSPORT_RCCL 0
#define ORT_GROUP_TRANSPORT_COPY 1
/* One frame in flight (= ort_group_create_pipelined(..., 1, out)). */
int ort_group_create(const int32_t* devices, int32_t n_devices, int32_t transport, ort_group** out);
/* frames_in_flight (1..ORT_GROUP_MAX_INFLIGHT) frame slots, each with its own context per
 * device (its own scene copy, stream, band tiles and, with RCCL, communicators): frames
 * submitted in turn take the slots in turn, so frame k+1's renders fill the tail of frame k's
 * (a 1/N band tile leaves most of the GPU idle while its last blocks finish).  No reference
 * counterpart: the GL loop renders one frame at a time (src/raytracer.cpp:480-519). */
int ort_group_create_pipelined(const int32_t* devices, int32_t n_devices, int32_t transport,
                               int32_t frames_in_flight, ort_group** out);
int ort_group_destroy(ort_group* group);
/* Last error of the group (or of the calling thread when group == NULL).  Never NULL. */
const char* ort_group_last_error(const ort_group* group);
int ort_group_size(const ort_group* group);
int ort_group_frames_in_flight(const ort_group* group);
/* The context of rank `rank` in frame slot 0 (owned by the group), e.g. for ort_scene_get_info. */
int ort_group_context(ort_group* group, int32_t rank, ort_ctx** ctx);
/* ort_set_option on every context (every slot). */
int ort_group_set_option(ort_group* group, int option, int value);
/* ort_upload_scene / ort_build_scene on every context of every slot (same arguments). */
int ort_group_upload_scene(ort_group* group, const float* sphere_center_radius, const float* sphere_mat_albedo,
                           const float* sphere_fuzz_ri, int32_t n_spheres, const float* node_min,
                           const float* node_max, const int32_t* children_offset, const int32_t* objects_offset,
                           const int32_t* object_count, int32_t n_nodes, const int32_t* object_indices,
                           int64_t n_indices);
int ort_group_build_scene(ort_group* group, const float* sphere_center_radius, const float* sphere_mat_albedo,
                          const float* sphere_fuzz_ri, int32_t n_spheres, int32_t max_depth,
                          int32_t max_spheres_per_node);
/* Enqueue one full frame (width x height RGB floats, row 0 = bottom) into rgb_out -- host
 * memory (pinned for a fully asynchronous copy), or (out_is_device != 0) device memory on
 * devices[0] -- and return at once with its ticket (0, 1, 2, ...).  Every rank's render is
 * enqueued before any of them runs (no host wait inside); the only wait is for the frame that
 * last used this frame's slot, frames_in_flight frames earlier.  The bands are received (and
 * then de-interleaved) on a gather stream of devices[0], each as soon as its rank has rendered
 * it, while rank 0 may still be rendering.  rgb_out must stay untouched until
 * ort_group_wait(ticket) returns.  With the RCCL transport, frames_in_flight > 1 runs several
 * slots' communicators concurrently: not yet measured between distinct devices. */
int ort_group_submit(ort_group* group, const ort_params* params, float* rgb_out, int32_t out_is_device,
                     int64_t* ticket);
/* Wait until frame `ticket` is in rgb_out (gathered, assembled and, for host output, copied).
 * The wait is bounded (ort_group_set_timeout): when it expires the call returns
 * ORT_ERR_TIMEOUT and ort_group_last_error names the frame, its slot and every rank whose
 * render / band send had not completed (or the gather and assembly on devices[0]); the frame
 * stays submitted, so a later ort_group_wait may still see it complete. */
int ort_group_wait(ort_group* group, int64_t ticket);
/* The bound of every wait of the group on a frame (ort_group_wait, ort_group_render, and the
 * wait of ort_group_submit for the frame that last used its slot), in milliseconds: default
 * 120000; 0 = poll once (ORT_ERR_TIMEOUT unless the frame has already completed). */
int ort_group_set_timeout(ort_group* group, int64_t timeout_ms);
/* submit + wait for it and every earlier frame: synchronous. */
int ort_group_render(ort_group* group, const ort_params* params, float* rgb_out, int32_t out_is_device);
/* Device time, on devices[0], of the frame the last ort_group_wait / ort_group_render waited
 * for: from its submission on devices[0]'s stream to its assembly (renders, gather,
 * de-interleave; HIP events), taken when that frame completed -- the frame's latency, not its
 * share of a pipelined throughput.  The group keeps the times of the last 64 frames: waiting
 * for an older ticket leaves the time unknown (ORT_ERR_NO_SCENE here). */
int ort_group_last_frame_ms(ort_group* group, float* ms);

/* ---- host scene-build stage (kept reference API, src/raytracer.cpp + src/octree.cpp) -- */

/* Raytracer::generateRandomSpheres (src/raytracer.cpp:254-337) with std::mt19937(seed)
 * in place of std::random_device.  Writes n records to each SoA array (4 floats each). */
int ort_scene_random(int32_t n, uint32_t seed, float* sphere_center_radius,
                     float* sphere_mat_albedo, float* sphere_fuzz_ri);
/* Raytracer::generatePreBuiltSpheres (src/raytracer.cpp:164-252): 83 spheres.
 * Pass NULL arrays to query *n_out only. */
int ort_scene_prebuilt(float* sphere_center_radius, float* sphere_mat_albedo,
                       float* sphere_fuzz_ri, int32_t* n_out);
/* The DEBUG scene (src/raytracer.cpp:342-347): 3 spheres. */
int ort_scene_debug(float* sphere_center_radius, float* sphere_mat_albedo,
                    float* sphere_fuzz_ri, int32_t* n_out);

typedef struct ort_octree ort_octree;
/* Octree(max_depth, max_spheres_per_node).build(spheres) (src/octree.cpp:47-95). */
int ort_octree_build(const float* sphere_center_radius, int32_t n_spheres, int32_t max_depth,
                     int32_t max_spheres_per_node, ort_octree** out);
int ort_octree_sizes(const ort_octree* tree, int64_t* n_nodes, int64_t* n_indices, double* build_seconds);
/* Copy out in SoA form (any pointer may be NULL to skip that array). */
int ort_octree_export(const ort_octree* tree, float* node_min, float* node_max,
                      int32_t* children_offset, int32_t* objects_offset, int32_t* object_count,
                      int32_t* object_indices);
/* Zero-copy views: GPUOctreeNode[n_nodes] (36-byte records) and objectIndices. */
const void* ort_octree_nodes(const ort_octree* tree);
const int32_t* ort_octree_indices(const ort_octree* tree);
void ort_octree_free(ort_octree* tree);

/* Camera(position, world_up, yaw, pitch).GetViewMatrix() (src/opengl/camera.h:45-67,115-126):
 * view_out[16] column-major. */
int ort_camera_view(const float position[3], const float world_up[3], float yaw_deg, float pitch_deg,
                    float view_out[16]);

/* Library version string. */
const char* ort_version(void);

#ifdef __cplusplus
}
#endif

#endif /* ORT_H */

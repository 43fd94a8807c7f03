// group.hip -- several GPUs behind the C ABI (include/ort.h ort_group_*): the multi-GPU
// path of SURVEY.md 8(e) for a single host process, the shape a caller of
// Raytracer::render() (src/raytracer.cpp:491-499 sits where that call sits) needs to reach
// the 8-GPU configs without torch.distributed.
//
//   * one ort_ctx per listed device (scene replicated: every context builds or receives it);
//   * the frame cut into 16-row bands dealt round-robin -- rank r renders bands r, r+N, ...
//     (identical to octreeraytracer_amd/distributed.py rank_tile), every rank the same
//     number of rows, so every message has the same size;
//   * one exchange step: the bands go to devices[0] -- RCCL (ncclSend/ncclRecv fused in one
//     ncclGroupStart/End, communicators from ncclCommInitAll) or, for testing, device copies
//     (hipMemcpyPeerAsync; works with one device listed several times) -- and one
//     de-interleave kernel on devices[0] writes the frame.
// RCCL is loaded with dlopen(RTLD_LOCAL) when a group asks for it, so libort.so has no link
// dependency on it and never interposes a second librccl into a process that has its own
// (torch ships one).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <chrono>
#include <mutex>
#include <thread>
#include <new>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/ort.h"
#include "group_map.h"
#include "ort_internal.h"

#ifndef ORT_ANALYSIS
#define ORT_ANALYSIS 0
#endif

namespace {

struct Rccl {
    void* so = nullptr;
    ncclResult_t (*commInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*groupStart)() = nullptr;
    ncclResult_t (*groupEnd)() = nullptr;
    const char* (*errorString)(ncclResult_t) = nullptr;
};

// Loaded once per process (std::call_once: groups may be created from several threads);
// failures leave so == nullptr and a message.
const Rccl& rccl(std::string& err) {
    static Rccl r;
    static std::string why;
    static std::once_flag once;
    std::call_once(once, [] {
        const char* names[] = {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"};
        for (const char* n : names)
            if ((r.so = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
        if (!r.so) {
            why = std::string("RCCL not loadable: ") + dlerror();
            return;
        }
        bool ok = true;
        auto sym = [&](auto& f, const char* name) {
            f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(r.so, name));
            ok = ok && f;
        };
        sym(r.commInitAll, "ncclCommInitAll");
        sym(r.commDestroy, "ncclCommDestroy");
        sym(r.send, "ncclSend");
        sym(r.recv, "ncclRecv");
        sym(r.groupStart, "ncclGroupStart");
        sym(r.groupEnd, "ncclGroupEnd");
        sym(r.errorString, "ncclGetErrorString");
        if (!ok) {
            why = "RCCL lacks a needed symbol";
            r.so = nullptr;
        }
    });
    err = why;
    return r;
}

// de-interleave: frame row y <- row group_src_row(y) of its rank's band tile
struct SrcTable {
    const float* tile[ORT_GROUP_MAX_DEVICES];
};
__global__ void __launch_bounds__(256) k_assemble(SrcTable src, int world, int width, int height, float* out) {
    const int y = blockIdx.x;
    if (y >= height) return;
    int rank, trow;
    ort::group_src_row(y, world, rank, trow);
    const size_t n = 3 * (size_t)width;
    const float* s = src.tile[rank] + (size_t)trow * n;
    float* d = out + (size_t)y * n;
    for (size_t i = threadIdx.x; i < n; i += blockDim.x) d[i] = s[i];
}

}  // namespace

// One frame slot: a context per rank (its own scene copy and stream), the band tiles, the
// gather buffers and the events of one frame in flight.  A group holds `inflight` slots and
// takes frames in turn on them, so frame k+1's renders fill the tail of frame k's.
struct GroupSlot {
    std::vector<ort_ctx*> ctx;
    std::vector<hipStream_t> stream;   // each context's own stream
    std::vector<ncclComm_t> comm;      // RCCL: this slot's communicators (one gather at a time each)
    std::vector<float*> tile;          // per rank, on its device: rows x W x 3
    std::vector<float*> recv;          // on devices[0]: the band tiles of ranks 1..n-1
    size_t tile_floats = 0;
    float* frame = nullptr;            // devices[0]: the assembled frame (host output path)
    size_t frame_floats = 0;
    std::vector<hipEvent_t> done;      // per rank: its tile has been copied (copy transport)
    // devices[0]: the gather's stream -- the receives (RCCL) or the waits for the copies, then
    // the de-interleave -- so that the bands of ranks 1..N-1 land while rank 0 still renders
    // (posted behind rank 0's render on stream[0], no band was received before it finished)
    hipStream_t gstream = nullptr;
    hipEvent_t rendered0 = nullptr;    // devices[0]: rank 0's band tile is rendered
    hipEvent_t assembled = nullptr;    // devices[0]: the de-interleave has read recv[]
    hipEvent_t finished = nullptr;     // devices[0]: the frame (and its host copy) is complete
    hipEvent_t t0 = nullptr, t1 = nullptr;
    long long ticket = -1;             // the frame last submitted on this slot
    bool assembled_once = false;
};

struct ort_group {
    int n = 0;
    int transport = ORT_GROUP_TRANSPORT_RCCL;
    std::vector<int> dev;
    std::vector<GroupSlot> slot;
    long long next_ticket = 0;
    // device time of each completed frame, taken when its slot's completion is first seen
    // (wait_slot: by ort_group_wait, or by the submit that reuses the slot) -- a later
    // submission on that slot cannot overwrite it
    static constexpr int kMsRing = 64;
    long long ms_ticket[kMsRing];
    float ms_value[kMsRing];
    float last_ms = -1.0f;             // of the frame ort_group_wait / ort_group_render saw complete last
    long long timeout_ms = 120000;     // every wait on a frame (ort_group_set_timeout)
    std::string err;
    ort_group() {
        for (int i = 0; i < kMsRing; ++i) ms_ticket[i] = -1;
    }
};

namespace {

int gfail(ort_group* g, int code, const std::string& msg) {
    if (g) g->err = msg;
    ort::set_thread_error(msg);
    return code;
}

#define GCHK(g, expr)                                                                             \
    do {                                                                                          \
        hipError_t _e = (expr);                                                                   \
        if (_e != hipSuccess)                                                                     \
            return gfail(g, _e == hipErrorOutOfMemory ? ORT_ERR_OUT_OF_MEMORY : ORT_ERR_HIP,      \
                         std::string(#expr) + ": " + hipGetErrorString(_e));                      \
    } while (0)

int each(ort_group* g, ort_ctx* c, int rc, int r) {
    if (rc != ORT_OK) return gfail(g, rc, "device " + std::to_string(g->dev[r]) + ": " + ort_last_error(c));
    return ORT_OK;
}

void free_buffers(ort_group* g, GroupSlot& S) {
    for (int r = 0; r < (int)S.tile.size(); ++r)
        if (S.tile[r]) {
            (void)hipSetDevice(g->dev[r]);
            (void)hipFree(S.tile[r]);
        }
    S.tile.assign(g->n, nullptr);
    (void)hipSetDevice(g->dev.empty() ? 0 : g->dev[0]);
    for (float* p : S.recv)
        if (p) (void)hipFree(p);
    S.recv.assign(g->n, nullptr);
    if (S.frame) (void)hipFree(S.frame);
    S.frame = nullptr;
    S.tile_floats = 0;
    S.frame_floats = 0;
}

// (Re)allocates a slot's buffers; the slot's previous frame is complete (ort_group_submit).
int ensure_buffers(ort_group* g, GroupSlot& S, size_t tile_floats, size_t frame_floats) {
    if (tile_floats > S.tile_floats) {
        free_buffers(g, S);
        for (int r = 0; r < g->n; ++r) {
            GCHK(g, hipSetDevice(g->dev[r]));
            GCHK(g, hipMalloc(&S.tile[r], tile_floats * sizeof(float)));
        }
        GCHK(g, hipSetDevice(g->dev[0]));
        for (int r = 1; r < g->n; ++r) GCHK(g, hipMalloc(&S.recv[r], tile_floats * sizeof(float)));
        S.tile_floats = tile_floats;
    }
    if (frame_floats > S.frame_floats) {
        GCHK(g, hipSetDevice(g->dev[0]));
        if (S.frame) (void)hipFree(S.frame);
        S.frame = nullptr;
        GCHK(g, hipMalloc(&S.frame, frame_floats * sizeof(float)));
        S.frame_floats = frame_floats;
    }
    return ORT_OK;
}

// Every context of every slot.
template <class F>
int for_each_ctx(ort_group* g, F f) {
    for (GroupSlot& S : g->slot)
        for (int r = 0; r < g->n; ++r) {
            const int rc = each(g, S.ctx[r], f(S.ctx[r]), r);
            if (rc) return rc;
        }
    return ORT_OK;
}

// hipSuccess when the event has completed, hipErrorNotReady while pending, else an error.
hipError_t query(int device, hipEvent_t e) {
    const hipError_t d = hipSetDevice(device);
    return d != hipSuccess ? d : hipEventQuery(e);
}

// The slot's frame: wait (bounded by g->timeout_ms) until it has completed.  On expiry the
// error names what is still pending: each rank whose render / band send has not completed
// (its `done` event, recorded after them on its stream) and the gather + assembly on
// devices[0] -- so a first multi-GPU run that stalls says where instead of hanging.
int wait_slot(ort_group* g, GroupSlot& S) {
    if (S.ticket < 0) return ORT_OK;
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t e = query(g->dev[0], S.finished);
        if (e == hipSuccess) break;
        if (e != hipErrorNotReady) GCHK(g, e);
        const long long ms =
            std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
        if (ms >= g->timeout_ms) {
            std::string pend;
            for (int r = 0; r < g->n; ++r) {
                const hipError_t q = S.done[r] ? query(g->dev[r], S.done[r]) : hipSuccess;
                if (q == hipErrorNotReady)
                    pend += (pend.empty() ? "" : ", ") + std::string("rank ") + std::to_string(r) + " (device " +
                            std::to_string(g->dev[r]) + ": render" + (r > 0 && g->n > 1 ? " / band send)" : ")");
            }
            if (pend.empty()) pend = "the gather / assembly on device " + std::to_string(g->dev[0]);
            (void)hipSetDevice(g->dev[0]);
            return gfail(g, ORT_ERR_TIMEOUT, "ort_group: frame " + std::to_string(S.ticket) + " (slot " +
                                                 std::to_string((long long)(S.ticket % (long long)g->slot.size())) +
                                                 ") not complete after " + std::to_string(ms) + " ms; pending: " + pend);
        }
        // poll: yield (no sleep) for twice the last frame's device time, at least 5 ms and at most
        // 250 ms -- a synchronous render is then seen complete within a yield of its end -- and
        // only past that window sleep, 50 us steps then 1 ms steps (a frame takes 0.2-50 ms)
        const float lf = g->last_ms > 0.0f ? g->last_ms : 0.0f;
        const long long busy_us = std::min(250000LL, std::max(5000LL, (long long)(2000.0f * lf)));
        const long long us =
            std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count();
        if (us < busy_us) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(us < busy_us + 50000 ? 50 : 1000));
    }
    GCHK(g, hipSetDevice(g->dev[0]));
    const int i = (int)(S.ticket % ort_group::kMsRing);
    if (g->ms_ticket[i] != S.ticket) {  // first time this frame is seen complete: keep its time
        float ms = 0.0f;
        GCHK(g, hipEventElapsedTime(&ms, S.t0, S.t1));
        g->ms_ticket[i] = S.ticket;
        g->ms_value[i] = ms;
    }
    return ORT_OK;
}

}  // namespace

extern "C" {

int ort_group_create_pipelined(const int32_t* devices, int32_t n_devices, int32_t transport, int32_t frames_in_flight,
                               ort_group** out) {
    if (!out || !devices || n_devices < 1 || n_devices > ORT_GROUP_MAX_DEVICES)
        return gfail(nullptr, ORT_ERR_INVALID_ARG, "ort_group_create: need 1.." + std::to_string(ORT_GROUP_MAX_DEVICES) +
                                                       " devices and an out pointer");
    if (transport != ORT_GROUP_TRANSPORT_RCCL && transport != ORT_GROUP_TRANSPORT_COPY)
        return gfail(nullptr, ORT_ERR_INVALID_ARG, "ort_group_create: unknown transport");
    if (frames_in_flight < 1 || frames_in_flight > ORT_GROUP_MAX_INFLIGHT)
        return gfail(nullptr, ORT_ERR_INVALID_ARG, "ort_group_create: frames in flight must be 1.." +
                                                       std::to_string(ORT_GROUP_MAX_INFLIGHT));
    *out = nullptr;
    if (transport == ORT_GROUP_TRANSPORT_RCCL)
        for (int i = 0; i < n_devices; ++i)
            for (int j = 0; j < i; ++j)
                if (devices[i] == devices[j])
                    return gfail(nullptr, ORT_ERR_INVALID_ARG,
                                 "ort_group_create: RCCL needs distinct devices (ORT_GROUP_TRANSPORT_COPY allows repeats)");
    ort_group* g = new (std::nothrow) ort_group();
    if (!g) return gfail(nullptr, ORT_ERR_OUT_OF_MEMORY, "ort_group_create: out of host memory");
    g->n = n_devices;
    g->transport = transport;
    g->dev.assign(devices, devices + n_devices);
    g->slot.resize(frames_in_flight);
    for (GroupSlot& S : g->slot) {
        S.ctx.assign(n_devices, nullptr);
        S.stream.assign(n_devices, nullptr);
        S.tile.assign(n_devices, nullptr);
        S.recv.assign(n_devices, nullptr);
        S.done.assign(n_devices, nullptr);
    }
    auto bail = [&](int rc) {
        const std::string m = g->err.empty() ? std::string(ort_last_error(nullptr)) : g->err;
        ort_group_destroy(g);
        ort::set_thread_error(m);
        return rc;
    };
    for (GroupSlot& S : g->slot) {
        for (int r = 0; r < n_devices; ++r) {
            int rc = ort_create(devices[r], &S.ctx[r]);
            if (rc != ORT_OK) return bail(rc);
            // ranks sharing a device, or frames in flight, fill each frame's tail themselves: no
            // split walks there (ORT_OPT_SPLIT_HEAVY's second stream only adds launches: C3 1/8 band
            // at 3 in flight -15 %; ort_group_set_option overrides)
            bool shared = frames_in_flight > 1;
            for (int q = 0; q < n_devices && !shared; ++q) shared = q != r && devices[q] == devices[r];
            if (shared) (void)ort_set_option(S.ctx[r], ORT_OPT_SPLIT_HEAVY, 0);
            void* s = nullptr;
            ort_get_stream(S.ctx[r], &s);
            S.stream[r] = (hipStream_t)s;
            if (hipSetDevice(devices[r]) != hipSuccess ||
                hipEventCreateWithFlags(&S.done[r], hipEventDisableTiming) != hipSuccess)
                return bail(gfail(g, ORT_ERR_HIP, "ort_group_create: events"));
        }
        if (hipSetDevice(devices[0]) != hipSuccess || hipEventCreate(&S.t0) != hipSuccess ||
            hipEventCreate(&S.t1) != hipSuccess ||
            hipStreamCreateWithFlags(&S.gstream, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&S.rendered0, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&S.assembled, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&S.finished, hipEventDisableTiming) != hipSuccess)
            return bail(gfail(g, ORT_ERR_HIP, "ort_group_create: timing events"));
        if (transport == ORT_GROUP_TRANSPORT_RCCL) {
            std::string why;
            const Rccl& R = rccl(why);
            if (!R.so) return bail(gfail(g, ORT_ERR_UNSUPPORTED, "ort_group_create: " + why));
            S.comm.assign(n_devices, nullptr);
            const ncclResult_t e = R.commInitAll(S.comm.data(), n_devices, g->dev.data());
            if (e != ncclSuccess) {
                S.comm.clear();
                return bail(gfail(g, ORT_ERR_HIP, std::string("ncclCommInitAll: ") + R.errorString(e)));
            }
        }
    }
    *out = g;
    return ORT_OK;
}

int ort_group_create(const int32_t* devices, int32_t n_devices, int32_t transport, ort_group** out) {
    return ort_group_create_pipelined(devices, n_devices, transport, 1, out);
}

int ort_group_destroy(ort_group* g) {
    if (!g) return ORT_OK;
    for (GroupSlot& S : g->slot) {
        for (int r = 0; r < g->n; ++r)
            if (S.ctx[r]) {
                (void)hipSetDevice(g->dev[r]);
                (void)hipStreamSynchronize(S.stream[r]);
            }
        if (S.gstream) {
            (void)hipSetDevice(g->dev[0]);
            (void)hipStreamSynchronize(S.gstream);
        }
    }
    for (GroupSlot& S : g->slot) {
        if (!S.comm.empty()) {
            std::string why;
            const Rccl& R = rccl(why);
            for (ncclComm_t c : S.comm)
                if (c && R.so) (void)R.commDestroy(c);
        }
        free_buffers(g, S);
        for (int r = 0; r < g->n; ++r) {
            if (S.done[r]) {
                (void)hipSetDevice(g->dev[r]);
                (void)hipEventDestroy(S.done[r]);
            }
            if (S.ctx[r]) ort_destroy(S.ctx[r]);
        }
        if (!g->dev.empty()) (void)hipSetDevice(g->dev[0]);
        for (hipEvent_t e : {S.t0, S.t1, S.rendered0, S.assembled, S.finished})
            if (e) (void)hipEventDestroy(e);
        if (S.gstream) (void)hipStreamDestroy(S.gstream);
    }
    delete g;
    return ORT_OK;
}

const char* ort_group_last_error(const ort_group* g) { return g ? g->err.c_str() : ort::thread_error(); }

int ort_group_size(const ort_group* g) { return g ? g->n : 0; }

int ort_group_frames_in_flight(const ort_group* g) { return g ? (int)g->slot.size() : 0; }

int ort_group_context(ort_group* g, int32_t rank, ort_ctx** ctx) {
    if (!g || !ctx || rank < 0 || rank >= g->n) return gfail(g, ORT_ERR_INVALID_ARG, "ort_group_context: bad rank");
    *ctx = g->slot[0].ctx[rank];
    return ORT_OK;
}

int ort_group_set_option(ort_group* g, int option, int value) {
    if (!g) return gfail(nullptr, ORT_ERR_INVALID_ARG, "ort_group_set_option: null group");
    return for_each_ctx(g, [&](ort_ctx* c) { return ort_set_option(c, option, value); });
}

int ort_group_upload_scene(ort_group* g, const float* cr, const float* ma, const float* fr, int32_t n_spheres,
                           const float* node_min, const float* node_max, const int32_t* children_offset,
                           const int32_t* objects_offset, const int32_t* object_count, int32_t n_nodes,
                           const int32_t* object_indices, int64_t n_indices) {
    if (!g) return gfail(nullptr, ORT_ERR_INVALID_ARG, "ort_group_upload_scene: null group");
    return for_each_ctx(g, [&](ort_ctx* c) {
        return ort_upload_scene(c, cr, ma, fr, n_spheres, node_min, node_max, children_offset, objects_offset,
                                object_count, n_nodes, object_indices, n_indices);
    });
}

int ort_group_build_scene(ort_group* g, const float* cr, const float* ma, const float* fr, int32_t n_spheres,
                          int32_t max_depth, int32_t max_spheres_per_node) {
    if (!g) return gfail(nullptr, ORT_ERR_INVALID_ARG, "ort_group_build_scene: null group");
    return for_each_ctx(g, [&](ort_ctx* c) {
        return ort_build_scene(c, cr, ma, fr, n_spheres, max_depth, max_spheres_per_node, 0);
    });
}

int ort_group_submit(ort_group* g, const ort_params* p, float* rgb_out, int32_t out_is_device, int64_t* ticket) {
    if (!g || !p) return gfail(g, ORT_ERR_INVALID_ARG, "ort_group_submit: null argument");
    if (!rgb_out) return gfail(g, ORT_ERR_INVALID_ARG, "ort_group_submit: null output");
    if (p->width <= 0 || p->height <= 0) return gfail(g, ORT_ERR_INVALID_ARG, "ort_group_submit: width/height must be positive");
    const int W = p->width, H = p->height, N = g->n;
    const long long tk = g->next_ticket;
    GroupSlot& S = g->slot[(size_t)(tk % (long long)g->slot.size())];
    int rc;
    // the slot's previous frame must be complete before its buffers are reused
    if ((rc = wait_slot(g, S))) return rc;
    const ort_tile t0 = ort::group_tile(W, H, 0, N);
    const size_t tile_floats = (size_t)t0.rows * W * 3, frame_floats = (size_t)H * W * 3;
    if ((rc = ensure_buffers(g, S, tile_floats, out_is_device ? 0 : frame_floats))) return rc;
    GCHK(g, hipSetDevice(g->dev[0]));
    GCHK(g, hipEventRecord(S.t0, S.stream[0]));
    // 1. every rank renders its bands on its own stream: ort_render with a stream never waits
    //    on the host (also for multi-bounce frames), so every rank is enqueued before any runs
    for (int r = 0; r < N; ++r) {
        const ort_tile t = ort::group_tile(W, H, r, N);
        if ((rc = each(g, S.ctx[r], ort_render(S.ctx[r], p, &t, S.tile[r], 1, S.stream[r]), r))) return rc;
    }
    GCHK(g, hipSetDevice(g->dev[0]));
    GCHK(g, hipEventRecord(S.rendered0, S.stream[0]));
    GCHK(g, hipEventRecord(S.done[0], S.stream[0]));
    // 2. the one exchange: bands of ranks 1..N-1 to devices[0], received on the gather stream
    //    (each band as soon as its rank is done, also while rank 0 still renders); the slot's
    //    previous assembly ran on that stream too, so recv[] is free when they land
    if (N > 1) {
        if (g->transport == ORT_GROUP_TRANSPORT_RCCL) {
            std::string why;
            const Rccl& R = rccl(why);
            ncclResult_t e = R.groupStart();
            for (int r = 1; r < N && e == ncclSuccess; ++r) {
                e = R.send(S.tile[r], tile_floats, ncclFloat32, 0, S.comm[r], S.stream[r]);
                if (e == ncclSuccess) e = R.recv(S.recv[r], tile_floats, ncclFloat32, r, S.comm[0], S.gstream);
            }
            const ncclResult_t e2 = R.groupEnd();
            if (e != ncclSuccess || e2 != ncclSuccess)
                return gfail(g, ORT_ERR_HIP, std::string("RCCL gather: ") + R.errorString(e != ncclSuccess ? e : e2));
            for (int r = 1; r < N; ++r) {  // each rank's render + send done (a bounded wait names the laggard)
                GCHK(g, hipSetDevice(g->dev[r]));
                GCHK(g, hipEventRecord(S.done[r], S.stream[r]));
            }
        } else {
            for (int r = 1; r < N; ++r) {
                GCHK(g, hipSetDevice(g->dev[r]));
                // recv[r] is free once this slot's previous assembly has read it
                if (S.assembled_once) GCHK(g, hipStreamWaitEvent(S.stream[r], S.assembled, 0));
                GCHK(g, hipMemcpyPeerAsync(S.recv[r], g->dev[0], S.tile[r], g->dev[r], tile_floats * sizeof(float),
                                           S.stream[r]));
                GCHK(g, hipEventRecord(S.done[r], S.stream[r]));
                GCHK(g, hipSetDevice(g->dev[0]));
                GCHK(g, hipStreamWaitEvent(S.gstream, S.done[r], 0));
            }
        }
    }
    // 3. de-interleave on devices[0], once rank 0's own tile is rendered too
    GCHK(g, hipSetDevice(g->dev[0]));
    GCHK(g, hipStreamWaitEvent(S.gstream, S.rendered0, 0));
    SrcTable src{};
    src.tile[0] = S.tile[0];
    for (int r = 1; r < N; ++r) src.tile[r] = S.recv[r];
    float* dst = out_is_device ? rgb_out : S.frame;
    hipLaunchKernelGGL(k_assemble, dim3((unsigned)H), dim3(256), 0, S.gstream, src, N, W, H, dst);
    GCHK(g, hipGetLastError());
    GCHK(g, hipEventRecord(S.assembled, S.gstream));
    S.assembled_once = true;
    GCHK(g, hipEventRecord(S.t1, S.gstream));
    if (!out_is_device)  // pageable rgb_out: the runtime may stage this copy synchronously
        GCHK(g, hipMemcpyAsync(rgb_out, S.frame, frame_floats * sizeof(float), hipMemcpyDeviceToHost, S.gstream));
    GCHK(g, hipEventRecord(S.finished, S.gstream));
    S.ticket = tk;
    g->next_ticket = tk + 1;
    if (ticket) *ticket = tk;
    return ORT_OK;
}

int ort_group_wait(ort_group* g, int64_t ticket) {
    if (!g) return gfail(nullptr, ORT_ERR_INVALID_ARG, "ort_group_wait: null group");
    if (ticket < 0 || ticket >= g->next_ticket) return gfail(g, ORT_ERR_INVALID_ARG, "ort_group_wait: no such frame");
    const int si = (int)(ticket % (long long)g->slot.size());
    GroupSlot& S = g->slot[(size_t)si];
    if (S.ticket == ticket) {  // else the slot took a later frame, so this one has completed
        const int rc = wait_slot(g, S);
        if (rc) return rc;
    }
    const int i = (int)(ticket % ort_group::kMsRing);
    // the ring keeps the last kMsRing frames' times: an older ticket's is gone
    g->last_ms = g->ms_ticket[i] == ticket ? g->ms_value[i] : -1.0f;
    return ORT_OK;
}

int ort_group_set_timeout(ort_group* g, int64_t timeout_ms) {
    if (!g || timeout_ms < 0) return gfail(g, ORT_ERR_INVALID_ARG, "ort_group_set_timeout: null group or negative bound");
    g->timeout_ms = timeout_ms;
    return ORT_OK;
}

int ort_group_render(ort_group* g, const ort_params* p, float* rgb_out, int32_t out_is_device) {
    int64_t tk = -1;
    int rc = ort_group_submit(g, p, rgb_out, out_is_device, &tk);
    if (rc) return rc;
    // synchronous, like ort_render without a stream: every earlier frame has completed too
    for (GroupSlot& S : g->slot)
        if ((rc = wait_slot(g, S))) return rc;
    return ort_group_wait(g, tk);
}

int ort_group_last_frame_ms(ort_group* g, float* ms) {
    if (!g || !ms) return gfail(g, ORT_ERR_INVALID_ARG, "ort_group_last_frame_ms: null argument");
    if (g->last_ms < 0.0f)
        return gfail(g, ORT_ERR_NO_SCENE, "no frame time: none completed yet, or the last ticket waited for is more "
                                          "than 64 frames old (ort_group_wait)");
    *ms = g->last_ms;  // taken when that frame completed (wait_slot): later submissions do not move it
    return ORT_OK;
}

#if ORT_ANALYSIS  // the analysis library only (libort_analysis.so)
// TEST-ONLY (no GPU): the group's partition and assembly with an in-memory transport -- every
// rank's band tile rendered by the host emulation of the kernel (ort_debug_emulate_render),
// one after another, then assembled by the same row map the device kernel uses.
int ort_debug_group_emulate(const float* cr, const float* ma, const float* fr, int32_t n_spheres, const float* node_min,
                            const float* node_max, const int32_t* co, const int32_t* oo, const int32_t* cnt,
                            int32_t n_nodes, const int32_t* idx, int64_t n_indices, int32_t world,
                            const ort_params* p, float* rgb_out) {
    if (!p || !rgb_out || world < 1 || world > ORT_GROUP_MAX_DEVICES)
        return gfail(nullptr, ORT_ERR_INVALID_ARG, "ort_debug_group_emulate: bad arguments");
    const int W = p->width, H = p->height;
    const ort_tile t0 = ort::group_tile(W, H, 0, world);
    std::vector<std::vector<float>> tiles(world, std::vector<float>((size_t)t0.rows * W * 3));
    for (int r = 0; r < world; ++r) {
        const ort_tile t = ort::group_tile(W, H, r, world);
        const int rc = ort_debug_emulate_render(cr, ma, fr, n_spheres, node_min, node_max, co, oo, cnt, n_nodes, idx,
                                                n_indices, ORT_LAYOUT_COMPACT, p, &t, tiles[r].data(), nullptr);
        if (rc != ORT_OK) return rc;
    }
    for (int y = 0; y < H; ++y) {
        int rank, trow;
        ort::group_src_row(y, world, rank, trow);
        std::memcpy(rgb_out + (size_t)y * W * 3, tiles[rank].data() + (size_t)trow * W * 3, (size_t)W * 3 * sizeof(float));
    }
    return ORT_OK;
}

#endif  // ORT_ANALYSIS

}  // extern "C"

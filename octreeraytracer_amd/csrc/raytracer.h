// raytracer.h -- the reference's Raytracer class (src/raytracer.h:13-60) on the MI355X
// kernel instead of OpenGL.
//
// Kept: Raytracer(), ~Raytracer(), initialize(), run(), and the private stages
// setupScene / setupBuffers / cleanupBuffers / generateSpheres / generatePreBuiltSpheres /
// generateRandomSpheres / saveStats with the reference's semantics and CSV schema.
// New: render() -- one frame into a caller buffer (the reference has no readback,
// SURVEY.md F3/F4) -- and RaytracerConfig, the runtime form of src/config.h.
// No window: initialize() creates the device context (the reference's GLFW/GLAD/shader
// setup, src/raytracer.cpp:32-60); run() renders warm-up + timed frames headless.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/ort.h"
#include "camera.h"
#include "octree.h"
#include "sphere.h"

// src/config.h as a runtime struct; defaults equal the reference's constants.
struct RaytracerConfig {
    int debug = 0;                 // DEBUG
    int useOctree = 1;             // USEOCTREE
    int usePrebuilt = 0;           // USEPREBUILT
    int numSpheres = 100;          // NUMSPHERES
    int maxDepth = 3;              // MAXDEPTH
    int debugDepth = 3;            // DEBUGDEPTH
    int maxSpheresPerNode = 0;     // MAXSPHERESPERNODE
    int debugSpheresPerNode = 2;   // DEBUGSPHERESPERNODE
    int numSamples = 16;           // NUMSAMPLES
    int maxRaysDepth = 8;          // MAXRAYSDEPTH
    unsigned width = 800;          // SCR_WIDTH
    unsigned height = 600;         // SCR_HEIGHT
    bool collectStats = false;     // COLLECTSTATS
    std::string outputFile = "stats.csv";  // OUTPUTFILE
    // new knobs
    uint32_t seed = 42;            // replaces std::random_device in generateRandomSpheres
    int device = 0;                // HIP device of the context
    std::vector<int> devices;      // several GPUs: an ort_group over these (bands dealt round-robin,
                                   // RCCL gather to devices[0]; a device listed twice
                                   // gathers by device copies instead); empty = `device` only
    int frames = 50;               // frames of run() (the reference stops after 50 with stats)
    int warmupFrames = 15;         // src/raytracer.cpp:455
    bool gpuBuild = false;         // build the octree on the GPU (ort_build_scene, same tree) instead
                                   // of Octree::build on the host; getOctree() then stays empty
    bool extendedStats = false;    // saveStats appends 5 throughput columns to the reference's 15
                                   // (see StatsWork / Raytracer::statsRow)
    bool readback = false;         // run(): copy every frame to host memory; default off: the frames
                                   // stay in a device buffer, as the reference's stay in its GL
                                   // framebuffer (src/raytracer.cpp:476-519 never reads them back)
};

// Work of one frame for the extended stats columns: ort_count_traffic over the full frame
// (reference-layout counters), plus the device and host-core counts.
struct StatsWork {
    uint64_t traversals = 0;       // octree walks per frame (all samples and bounces)
    double algorithmicBytes = 0;   // 36/node popped + 32/child record + 20/leaf object + 32/hit + 12/pixel
    int gpus = 1;
    int hostCores = 1;
};

class Raytracer {
public:
    Raytracer();
    explicit Raytracer(const RaytracerConfig& cfg);
    ~Raytracer();
    Raytracer(const Raytracer&) = delete;
    Raytracer& operator=(const Raytracer&) = delete;

    bool initialize();
    void run();

    // One full frame of the current scene seen from `cam` into rgb (width*height*3
    // floats, row 0 = bottom row, as the GL framebuffer).  Builds and uploads the scene on
    // first use.  Returns ORT_OK or an ORT_ERR_* code (message: lastError()).
    int render(const Camera& cam, float* rgb);
    // A tile (see ort_tile in include/ort.h) into host or device memory, optionally
    // stream-ordered on a caller hipStream_t.  Single-device configurations only (a group
    // renders whole frames: ORT_ERR_UNSUPPORTED).
    int render(const Camera& cam, const ort_tile& tile, float* out, bool outIsDevice, void* stream);

    Camera camera;  // the reference keeps a global Camera (src/main.cpp:18); pose set like main()
    const RaytracerConfig& config() const { return cfg; }
    const std::vector<Sphere>& getSpheres() const { return spheres; }
    const Octree& getOctree() const { return octree; }
    const std::vector<double>& getRenderTimes() const { return renderTimes; }
    const char* lastError() const;

    // The saveStats row for these frame times (seconds), without the newline: the reference's
    // 15 ';'-separated columns (src/raytracer.cpp:441-446: useOctree, numSpheres, maxDepth,
    // maxSpheresPerNode, numSamples, maxRaysDepth, width, height, min, max, avg, minFPS,
    // maxFPS, fpsAvg, buildTime) after its 2.5-sigma z-score filter (:372-434), then, when
    // `work` is given, mrays_per_s (traversals / avg frame time), bytes_per_ray (algorithmic
    // reference-layout bytes / traversal), ref_layout_bytes_frac (mrays_per_s x bytes_per_ray /
    // 8 TB/s: the bytes the REFERENCE's record layout would move at this ray rate, SURVEY.md
    // 8(d)'s algorithmic figure -- not a roofline: it exceeds 1 because the compact layout never
    // reads the reference's child records; bench.py reports the measured VALU-issue roofline),
    // gpus, host_cores.  buildSeconds: Octree::buildTime, the root box + subdivision like the
    // reference's column (its flatten excluded), or with gpuBuild the GPU builder's device time
    // (one pass, the layout included: there is no separate flatten to leave out).
    // Returns "" for no frames.
    static std::string statsRow(const RaytracerConfig& cfg, const std::vector<double>& frameSeconds,
                                double buildSeconds, const StatsWork* work);

private:
    RaytracerConfig cfg;
    int width, height;
    ort_ctx* ctx;
    ort_group* group = nullptr;    // cfg.devices.size() > 1
    bool sceneReady;
    std::vector<Sphere> spheres;
    Octree octree;
    std::string statsFilename;
    int frameCount;
    std::vector<double> renderTimes;
    std::vector<float> frame;
    float* dframe = nullptr;       // run()'s device frame (readback off), on the context's device
    int renderRun();               // one frame of run(): into dframe, or into `frame` with readback
    double gpuBuildSeconds = 0.0;
    StatsWork work;               // counted after the timed frames when cfg.extendedStats

    void setupScene();
    void setupBuffers();
    void cleanupBuffers();
    std::vector<Sphere> generateSpheres();
    std::vector<Sphere> generatePreBuiltSpheres();
    std::vector<Sphere> generateRandomSpheres();
    void saveStats();
    bool countWork();
    ort_params frameParams(const Camera& cam) const;
};

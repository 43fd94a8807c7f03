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
    double gpuBuildSeconds = 0.0;

    void setupScene();
    void setupBuffers();
    void cleanupBuffers();
    std::vector<Sphere> generateSpheres();
    std::vector<Sphere> generatePreBuiltSpheres();
    std::vector<Sphere> generateRandomSpheres();
    void saveStats();
    ort_params frameParams(const Camera& cam) const;
};

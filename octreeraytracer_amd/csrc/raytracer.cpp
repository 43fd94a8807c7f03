// raytracer.cpp -- Raytracer on the gfx950 kernel (see raytracer.h).
#include "raytracer.h"

#include <chrono>
#include <cmath>
#include <fstream>
#include <iostream>
#include <sstream>

#include <sched.h>

#include <hip/hip_runtime_api.h>

#include "scene.h"

Raytracer::Raytracer() : Raytracer(RaytracerConfig()) {}

Raytracer::Raytracer(const RaytracerConfig& c)
    : camera(ortm::vec3(0.0f, 8.0f, 30.0f)),
      cfg(c),
      width((int)c.width),
      height((int)c.height),
      ctx(nullptr),
      sceneReady(false),
      octree(c.debug ? c.debugDepth : c.maxDepth, c.debug ? c.debugSpheresPerNode : c.maxSpheresPerNode),
      statsFilename(c.outputFile),
      frameCount(0) {
    // camera pose of main() (src/main.cpp:29-40)
    if (cfg.debug) camera.Position = ortm::vec3(30.0f, 20.0f, -50.0f);
    else camera.Position = ortm::vec3(0.0f, 2.5f, -10.0f);
    camera.updateCameraVectors();
}

Raytracer::~Raytracer() { cleanupBuffers(); }

bool Raytracer::initialize() {
    if (ctx || group) return true;
    if (cfg.devices.size() > 1) {  // several GPUs: one context each inside an ort_group
        // RCCL over distinct devices; a device listed twice (testing on one GPU) gathers by copies
        bool distinct = true;
        for (size_t i = 0; i < cfg.devices.size(); ++i)
            for (size_t j = 0; j < i; ++j) distinct = distinct && cfg.devices[i] != cfg.devices[j];
        const int32_t transport = distinct ? ORT_GROUP_TRANSPORT_RCCL : ORT_GROUP_TRANSPORT_COPY;
        if (ort_group_create(cfg.devices.data(), (int32_t)cfg.devices.size(), transport, &group) != ORT_OK) {
            std::cerr << "Failed to create the MI355X device group: " << ort_group_last_error(nullptr) << std::endl;
            group = nullptr;
            return false;
        }
        return true;
    }
    if (ort_create(cfg.device, &ctx) != ORT_OK) {
        std::cerr << "Failed to create the MI355X context: " << ort_last_error(nullptr) << std::endl;
        ctx = nullptr;
        return false;
    }
    return true;
}

const char* Raytracer::lastError() const { return group ? ort_group_last_error(group) : ort_last_error(ctx); }

std::vector<Sphere> Raytracer::generatePreBuiltSpheres() { return ort::generatePreBuiltSpheres(); }
std::vector<Sphere> Raytracer::generateRandomSpheres() { return ort::generateRandomSpheres(cfg.numSpheres, cfg.seed); }

std::vector<Sphere> Raytracer::generateSpheres() {
    if (cfg.debug) return ort::generateDebugSpheres();
    if (cfg.usePrebuilt) return generatePreBuiltSpheres();
    return generateRandomSpheres();
}

void Raytracer::setupScene() {
    spheres = generateSpheres();
    const int maxDepth = cfg.debug ? cfg.debugDepth : cfg.maxDepth;
    const int maxSpheresPerNode = cfg.debug ? cfg.debugSpheresPerNode : cfg.maxSpheresPerNode;
    octree = Octree(maxDepth, maxSpheresPerNode);
    if (cfg.gpuBuild && !cfg.debug) return;  // setupBuffers builds it on the device
    octree.build(spheres, cfg.debug);
    if (cfg.debug) octree.printFlattenedTree();
}

void Raytracer::setupBuffers() {
    // SoA packing of src/raytracer.cpp:87-101, then one upload (replaces 7x glBufferData)
    std::vector<float> cr(4 * spheres.size()), ma(4 * spheres.size()), fr(4 * spheres.size());
    ort::packSpheres(spheres, cr.data(), ma.data(), fr.data());
    int rc = ORT_OK;
    const int ranks = group ? ort_group_size(group) : 1;
    for (int r = 0; r < ranks && rc == ORT_OK; ++r) {  // every device holds the whole scene
        ort_ctx* c = ctx;
        if (group) ort_group_context(group, r, &c);
        if (cfg.gpuBuild && !cfg.debug) {
            rc = ort_build_scene(c, cr.data(), ma.data(), fr.data(), (int32_t)spheres.size(), octree.getMaxDepth(),
                                 octree.getMaxSpheresPerNode(), 0);
            float ms = 0.0f;
            if (rc == ORT_OK) ort_last_build_ms(c, &ms);
            gpuBuildSeconds = ms * 1e-3;
        } else {
            rc = ort_upload_octree_nodes(c, cr.data(), ma.data(), fr.data(), (int32_t)spheres.size(),
                                         octree.flattenedTree.data(), (int32_t)octree.flattenedTree.size(),
                                         octree.objectIndices.data(), (int64_t)octree.objectIndices.size());
        }
        if (rc != ORT_OK) std::cerr << "scene upload failed: " << ort_last_error(c) << std::endl;
    }
    sceneReady = rc == ORT_OK;
}

void Raytracer::cleanupBuffers() {
    if (dframe) (void)hipFree(dframe);
    dframe = nullptr;
    if (ctx) ort_destroy(ctx);
    if (group) ort_group_destroy(group);
    ctx = nullptr;
    group = nullptr;
    sceneReady = false;
}

ort_params Raytracer::frameParams(const Camera& cam) const {
    ort_params p;
    p.width = width;
    p.height = height;
    p.num_samples = cfg.numSamples;
    p.max_depth = cfg.maxRaysDepth;
    p.use_octree = cfg.useOctree;
    const ortm::mat4 v = cam.GetViewMatrix();
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) p.view[4 * c + r] = v[c][r];
    p.camera_position[0] = cam.Position.x;
    p.camera_position[1] = cam.Position.y;
    p.camera_position[2] = cam.Position.z;
    p.camera_zoom = cam.Zoom;
    return p;
}

int Raytracer::render(const Camera& cam, const ort_tile& tile, float* out, bool outIsDevice, void* stream) {
    if (!ctx && !group && !initialize()) return ORT_ERR_HIP;
    if (group) return ORT_ERR_UNSUPPORTED;  // a group renders whole frames (render(cam, rgb))
    if (!sceneReady) {
        setupScene();
        setupBuffers();
        if (!sceneReady) return ORT_ERR_INVALID_ARG;
    }
    const ort_params p = frameParams(cam);
    return ort_render(ctx, &p, &tile, out, outIsDevice ? 1 : 0, stream);
}

int Raytracer::render(const Camera& cam, float* rgb) {
    if (!ctx && !group && !initialize()) return ORT_ERR_HIP;
    if (group) {
        if (!sceneReady) {
            setupScene();
            setupBuffers();
            if (!sceneReady) return ORT_ERR_INVALID_ARG;
        }
        const ort_params p = frameParams(cam);
        return ort_group_render(group, &p, rgb, 0);
    }
    ort_tile t{0, width, 0, height, 0, 0};
    return render(cam, t, rgb, false, nullptr);
}

void Raytracer::run() {
    if (!initialize()) return;
    setupScene();
    setupBuffers();
    if (!sceneReady) return;
    const size_t frameBytes = sizeof(float) * 3 * (size_t)width * height;
    if (cfg.readback) {
        frame.assign((size_t)width * height * 3, 0.0f);
    } else if (!dframe) {  // on the device that renders (a group: devices[0], where it assembles)
        const int dev = cfg.devices.size() > 1 ? cfg.devices[0] : cfg.device;
        if (hipSetDevice(dev) != hipSuccess || hipMalloc((void**)&dframe, frameBytes) != hipSuccess) {
            dframe = nullptr;
            std::cerr << "run: no device frame buffer of " << frameBytes << " bytes" << std::endl;
            return;
        }
    }
    for (int i = 0; i < cfg.warmupFrames; i++) renderRun();
    for (int i = 0; i < cfg.frames; i++) {
        const auto frameStart = std::chrono::steady_clock::now();
        if (renderRun() != ORT_OK) {
            std::cerr << "render failed: " << lastError() << std::endl;
            break;
        }
        const double frameTime = std::chrono::duration<double>(std::chrono::steady_clock::now() - frameStart).count();
        if (cfg.collectStats) {
            renderTimes.push_back(frameTime);
            frameCount++;
        }
    }
    if (cfg.collectStats) {
        if (cfg.extendedStats && !countWork()) std::cerr << "counting the frame's work failed: " << lastError() << std::endl;
        saveStats();
    }
}

// A synchronous frame either way (ort_render / ort_group_render on the context's own stream
// return once the frame is complete).
int Raytracer::renderRun() {
    if (!dframe) return render(camera, frame.data());
    if (group) {
        const ort_params p = frameParams(camera);
        return ort_group_render(group, &p, dframe, 1);
    }
    const ort_tile t{0, width, 0, height, 0, 0};
    return render(camera, t, dframe, true, nullptr);
}

// saveStats (src/raytracer.cpp:359-449): 2.5-sigma z-score filter, one ';' row.
std::string Raytracer::statsRow(const RaytracerConfig& cfg, const std::vector<double>& all, double buildSeconds,
                                const StatsWork* w) {
    if (all.empty()) return std::string();
    double sum = 0.0;
    for (double t : all) sum += t;
    const double mean = sum / all.size();
    double variance = 0.0;
    for (double t : all) variance += (t - mean) * (t - mean);
    const double stdDev = std::sqrt(variance / all.size());
    const double THRESHOLD = 2.5;
    std::vector<double> clean;
    int outliers = 0;
    for (double t : all) {
        const double z = std::abs(t - mean) / stdDev;
        if (z <= THRESHOLD) clean.push_back(t);
        else outliers++;
    }
    if (outliers > 0) std::cout << "Removed " << outliers << " outliers from " << all.size() << " samples" << std::endl;
    double total = 0.0, mn = clean.empty() ? 9999 : clean[0], mx = clean.empty() ? 0 : clean[0], fpsTotal = 0.0;
    for (double t : clean) {
        total += t;
        mn = std::min(mn, t);
        mx = std::max(mx, t);
        fpsTotal += 1.0 / t;
    }
    if (clean.empty()) {  // every sample an outlier (all equal: stdDev 0, z NaN): the unfiltered data
        clean = all;
        total = sum;
        for (double t : clean) {
            mn = std::min(mn, t);
            mx = std::max(mx, t);
            fpsTotal += 1.0 / t;
        }
    }
    const double avg = total / clean.size();
    const double fpsAvg = fpsTotal / clean.size();
    std::ostringstream row;
    row << cfg.useOctree << ";" << cfg.numSpheres << ";" << cfg.maxDepth << ";" << cfg.maxSpheresPerNode << ";"
        << cfg.numSamples << ";" << cfg.maxRaysDepth << ";" << cfg.width << ";" << cfg.height << ";" << mn << ";" << mx
        << ";" << avg << ";" << 1.0 / mx << ";" << 1.0 / mn << ";" << fpsAvg << ";" << buildSeconds;
    if (w) {
        const double mrays = (double)w->traversals / avg / 1e6;
        const double bytesPerRay = w->traversals ? w->algorithmicBytes / (double)w->traversals : 0.0;
        const double hbmPeakBytes = 8.0e12;  // MI355X HBM3E
        row << ";" << mrays << ";" << bytesPerRay << ";" << mrays * 1e6 * bytesPerRay / hbmPeakBytes << ";" << w->gpus
            << ";" << w->hostCores;
    }
    return row.str();
}

void Raytracer::saveStats() {
    if (renderTimes.empty()) {
        std::cout << "No render times recorded." << std::endl;
        return;
    }
    std::ofstream outFile(statsFilename, std::ios::out | std::ios::app);
    if (!outFile || !outFile.is_open()) {
        std::cerr << "Error opening file for writing: " << statsFilename << std::endl;
        return;
    }
    const double build = (cfg.gpuBuild && !cfg.debug) ? gpuBuildSeconds : octree.buildTime;
    outFile << statsRow(cfg, renderTimes, build, cfg.extendedStats ? &work : nullptr) << std::endl;
}

// The frame's work for the extended columns: the counting variant of the kernel over the
// full frame (untimed; on devices[0]'s context for a group, which holds the same scene).
bool Raytracer::countWork() {
    ort_ctx* c = ctx;
    if (group && ort_group_context(group, 0, &c) != ORT_OK) return false;
    const ort_params p = frameParams(camera);
    const ort_tile t{0, width, 0, height, 0, 0};
    uint64_t n[ORT_COUNT_N] = {0};
    if (ort_count_traffic(c, &p, &t, n) != ORT_OK) return false;
    work.traversals = n[ORT_COUNT_TRAVERSALS];
    work.algorithmicBytes = 36.0 * n[ORT_COUNT_NODES_POPPED] + 32.0 * n[ORT_COUNT_CHILD_RECORDS] +
                            20.0 * n[ORT_COUNT_LEAF_OBJECTS] + 32.0 * n[ORT_COUNT_ACCEPTED_HITS] +
                            12.0 * n[ORT_COUNT_PIXELS];
    work.gpus = group ? ort_group_size(group) : 1;
    cpu_set_t set;
    work.hostCores = sched_getaffinity(0, sizeof(set), &set) == 0 ? CPU_COUNT(&set) : 1;
    return true;
}

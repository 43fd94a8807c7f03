// examples/main.cpp -- the reference's entry point (src/main.cpp:28-54) on this library:
// configure, Raytracer::initialize(), Raytracer::run().  Headless: instead of a window it
// can write the last frame as a PPM (--ppm) and appends the saveStats CSV row (--stats).
//   build: make examples   ->  build/ort_main
//   run:   build/ort_main --spheres 1000 --depth 5 --samples 4 --bounces 4 --width 800
//          --height 600 --frames 10 --stats stats.csv [--stats-ext] [--readback] --ppm frame.ppm
// tools/sweep.py drives it over the reference's experiment grid (analysis/runner.py:99-192).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <vector>

#include "raytracer.h"

int main(int argc, char** argv) {
    RaytracerConfig cfg;
    const char* ppm = nullptr;
    for (int i = 1; i < argc; ++i) {
        auto next = [&](void) -> const char* { return (i + 1 < argc) ? argv[++i] : "0"; };
        if (!std::strcmp(argv[i], "--spheres")) cfg.numSpheres = std::atoi(next());
        else if (!std::strcmp(argv[i], "--depth")) cfg.maxDepth = std::atoi(next());
        else if (!std::strcmp(argv[i], "--per-node")) cfg.maxSpheresPerNode = std::atoi(next());
        else if (!std::strcmp(argv[i], "--samples")) cfg.numSamples = std::atoi(next());
        else if (!std::strcmp(argv[i], "--bounces")) cfg.maxRaysDepth = std::atoi(next());
        else if (!std::strcmp(argv[i], "--width")) cfg.width = (unsigned)std::atoi(next());
        else if (!std::strcmp(argv[i], "--height")) cfg.height = (unsigned)std::atoi(next());
        else if (!std::strcmp(argv[i], "--frames")) cfg.frames = std::atoi(next());
        else if (!std::strcmp(argv[i], "--warmup")) cfg.warmupFrames = std::atoi(next());
        else if (!std::strcmp(argv[i], "--no-octree")) cfg.useOctree = 0;
        else if (!std::strcmp(argv[i], "--prebuilt")) cfg.usePrebuilt = 1;
        else if (!std::strcmp(argv[i], "--debug")) cfg.debug = 1;
        else if (!std::strcmp(argv[i], "--gpu-build")) cfg.gpuBuild = true;
        else if (!std::strcmp(argv[i], "--seed")) cfg.seed = (uint32_t)std::strtoul(next(), nullptr, 10);
        else if (!std::strcmp(argv[i], "--device")) cfg.device = std::atoi(next());
        else if (!std::strcmp(argv[i], "--devices")) {  // e.g. 0,1,2,3,4,5,6,7: one ort_group (RCCL gather)
            cfg.devices.clear();
            for (const char* q = next(); *q;) {
                cfg.devices.push_back(std::atoi(q));
                while (*q && *q != ',') ++q;
                if (*q == ',') ++q;
            }
        }
        else if (!std::strcmp(argv[i], "--stats")) { cfg.collectStats = true; cfg.outputFile = next(); }
        else if (!std::strcmp(argv[i], "--stats-ext")) cfg.extendedStats = true;  // + 5 throughput columns
        else if (!std::strcmp(argv[i], "--readback")) cfg.readback = true;  // timed frames copied to the host
        else if (!std::strcmp(argv[i], "--ppm")) ppm = next();
        else { std::fprintf(stderr, "unknown argument %s\n", argv[i]); return 2; }
    }
    Raytracer raytracer(cfg);
    if (!raytracer.initialize()) return -1;
    raytracer.run();
    if (ppm) {
        std::vector<float> rgb((size_t)cfg.width * cfg.height * 3);
        if (raytracer.render(raytracer.camera, rgb.data()) != ORT_OK) {
            std::fprintf(stderr, "render failed: %s\n", raytracer.lastError());
            return 1;
        }
        std::ofstream f(ppm, std::ios::binary);
        f << "P6\n" << cfg.width << " " << cfg.height << "\n255\n";
        for (int y = (int)cfg.height - 1; y >= 0; --y)  // GL rows are bottom-up
            for (unsigned x = 0; x < cfg.width; ++x)
                for (int c = 0; c < 3; ++c) {
                    float v = rgb[3 * ((size_t)y * cfg.width + x) + c];
                    v = v != v ? 0.0f : (v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v));
                    f.put((char)(unsigned char)(v * 255.0f + 0.5f));
                }
    }
    const auto& t = raytracer.getRenderTimes();
    if (!t.empty()) {
        double s = 0;
        for (double v : t) s += v;
        std::printf("%zu frames, mean %.3f ms/frame\n", t.size(), 1e3 * s / t.size());
    }
    return 0;
}

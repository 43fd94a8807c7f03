// tests/cpp/stats_row.cpp -- prints Raytracer::statsRow for frame times given on the command
// line (no GPU): the CPU test of the saveStats schema (src/raytracer.cpp:359-449) and of the
// extended throughput columns.
//   stats_row <traversals> <algorithmic bytes> <gpus> <host cores> <t0> <t1> ...   (seconds)
// traversals == 0 prints the reference's 15-column row only.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "raytracer.h"

int main(int argc, char** argv) {
    if (argc < 6) {
        std::fprintf(stderr, "usage: %s traversals bytes gpus cores t0 [t1 ...]\n", argv[0]);
        return 2;
    }
    RaytracerConfig cfg;
    cfg.numSpheres = 100000;
    cfg.maxDepth = 8;
    cfg.numSamples = 1;
    cfg.maxRaysDepth = 1;
    cfg.width = 3840;
    cfg.height = 2160;
    StatsWork w;
    w.traversals = std::strtoull(argv[1], nullptr, 10);
    w.algorithmicBytes = std::atof(argv[2]);
    w.gpus = std::atoi(argv[3]);
    w.hostCores = std::atoi(argv[4]);
    std::vector<double> t;
    for (int i = 5; i < argc; ++i) t.push_back(std::atof(argv[i]));
    std::printf("%s\n", Raytracer::statsRow(cfg, t, 0.25, w.traversals ? &w : nullptr).c_str());
    return 0;
}

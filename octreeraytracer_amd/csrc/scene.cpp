// scene.cpp -- restatement of the reference's scene generators (see scene.h).
#include "scene.h"

#include <algorithm>
#include <cmath>
#include <random>

namespace ort {

std::vector<Sphere> generateRandomSpheres(int numSpheres, uint32_t seed) {
    std::vector<Sphere> spheres;
    if (numSpheres <= 0) return spheres;
    spheres.reserve((size_t)numSpheres);
    std::mt19937 gen(seed);

    std::uniform_real_distribution<float> colorDis(0.0f, 1.0f);
    std::uniform_real_distribution<float> fuzzDis(0.0f, 0.5f);
    std::uniform_real_distribution<float> refIndexDis(1.3f, 1.7f);
    std::uniform_real_distribution<float> smallJitter(-0.2f, 0.2f);
    std::uniform_real_distribution<float> heightDis(0.0f, 4.0f);

    const float radius = 0.2f;
    const float minSpacing = radius * 2.5f;
    const int gridSize = static_cast<int>(std::ceil(std::sqrt(numSpheres)));
    float worldSize = gridSize * minSpacing * 1.2f;
    worldSize = std::min(worldSize, 100.0f);
    const float halfWorld = worldSize / 2.0f;
    float cellSize = worldSize / gridSize;
    if (cellSize < minSpacing) cellSize = minSpacing;

    const int totalSpheres = numSpheres;
    const int metalCount = totalSpheres / 5;
    const int glassCount = totalSpheres / 5;
    int metalRemaining = metalCount;
    int glassRemaining = glassCount;
    int diffuseRemaining = totalSpheres - metalCount - glassCount;

    int count = 0;
    for (int i = 0; i < gridSize && count < numSpheres; i++) {
        for (int j = 0; j < gridSize && count < numSpheres; j++) {
            const float baseX = -halfWorld + (i + 0.5f) * cellSize;
            const float baseY = radius + (heightDis(gen) * (i % 3 + j % 3 + 1) / 5.0f);
            const float baseZ = -halfWorld + (j + 0.5f) * cellSize;
            const float jitterAmount = std::min(cellSize * 0.3f, minSpacing * 0.4f);
            const float offsetX = smallJitter(gen) * jitterAmount;
            const float offsetZ = smallJitter(gen) * jitterAmount;
            const ortm::vec3 center(baseX + offsetX, baseY, baseZ + offsetZ);

            int materialType = 0;
            if (metalRemaining > 0 && (diffuseRemaining <= 0 || (count % 5 == 1))) {
                materialType = 1;
                metalRemaining--;
            } else if (glassRemaining > 0 && (diffuseRemaining <= 0 || (count % 5 == 3))) {
                materialType = 2;
                glassRemaining--;
            } else {
                materialType = 0;
                diffuseRemaining--;
            }
            const float ax = colorDis(gen);
            const float ay = colorDis(gen);
            const float az = colorDis(gen);
            const float fuzz = (materialType == 1) ? fuzzDis(gen) : 0.0f;
            const float refractionIndex = (materialType == 2) ? refIndexDis(gen) : 1.0f;
            spheres.emplace_back(center, radius, materialType, ortm::vec3(ax, ay, az), fuzz, refractionIndex);
            count++;
        }
    }
    return spheres;
}

namespace {
struct PrebuiltRow {
    double cx, cy, cz, r;
    int mat;
    double ax, ay, az, fuzz, ri;
};
const PrebuiltRow kPrebuilt[] = {
#include "prebuilt_scene.inc"
};
}  // namespace

std::vector<Sphere> generatePreBuiltSpheres() {
    std::vector<Sphere> spheres;
    spheres.reserve(sizeof(kPrebuilt) / sizeof(kPrebuilt[0]));
    for (const PrebuiltRow& p : kPrebuilt)
        spheres.emplace_back(ortm::vec3((float)p.cx, (float)p.cy, (float)p.cz), (float)p.r, p.mat,
                             ortm::vec3((float)p.ax, (float)p.ay, (float)p.az), (float)p.fuzz, (float)p.ri);
    return spheres;
}

std::vector<Sphere> generateDebugSpheres() {
    std::vector<Sphere> s;
    s.emplace_back(ortm::vec3(-10.0f, -10.0f, -10.0f), 3.0f, 0, ortm::vec3((float)0.596282, (float)0.140784, (float)0.017972), 1.0f, 1.0f);
    s.emplace_back(ortm::vec3(10.0f, 10.0f, 10.0f), 3.0f, 0, ortm::vec3((float)0.952200, (float)0.391551, (float)0.915972), 1.0f, 1.0f);
    s.emplace_back(ortm::vec3(-10.0f, 10.0f, -10.0f), 3.0f, 0, ortm::vec3((float)0.002612, (float)0.598319, (float)0.435378), 1.0f, 1.0f);
    return s;
}

void packSpheres(const std::vector<Sphere>& spheres, float* cr, float* ma, float* fr) {
    for (size_t i = 0; i < spheres.size(); ++i) {
        const Sphere& s = spheres[i];
        if (cr) { cr[4 * i] = s.center.x; cr[4 * i + 1] = s.center.y; cr[4 * i + 2] = s.center.z; cr[4 * i + 3] = s.radius; }
        if (ma) { ma[4 * i] = float(s.materialType); ma[4 * i + 1] = s.albedo.x; ma[4 * i + 2] = s.albedo.y; ma[4 * i + 3] = s.albedo.z; }
        if (fr) { fr[4 * i] = s.fuzz; fr[4 * i + 1] = s.refractionIndex; fr[4 * i + 2] = 0.0f; fr[4 * i + 3] = 0.0f; }
    }
}

std::vector<Sphere> unpackSpheres(const float* cr, const float* ma, const float* fr, int n) {
    std::vector<Sphere> out;
    out.reserve((size_t)std::max(n, 0));
    for (int i = 0; i < n; ++i) {
        const ortm::vec3 c(cr[4 * i], cr[4 * i + 1], cr[4 * i + 2]);
        const int mt = ma ? (int)ma[4 * i] : 0;
        const ortm::vec3 alb = ma ? ortm::vec3(ma[4 * i + 1], ma[4 * i + 2], ma[4 * i + 3]) : ortm::vec3(1.0f);
        out.emplace_back(c, cr[4 * i + 3], mt, alb, fr ? fr[4 * i] : 0.0f, fr ? fr[4 * i + 1] : 1.0f);
    }
    return out;
}

}  // namespace ort

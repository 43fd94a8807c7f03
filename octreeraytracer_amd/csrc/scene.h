// scene.h -- scene generators of the reference's Raytracer (src/raytracer.cpp:164-357),
// exposed as free functions so the C ABI, the C++ Raytracer and the tests share them.
#pragma once
#include <cstdint>
#include <vector>
#include "sphere.h"

namespace ort {

// generateRandomSpheres (src/raytracer.cpp:254-337).  The reference seeds std::mt19937
// from std::random_device (:256-257), which is not reproducible; here the seed is an
// argument.  Draw order: heightDis, smallJitter x2, colorDis x3 (x, y, z), fuzzDis if
// metal, refIndexDis if glass.  materialTypeDis (:260) is never drawn, as in the reference.
std::vector<Sphere> generateRandomSpheres(int numSpheres, uint32_t seed);

// generatePreBuiltSpheres (src/raytracer.cpp:164-252): 83 deterministic spheres.
std::vector<Sphere> generatePreBuiltSpheres();

// The DEBUG scene (src/raytracer.cpp:342-347): 3 spheres of radius 3.
std::vector<Sphere> generateDebugSpheres();

// SoA packing of setupBuffers (src/raytracer.cpp:87-91).
void packSpheres(const std::vector<Sphere>& spheres, float* centerRadius, float* matAlbedo, float* fuzzRi);
std::vector<Sphere> unpackSpheres(const float* centerRadius, const float* matAlbedo, const float* fuzzRi, int n);

}  // namespace ort

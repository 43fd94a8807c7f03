// sphere.h -- the reference's Sphere (src/sphere.h:7-23; src/sphere.cpp is empty).
// Same members, same constructor defaults; vec3 is ortm::vec3 (glm-layout compatible).
#pragma once
#include "vecmath.h"

class Sphere {
public:
    // sphere properties
    ortm::vec3 center;
    float radius;

    // material: 0 = Lambert, 1 = Metal, 2 = Dielectric (glsl:5-7)
    int materialType;
    ortm::vec3 albedo;
    float fuzz;
    float refractionIndex;

    Sphere(const ortm::vec3& center, float radius, int materialType = 0,
           const ortm::vec3& albedo = ortm::vec3(1.0f), float fuzz = 0.0f, float refractionIndex = 1.0f)
        : center(center), radius(radius), materialType(materialType), albedo(albedo), fuzz(fuzz),
          refractionIndex(refractionIndex) {}
};

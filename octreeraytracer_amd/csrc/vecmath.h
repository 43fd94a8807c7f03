// vecmath.h -- the small slice of glm 1.0.0 the reference's host code uses
// (vec3/vec4/mat4, dot/cross/normalize/min/max/lookAt), restated with glm's exact
// float evaluation order so the scene-build stage is bit-identical to the reference:
//   dot        include/glm/detail/func_geometric.inl:48-55   (x*x' + y*y') + z*z'
//   cross      include/glm/detail/func_geometric.inl:68-79
//   normalize  include/glm/detail/func_geometric.inl:82-90 + func_exponential.inl:136-139
//   min/max    include/glm/detail/func_common.inl:17-21      (y < x) ? y : x
//   lookAtRH   include/glm/ext/matrix_transform.inl:153-173
// glm itself is not installed on this system and is not vendored; vec3 is layout
// compatible with glm::vec3 (three packed floats) for callers that convert.
#pragma once
#include <cmath>

namespace ortm {

struct vec3 {
    float x = 0.f, y = 0.f, z = 0.f;
    vec3() = default;
    explicit vec3(float s) : x(s), y(s), z(s) {}
    vec3(float a, float b, float c) : x(a), y(b), z(c) {}
    float& operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
    float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};
static_assert(sizeof(vec3) == 12, "vec3 must be three packed floats");

inline vec3 operator+(const vec3& a, const vec3& b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline vec3 operator-(const vec3& a, const vec3& b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline vec3 operator*(const vec3& a, const vec3& b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline vec3 operator*(const vec3& a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline vec3 operator*(float s, const vec3& a) { return {s * a.x, s * a.y, s * a.z}; }
inline vec3 operator/(const vec3& a, float s) { return {a.x / s, a.y / s, a.z / s}; }
inline vec3 operator-(const vec3& a) { return {-a.x, -a.y, -a.z}; }
inline vec3& operator+=(vec3& a, const vec3& b) { a = a + b; return a; }
inline vec3& operator-=(vec3& a, const vec3& b) { a = a - b; return a; }
inline bool operator==(const vec3& a, const vec3& b) { return a.x == b.x && a.y == b.y && a.z == b.z; }

inline float fmin_glm(float x, float y) { return (y < x) ? y : x; }
inline float fmax_glm(float x, float y) { return (x < y) ? y : x; }
inline vec3 min(const vec3& a, const vec3& b) { return {fmin_glm(a.x, b.x), fmin_glm(a.y, b.y), fmin_glm(a.z, b.z)}; }
inline vec3 max(const vec3& a, const vec3& b) { return {fmax_glm(a.x, b.x), fmax_glm(a.y, b.y), fmax_glm(a.z, b.z)}; }
inline float dot(const vec3& a, const vec3& b) {
    const vec3 t = a * b;
    return t.x + t.y + t.z;
}
inline vec3 cross(const vec3& a, const vec3& b) {
    return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y};
}
inline vec3 normalize(const vec3& v) { return v * (1.0f / std::sqrt(dot(v, v))); }
inline float radians(float deg) { return deg * 0.01745329251994329576923690768489f; }

struct vec4 {
    float x = 0.f, y = 0.f, z = 0.f, w = 0.f;
    vec4() = default;
    vec4(float a, float b, float c, float d) : x(a), y(b), z(c), w(d) {}
    vec4(const vec3& v, float d) : x(v.x), y(v.y), z(v.z), w(d) {}
};

// Column-major 4x4 like glm::mat4: m[col][row].
struct mat4 {
    float m[4][4];
    explicit mat4(float diag = 1.0f) {
        for (int c = 0; c < 4; ++c)
            for (int r = 0; r < 4; ++r) m[c][r] = (c == r) ? diag : 0.0f;
    }
    float* operator[](int c) { return m[c]; }
    const float* operator[](int c) const { return m[c]; }
};

inline mat4 lookAt(const vec3& eye, const vec3& center, const vec3& up) {
    const vec3 f = normalize(center - eye);
    const vec3 s = normalize(cross(f, up));
    const vec3 u = cross(s, f);
    mat4 R(1.0f);
    R[0][0] = s.x; R[1][0] = s.y; R[2][0] = s.z;
    R[0][1] = u.x; R[1][1] = u.y; R[2][1] = u.z;
    R[0][2] = -f.x; R[1][2] = -f.y; R[2][2] = -f.z;
    R[3][0] = -dot(s, eye);
    R[3][1] = -dot(u, eye);
    R[3][2] = dot(f, eye);
    return R;
}

}  // namespace ortm

// camera.h -- the reference's Euler-angle Camera (src/opengl/camera.h:11-128) without
// the GL include, plus the per-frame camera frame the shader derives from the view
// uniform (Camera_initFromViewMatrix, glsl:176-202), computed once per frame on the host.
#pragma once
#include <cmath>
#include "../../include/ort_math.h"
#include "vecmath.h"

enum Camera_Movement { FORWARD, BACKWARD, LEFT, RIGHT };

const float YAW = -90.0f;
const float PITCH = 0.0f;
const float SPEED = 2.5f;
const float SENSITIVITY = 0.1f;
const float ZOOM = 45.0f;

class Camera {
public:
    ortm::vec3 Position;
    ortm::vec3 Front;
    ortm::vec3 Up;
    ortm::vec3 Right;
    ortm::vec3 WorldUp;
    float Yaw;
    float Pitch;
    float MovementSpeed;
    float MouseSensitivity;
    float Zoom;

    Camera(ortm::vec3 position = ortm::vec3(0.0f, 0.0f, 0.0f), ortm::vec3 up = ortm::vec3(0.0f, 1.0f, 0.0f),
           float yaw = YAW, float pitch = PITCH)
        : Front(ortm::vec3(0.0f, 0.0f, -1.0f)), MovementSpeed(SPEED), MouseSensitivity(SENSITIVITY), Zoom(ZOOM) {
        Position = position;
        WorldUp = up;
        Yaw = yaw;
        Pitch = pitch;
        updateCameraVectors();
    }

    ortm::mat4 GetViewMatrix() const { return ortm::lookAt(Position, Position + Front, Up); }

    // Inverted WASD exactly as the reference (camera.h:70-81).
    void ProcessKeyboard(Camera_Movement direction, float deltaTime) {
        const float velocity = MovementSpeed * deltaTime;
        if (direction == FORWARD) Position -= Front * velocity;
        if (direction == BACKWARD) Position += Front * velocity;
        if (direction == LEFT) Position -= Right * velocity;
        if (direction == RIGHT) Position += Right * velocity;
    }

    void ProcessMouseMovement(float xoffset, float yoffset, bool constrainPitch = true) {
        xoffset *= MouseSensitivity;
        yoffset *= MouseSensitivity;
        Yaw -= xoffset;
        Pitch -= yoffset;
        if (constrainPitch) {
            if (Pitch > 89.0f) Pitch = 89.0f;
            if (Pitch < -89.0f) Pitch = -89.0f;
        }
        updateCameraVectors();
    }

    void ProcessMouseScroll(float yoffset) {
        Zoom -= yoffset;
        if (Zoom < 1.0f) Zoom = 1.0f;
        if (Zoom > 45.0f) Zoom = 45.0f;
    }

    void updateCameraVectors() {
        ortm::vec3 front;
        front.x = std::cos(ortm::radians(Yaw)) * std::cos(ortm::radians(Pitch));
        front.y = std::sin(ortm::radians(Pitch));
        front.z = std::sin(ortm::radians(Yaw)) * std::cos(ortm::radians(Pitch));
        Front = ortm::normalize(front);
        Right = ortm::normalize(ortm::cross(Front, WorldUp));
        Up = ortm::normalize(ortm::cross(Right, Front));
    }
};

namespace ort {

// Camera struct of glsl:79-86 as derived by Camera_initFromViewMatrix (glsl:176-202).
struct CameraFrame {
    float origin[3], lowerLeft[3], horizontal[3], vertical[3], u[3], v[3], w[3];
    float lensRadius;
};

inline void glsl_normalize3(const float in[3], float out[3]) {
    const float d = (in[0] * in[0] + in[1] * in[1]) + in[2] * in[2];
    const float s = 1.0f / sqrtf(d);
    out[0] = in[0] * s;
    out[1] = in[1] * s;
    out[2] = in[2] * s;
}

// view: column-major mat4 (view[4*col + row]), so GLSL viewMatrix[c][r] == view[4*c + r].
inline CameraFrame cameraFrameFromView(const float view[16], const float position[3], float fovDegrees, float aspect) {
    CameraFrame c;
    for (int k = 0; k < 3; ++k) c.origin[k] = position[k];
    const float wcol[3] = {view[0 * 4 + 2], view[1 * 4 + 2], view[2 * 4 + 2]};
    const float ucol[3] = {view[0 * 4 + 0], view[1 * 4 + 0], view[2 * 4 + 0]};
    const float vcol[3] = {view[0 * 4 + 1], view[1 * 4 + 1], view[2 * 4 + 1]};
    float wn[3];
    glsl_normalize3(wcol, wn);
    for (int k = 0; k < 3; ++k) c.w[k] = -wn[k];
    glsl_normalize3(ucol, c.u);
    glsl_normalize3(vcol, c.v);
    const float aperture = 0.1f;
    c.lensRadius = aperture / 2.0f;
    const float distToFocus = 10.0f;
    const float PI_F = (float)3.14159265359;
    const float theta = fovDegrees * PI_F / 180.0f;
    const float halfHeight = ort_tanf(theta / 2.0f);
    const float halfWidth = aspect * halfHeight;
    const float hw = halfWidth * distToFocus, hh = halfHeight * distToFocus;
    const float hw2 = 2.0f * halfWidth * distToFocus, hh2 = 2.0f * halfHeight * distToFocus;
    for (int k = 0; k < 3; ++k) {
        c.lowerLeft[k] = ((c.origin[k] - hw * c.u[k]) - hh * c.v[k]) - distToFocus * c.w[k];
        c.horizontal[k] = hw2 * c.u[k];
        c.vertical[k] = hh2 * c.v[k];
    }
    return c;
}

}  // namespace ort

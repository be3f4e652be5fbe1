// camera.h — headless orbit camera (Utils/camera.h:8-75) and the glm helpers
// main.cpp uses (perspective, lookAt, inverse of a rigid view, mat4 product),
// in float32 with glm's column-major layout. Same arithmetic, operation for
// operation, as ptsvgf/camera.py, so the C++ and Python drivers issue
// bit-identical uniforms.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstring>

namespace host {

struct mat4 {
  float m[16];  // column-major: m[c*4 + r]
};

inline float radians(float deg) { return deg * 0.01745329251994329576923690768489f; }

inline mat4 perspective(float fovy, float aspect, float znear, float zfar) {  // glm::perspective (RH, -1..1)
  const float t = (float)std::tan((double)(fovy / 2.0f));
  mat4 r;
  std::memset(r.m, 0, sizeof r.m);
  r.m[0] = 1.0f / (aspect * t);
  r.m[5] = 1.0f / t;
  r.m[10] = -(zfar + znear) / (zfar - znear);
  r.m[11] = -1.0f;
  r.m[14] = -(2.0f * zfar * znear) / (zfar - znear);
  return r;
}

inline void normalize3(float* v) {
  const float d = (v[0] * v[0] + v[1] * v[1]) + v[2] * v[2];
  const float k = 1.0f / std::sqrt(d);
  v[0] *= k;
  v[1] *= k;
  v[2] *= k;
}
inline void cross3(const float* a, const float* b, float* o) {
  o[0] = a[1] * b[2] - b[1] * a[2];
  o[1] = a[2] * b[0] - b[2] * a[0];
  o[2] = a[0] * b[1] - b[0] * a[1];
}
inline float dot3(const float* a, const float* b) { return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]; }

inline mat4 look_at(const float* eye, const float* center, const float* up) {  // glm::lookAt (RH)
  float f[3] = {center[0] - eye[0], center[1] - eye[1], center[2] - eye[2]};
  normalize3(f);
  float s[3];
  cross3(f, up, s);
  normalize3(s);
  float u[3];
  cross3(s, f, u);
  mat4 r;
  std::memset(r.m, 0, sizeof r.m);
  r.m[15] = 1.0f;
  r.m[0] = s[0]; r.m[4] = s[1]; r.m[8] = s[2];
  r.m[1] = u[0]; r.m[5] = u[1]; r.m[9] = u[2];
  r.m[2] = -f[0]; r.m[6] = -f[1]; r.m[10] = -f[2];
  r.m[12] = -dot3(s, eye);
  r.m[13] = -dot3(u, eye);
  r.m[14] = dot3(f, eye);
  return r;
}

inline mat4 rigid_inverse(const mat4& v) {  // inverse(view), main.cpp:445
  mat4 r;
  std::memset(r.m, 0, sizeof r.m);
  for (int row = 0; row < 3; ++row)
    for (int col = 0; col < 3; ++col) r.m[col * 4 + row] = v.m[row * 4 + col];
  const float* t = v.m + 12;
  for (int row = 0; row < 3; ++row) r.m[12 + row] = -((r.m[row] * t[0] + r.m[4 + row] * t[1]) + r.m[8 + row] * t[2]);
  r.m[15] = 1.0f;
  return r;
}

inline mat4 mul(const mat4& a, const mat4& b) {  // glm mat4 * mat4
  mat4 o;
  for (int c = 0; c < 4; ++c)
    for (int r = 0; r < 4; ++r)
      o.m[c * 4 + r] = ((a.m[r] * b.m[c * 4] + a.m[4 + r] * b.m[c * 4 + 1]) + a.m[8 + r] * b.m[c * 4 + 2]) +
                       a.m[12 + r] * b.m[c * 4 + 3];
  return o;
}

// Utils/camera.h:8-75; orbit() stands in for the mouse callbacks (main.cpp:614-655)
struct Camera {
  int width, height;
  float near_plane = 0.01f, far_plane = 1000.0f;
  float upAngle = 10.0f, rotatAngle = 0.0f, r_dis = 2.0f;
  float move_vec[3] = {0, 0, 0};
  float look_at_point[3] = {0, 0, 0};
  float cam_position[3];
  unsigned frameCounter = 0;
  bool dirty = false;
  mat4 cam_proj_mat, cam_view_mat;

  Camera(int w, int h) : width(w), height(h) {
    orbit_eye(cam_position);
    cam_proj_mat = perspective(radians(90.0f), (float)width / (float)height, near_plane, far_plane);
    const float up[3] = {0, 1, 0};
    cam_view_mat = look_at(cam_position, move_vec, up);
  }
  void orbit_eye(float* e) const {
    const double ra = radians(rotatAngle), ua = radians(upAngle);
    e[0] = (float)(-std::sin(ra) * std::cos(ua)) * r_dis;
    e[1] = (float)std::sin(ua) * r_dis;
    e[2] = (float)(std::cos(ra) * std::cos(ua)) * r_dis;
  }
  void orbit(float d_rot_deg, float d_up_deg) {  // cursor_position_callback, main.cpp:614-630
    frameCounter = 0;
    rotatAngle = rotatAngle + d_rot_deg;
    upAngle = std::min(std::max(upAngle + d_up_deg, -89.0f), 89.0f);
    dirty = true;
  }
  void update() {  // Camera::update, camera.h:62-74
    if (!dirty) return;
    float e[3];
    orbit_eye(e);
    for (int k = 0; k < 3; ++k) {
      cam_position[k] = e[k] + move_vec[k];
      look_at_point[k] = move_vec[k];
    }
    const float up[3] = {0, 1, 0};
    cam_view_mat = look_at(cam_position, look_at_point, up);
    frameCounter = 0;
    dirty = false;
  }
};

// Utils/gui_config.h:19-46 slider defaults (accumulate off for 1 spp + SVGF)
struct parameter_config {
  float sigma_z = 1.0f, sigma_n = 128.0f, sigma_l = 4.0f;
  float reproj_normal_threshold = 16.0f, reproj_depth_threshold = 10.0f, clamp_threshold = 10.0f;
  int max_tracing_depth = 2, num_atrous_iterations = 5;
  bool accumulate_color = false, use_normal_texture = false;
};

}  // namespace host

// render_pass.h — the reference's GL plumbing classes re-expressed over the
// C ABI of include/ptsvgf.h, so main.cpp-style C++ host code drives the
// MI355X kernels unchanged. Same class names, members and
// call semantics as:
//   RenderPass            Utils/render_pass.h:82-182
//   Rasterize_RenderPass  Utils/render_pass.h:5-80
//   getShaderProgram      Utils/shader.h:21-67
//   getTextureRGB32F      Utils/help_func.h:22-32
// Errors: the reference exits on a missing shader (shader.h:8-12); every
// failing call here prints pt_last_error() and exits the same way.
#pragma once
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/ptsvgf.h"

typedef uint32_t GLuint;
typedef int GLint;
typedef uint32_t GLenum;
typedef char GLchar;
#define GL_TEXTURE_2D PT_TEXTURE_2D
#define GL_TEXTURE_BUFFER PT_TEXTURE_BUFFER
#define GL_TEXTURE_2D_ARRAY PT_TEXTURE_2D_ARRAY
#define GL_RGB32F PT_RGB32F
#define GL_RGBA32F PT_RGBA32F

#ifndef SCR_WIDTH
#define SCR_WIDTH 800   // Utils/camera.h:5-6
#define SCR_HEIGHT 800
#endif

inline void pt_check(int rc, const char* what) {
  if (rc < 0) {
    std::fprintf(stderr, "ptsvgf: %s failed: %s\n", what, pt_last_error());
    std::exit(-1);
  }
}

inline GLuint getShaderProgram(const std::string& fshader, const std::string& vshader) {
  uint32_t h = 0;
  pt_check(pt_program_create(fshader.c_str(), vshader.c_str(), &h), "getShaderProgram");
  return h;
}

inline GLuint getTextureRGB32F(int width, int height) {
  uint32_t t = 0;
  pt_check(pt_texture2d_create(width, height, &t), "getTextureRGB32F");
  return t;
}

class RenderPass {
 public:
  std::vector<GLuint> colorAttachments;
  GLuint program = 0;
  int width = SCR_WIDTH;
  int height = SCR_HEIGHT;
  GLint texture_slot = 0;

  void bindData(bool finalPass = false) {
    for (GLuint t : colorAttachments) pt_check(pt_pass_add_color_attachment(handle(), t), "bindData");
    pt_check(pt_pass_bind(handle(), finalPass ? 1 : 0), "bindData");
  }
  void draw(const std::vector<GLuint>& texPassArray = {}) {
    for (size_t i = 0; i < texPassArray.size(); ++i)
      pt_check(pt_pass_set_texture(handle(), GL_TEXTURE_2D, texPassArray[i], ("texPass" + std::to_string(i)).c_str()),
               "draw");
    pt_check(pt_pass_draw(handle()), "draw");
  }
  void reset_texture_slot() {
    texture_slot = 0;
    pt_check(pt_pass_reset_texture_slot(handle()), "reset_texture_slot");
  }
  void set_texture_uniform(GLenum target, GLuint tex, const GLchar* name) {
    pt_check(pt_pass_set_texture(handle(), target, tex, name), name);
    ++texture_slot;
  }
  void set_uniform_mat4(const GLchar* n, const float* m16) { pt_check(pt_pass_set_uniform_mat4(handle(), n, m16), n); }
  void set_uniform_float(const GLchar* n, float v) { pt_check(pt_pass_set_uniform_float(handle(), n, v), n); }
  void set_uniform_int(const GLchar* n, int v) { pt_check(pt_pass_set_uniform_int(handle(), n, v), n); }
  void set_uniform_uint(const GLchar* n, unsigned v) { pt_check(pt_pass_set_uniform_uint(handle(), n, v), n); }
  void set_uniform_bool(const GLchar* n, bool v) { pt_check(pt_pass_set_uniform_bool(handle(), n, v ? 1 : 0), n); }
  void set_uniform_vec3(const GLchar* n, const float* v3) { pt_check(pt_pass_set_uniform_vec3(handle(), n, v3), n); }

  // MI355X additions (no reference counterpart)
  float last_ms() {
    float ms = 0.0f;
    pt_check(pt_pass_last_ms(handle(), &ms), "last_ms");
    return ms;
  }

 protected:
  uint32_t h_ = 0;
  uint32_t handle() {
    if (!h_) pt_check(pt_pass_create(program, width, height, &h_), "pt_pass_create");
    return h_;
  }
};

class Rasterize_RenderPass : public RenderPass {
 public:
  // Utils/render_pass.h:19-62: the vertex list is pos3 + normal3 per vertex
  void bindData(const std::vector<float>& vertices) {
    for (GLuint t : colorAttachments) pt_check(pt_pass_add_color_attachment(handle(), t), "bindData");
    pt_check(pt_raster_pass_bind(handle(), vertices.data(), vertices.size()), "Rasterize_RenderPass::bindData");
  }
  void draw() { pt_check(pt_pass_draw(handle()), "draw"); }
};

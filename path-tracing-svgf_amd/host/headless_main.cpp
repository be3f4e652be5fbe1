// headless_main.cpp — the reference's main.cpp driven headless through the
// C++ RenderPass mirror (render_pass.h) over the HIP C ABI: the same program
// objects, textures, pass wiring, uniforms and per-frame call order as
// main.cpp:65-602 (window, ImGui and input callbacks removed; the camera orbit
// is scripted). Scene preparation goes through include/ptsvgf_scene.h
// (readObj / buildBVHwithSAH / encode / calculateHdrCache).
//
// usage: ptsvgf_headless [--width W] [--height H] [--frames N] [--orbit DEG]
//                        [--scene table_clock_plant|clock] [--assets DIR]
//                        [--hdr WxH] [--leaves N] [--atrous-exact] [--out FILE]
// --out writes, per frame, the planes color, albedo, modulate, taa, output as
// float32 RGBA (H x W x 4 each) for the cross-driver test (tests/test_gpu_host.py).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ptsvgf_scene.h"
#include "camera.h"
#include "render_pass.h"

namespace {

const std::string SHADERS = "./shaders/";

struct Scene {
  std::vector<float> tri, node, raster, lights, hdr, cache;
  int ntris = 0, nnodes = 0, hdr_w = 0, hdr_h = 0;
};

void host_check(int rc, const char* what) {
  if (rc < 0) {
    std::fprintf(stderr, "scene: %s failed: %s\n", what, pts_last_error());
    std::exit(-1);
  }
}

// Utils/Material.h:8-22 defaults, in the 18-float order of ptsvgf_scene.h
struct Material {
  float emissive[3] = {0, 0, 0}, baseColor[3] = {1, 1, 1};
  float subsurface = 0, metallic = 0, specular = 0.5f, specularTint = 0, roughness = 0.5f, anisotropic = 0;
  float sheen = 0, sheenTint = 0.5f, clearcoat = 0, clearcoatGloss = 1.0f, IOR = 1.0f, transmission = 0;
  void pack(float* o) const {
    const float v[18] = {emissive[0], emissive[1], emissive[2], baseColor[0], baseColor[1], baseColor[2],
                         subsurface, metallic, specular, specularTint, roughness, anisotropic,
                         sheen, sheenTint, clearcoat, clearcoatGloss, IOR, transmission};
    std::memcpy(o, v, sizeof v);
  }
};

std::vector<float> transform(const float* trans, float scale) {
  const float rot[3] = {0, 0, 0}, sc[3] = {scale, scale, scale};
  std::vector<float> m(16);
  pts_transform_matrix(rot, trans, sc, m.data());
  return m;
}

Scene build_scene(const std::string& name, const std::string& assets, int hdr_w, int hdr_h, int leaves) {
  pts_scene* s = pts_scene_create();
  Material brass;
  brass.baseColor[0] = 0.80f; brass.baseColor[1] = 0.62f; brass.baseColor[2] = 0.35f;
  brass.metallic = 0.6f; brass.specular = 0.0f; brass.roughness = 0.35f; brass.clearcoat = 0.0f;
  brass.clearcoatGloss = 0.0f;
  float mb[18];
  brass.pack(mb);
  const std::string clock = assets + "/clock.obj", table = assets + "/table.obj";
  if (name == "clock") {
    const float t0[3] = {0, 0, 0};
    host_check(pts_scene_add_obj(s, clock.c_str(), mb, transform(t0, 1.0f).data(), 1, 0), "clock.obj");
  } else if (name == "table_clock_plant") {  // same placement as ptsvgf.scene.build_scene
    Material wood, leaf;
    wood.baseColor[0] = 0.45f; wood.baseColor[1] = 0.28f; wood.baseColor[2] = 0.14f;
    wood.roughness = 0.6f; wood.clearcoat = 0.5f; wood.clearcoatGloss = 0.8f;
    leaf.baseColor[0] = 0.16f; leaf.baseColor[1] = 0.42f; leaf.baseColor[2] = 0.12f;
    leaf.roughness = 0.7f; leaf.sheen = 0.3f;
    float mw[18], ml[18];
    wood.pack(mw);
    leaf.pack(ml);
    const float tt[3] = {0.176f, -0.73f, -0.16f}, tc[3] = {-0.914f, -0.155f, -1.03f}, tp[3] = {0.8f, -0.4f, -0.24f};
    host_check(pts_scene_add_obj(s, table.c_str(), mw, transform(tt, 3.84f).data(), 1, 0), "table.obj");
    host_check(pts_scene_add_obj(s, clock.c_str(), mb, transform(tc, 1.12f).data(), 1, 1), "clock.obj");
    int nv = 0, nt = 0;
    host_check(pts_gen_plant(0, leaves, &nv, &nt, nullptr, nullptr), "plant");
    std::vector<float> pos((size_t)nv * 3);
    std::vector<int> idx((size_t)nt * 3);
    host_check(pts_gen_plant(0, leaves, &nv, &nt, pos.data(), idx.data()), "plant");
    host_check(pts_scene_add_mesh(s, pos.data(), nullptr, nv, idx.data(), nt, ml, transform(tp, 1.28f).data(), 1, 2),
               "plant mesh");
  } else {
    std::fprintf(stderr, "unknown scene %s\n", name.c_str());
    std::exit(-1);
  }
  host_check(pts_scene_build_bvh(s, 8), "buildBVHwithSAH");
  int64_t c[6];
  pts_scene_counts(s, c);
  Scene sc;
  sc.ntris = (int)c[0];
  sc.nnodes = (int)c[1];
  sc.tri.resize((size_t)c[0] * 45);
  sc.node.resize((size_t)c[1] * 12);
  sc.raster.resize((size_t)c[5]);
  host_check(pts_scene_encode(s, sc.tri.data(), sc.node.data(), sc.raster.data()), "encode");
  pts_scene_destroy(s);
  // main.cpp:157-160
  sc.lights = {0.5f, 0.5f, 0.5f, 10, 10, 10, -0.5f, 0.75f, 0.5f, 8, 4, 4,
               -0.5f, 0.75f, 0.75f, 0, 3, 4, 0.75f, 0.75f, 0.75f, 12, 3, 4};
  sc.hdr_w = hdr_w;
  sc.hdr_h = hdr_h;
  sc.hdr.resize((size_t)hdr_w * hdr_h * 3);
  sc.cache.resize(sc.hdr.size());
  host_check(pts_gen_env_map(hdr_w, hdr_h, sc.hdr.data()), "env map");
  host_check(pts_hdr_cache(sc.hdr.data(), hdr_w, hdr_h, sc.cache.data()), "calculateHdrCache");
  return sc;
}

GLuint texture_buffer(const std::vector<float>& v) {  // glGenBuffers + glBufferData + glTexBuffer(RGB32F)
  uint32_t t = 0;
  pt_check(pt_texbuffer_create(v.data(), v.size() * sizeof(float), PT_RGB32F, &t), "glTexBuffer");
  return t;
}

RenderPass svgf_pass(const char* frag, std::vector<GLuint> atts, int W, int H) {
  RenderPass p;
  p.program = getShaderProgram(SHADERS + frag, SHADERS + "vert.vert");
  p.width = W;
  p.height = H;
  p.colorAttachments = std::move(atts);
  p.bindData(false);
  return p;
}

void write_plane(FILE* f, GLuint tex, int W, int H) {
  std::vector<float> buf((size_t)W * H * 4);
  pt_check(pt_texture_readback(tex, buf.data(), buf.size() * sizeof(float)), "readback");
  std::fwrite(buf.data(), sizeof(float), buf.size(), f);
}

}  // namespace

int main(int argc, char** argv) {
  int W = 800, H = 800, frames = 4, hdr_w = 2048, hdr_h = 1024, leaves = 150;
  float orbit = 0.0f;
  bool atrous_exact = false;
  std::string scene_name = "table_clock_plant", assets = "assets/models", out;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> std::string { return i + 1 < argc ? argv[++i] : ""; };
    if (a == "--width") W = std::atoi(next().c_str());
    else if (a == "--height") H = std::atoi(next().c_str());
    else if (a == "--frames") frames = std::atoi(next().c_str());
    else if (a == "--orbit") orbit = (float)std::atof(next().c_str());
    else if (a == "--scene") scene_name = next();
    else if (a == "--assets") assets = next();
    else if (a == "--leaves") leaves = std::atoi(next().c_str());
    else if (a == "--atrous-exact") atrous_exact = true;
    else if (a == "--out") out = next();
    else if (a == "--hdr") { std::string v = next(); std::sscanf(v.c_str(), "%dx%d", &hdr_w, &hdr_h); }
    else { std::fprintf(stderr, "unknown argument %s\n", a.c_str()); return 2; }
  }

  pt_check(pt_init(0), "pt_init");  // replaces the GLFW window + GL context (main.cpp:13-62)
  host::Camera camera(W, H);
  host::parameter_config config;
  Scene scene = build_scene(scene_name, assets, hdr_w, hdr_h, leaves);

  // scene buffers (main.cpp:136-181)
  GLuint trianglesTextureBuffer = texture_buffer(scene.tri);
  GLuint nodesTextureBuffer = texture_buffer(scene.node);
  GLuint pointLightBuffer = texture_buffer(scene.lights);
  GLuint hdrMap = getTextureRGB32F(scene.hdr_w, scene.hdr_h);
  pt_check(pt_texture2d_upload(hdrMap, scene.hdr_w, scene.hdr_h, PT_RGB32F, scene.hdr.data()), "hdrMap");
  GLuint hdrCache = getTextureRGB32F(scene.hdr_w, scene.hdr_h);
  pt_check(pt_texture2d_upload(hdrCache, scene.hdr_w, scene.hdr_h, PT_RGB32F, scene.cache.data()), "hdrCache");
  const int hdrResolution = scene.hdr_w;

  // G-buffer (main.cpp:208-226)
  GLuint init_world = getTextureRGB32F(W, H), init_normal_depth = getTextureRGB32F(W, H);
  GLuint init_velocity = getTextureRGB32F(W, H), init_fwidth = getTextureRGB32F(W, H);
  Rasterize_RenderPass init_pass;
  init_pass.program = getShaderProgram(SHADERS + "rasterize_frag.frag", SHADERS + "rasterize_vert.vert");
  init_pass.width = W;
  init_pass.height = H;
  init_pass.colorAttachments = {init_world, init_normal_depth, init_velocity, init_fwidth};
  init_pass.bindData(scene.raster);
  init_pass.set_uniform_int("screen_width", W);
  init_pass.set_uniform_int("screen_height", H);

  // path tracer (main.cpp:229-248)
  RenderPass pass_path_tracing;
  pass_path_tracing.program = getShaderProgram(SHADERS + "path_tracing.frag", SHADERS + "vert.vert");
  pass_path_tracing.width = W;
  pass_path_tracing.height = H;
  GLuint curColor = getTextureRGB32F(W, H), Emission = getTextureRGB32F(W, H), Albedo = getTextureRGB32F(W, H);
  pass_path_tracing.colorAttachments = {curColor, Emission, Albedo};
  pass_path_tracing.bindData(false);
  pass_path_tracing.set_uniform_int("nTriangles", scene.ntris);
  pass_path_tracing.set_uniform_int("nNodes", scene.nnodes);
  pass_path_tracing.set_uniform_int("width", W);
  pass_path_tracing.set_uniform_int("height", H);
  pass_path_tracing.set_uniform_int("pointLightSize", (int)(scene.lights.size() / 6));
  pass_path_tracing.set_uniform_int("aspect_corrected", W != H ? 1 : 0);  // SURVEY.md §7 hard part 4
  pass_path_tracing.set_uniform_int("prune", 1);

  // SVGF targets and passes (main.cpp:250-334)
  GLuint tmp_atrous_result = getTextureRGB32F(W, H);
  RenderPass bilt_pass = svgf_pass("bilt.frag", {tmp_atrous_result}, W, H);
  GLuint next_frame_color_input = getTextureRGB32F(W, H);
  RenderPass save_next_frame_pass = svgf_pass("bilt.frag", {next_frame_color_input}, W, H);
  GLuint taa_output = getTextureRGB32F(W, H);
  RenderPass pass_taa = svgf_pass("taa.frag", {taa_output}, W, H);
  pass_taa.set_uniform_int("screen_width", W);
  pass_taa.set_uniform_int("screen_height", H);
  GLuint curIllumination = getTextureRGB32F(W, H), curMomentHistory = getTextureRGB32F(W, H);
  RenderPass reproject_pass = svgf_pass("svgf_reproject.frag", {curIllumination, curMomentHistory}, W, H);
  GLuint variance_compute_illumination = getTextureRGB32F(W, H);
  RenderPass variance_compute_pass = svgf_pass("svgf_variance.frag", {variance_compute_illumination}, W, H);
  GLuint atrous_output = getTextureRGB32F(W, H);
  RenderPass atrous_pass = svgf_pass("svgf_Atrous.frag", {atrous_output}, W, H);
  GLuint modulate_color = getTextureRGB32F(W, H);
  RenderPass svgf_modulate_pass = svgf_pass("svgf_modulate.frag", {modulate_color}, W, H);
  GLuint lastIllumination = getTextureRGB32F(W, H), last_normal_depth = getTextureRGB32F(W, H);
  GLuint last_Moments_HistoryLength = getTextureRGB32F(W, H), last_acc_color = getTextureRGB32F(W, H);
  GLuint last_taa_color = getTextureRGB32F(W, H);
  RenderPass next_frame_input = svgf_pass("save_frame_data.frag", {lastIllumination, last_normal_depth,
                                           last_Moments_HistoryLength, last_acc_color, last_taa_color}, W, H);
  for (RenderPass* p : {&reproject_pass, &variance_compute_pass, &atrous_pass}) {
    p->set_uniform_float("inv_screen_width", 1.0f / W);
    p->set_uniform_float("inv_screen_height", 1.0f / H);
  }
  // output / tonemap (main.cpp:336-338), into a readable target instead of the default framebuffer
  GLuint output_tex = getTextureRGB32F(W, H);
  RenderPass output_pass;
  output_pass.program = getShaderProgram(SHADERS + "output_pass.frag", SHADERS + "vert.vert");
  output_pass.width = W;
  output_pass.height = H;
  output_pass.colorAttachments = {output_tex};
  output_pass.bindData(true);

  host::mat4 pre_viewproj = host::mul(camera.cam_proj_mat, camera.cam_view_mat);  // main.h:48
  FILE* fo = out.empty() ? nullptr : std::fopen(out.c_str(), "wb");
  if (!out.empty() && !fo) { std::fprintf(stderr, "cannot write %s\n", out.c_str()); return 1; }

  double total_ms = 0.0;
  for (int frame = 0; frame < frames; ++frame) {
    if (frame >= 2 && orbit != 0.0f) camera.orbit(orbit, 0.0f);  // scripted mouse drag
    const auto t0 = std::chrono::steady_clock::now();
    camera.update();
    const host::mat4& view = camera.cam_view_mat;
    const host::mat4& projection = camera.cam_proj_mat;
    init_pass.set_uniform_mat4("view", view.m);  // main.cpp:436-443
    init_pass.set_uniform_mat4("projection", projection.m);
    init_pass.set_uniform_mat4("pre_viewproj", pre_viewproj.m);
    init_pass.set_uniform_uint("frameCounter", camera.frameCounter);
    init_pass.draw();
    host::mat4 cameraRotate = host::rigid_inverse(view);  // main.cpp:445
    RenderPass& pt = pass_path_tracing;  // main.cpp:447-470
    pt.set_uniform_vec3("eye", camera.cam_position);
    pt.set_uniform_mat4("cameraRotate", cameraRotate.m);
    pt.set_uniform_uint("frameCounter", camera.frameCounter);
    pt.set_uniform_int("hdrResolution", hdrResolution);
    pt.set_uniform_bool("use_normal_map", config.use_normal_texture);
    pt.set_uniform_bool("accumulate", config.accumulate_color);
    pt.set_uniform_float("clamp_threshold", config.clamp_threshold);
    pt.set_uniform_int("max_tracing_depth", config.max_tracing_depth);
    pt.reset_texture_slot();
    pt.set_texture_uniform(GL_TEXTURE_BUFFER, trianglesTextureBuffer, "triangles");
    pt.set_texture_uniform(GL_TEXTURE_BUFFER, nodesTextureBuffer, "nodes");
    if (config.accumulate_color) pt.set_texture_uniform(GL_TEXTURE_2D, last_acc_color, "lastFrame");
    pt.set_texture_uniform(GL_TEXTURE_2D, hdrMap, "hdrMap");
    pt.set_texture_uniform(GL_TEXTURE_2D, hdrCache, "hdrCache");
    pt.set_texture_uniform(GL_TEXTURE_BUFFER, pointLightBuffer, "pointLights");
    pt.draw();
    RenderPass& rp = reproject_pass;  // main.cpp:474-486
    rp.reset_texture_slot();
    rp.set_uniform_float("depth_threshold", config.reproj_depth_threshold);
    rp.set_uniform_float("normal_threshold", config.reproj_normal_threshold);
    rp.set_texture_uniform(GL_TEXTURE_2D, init_velocity, "gMotion");
    rp.set_texture_uniform(GL_TEXTURE_2D, curColor, "gColor");
    rp.set_texture_uniform(GL_TEXTURE_2D, Albedo, "gAlbedo");
    rp.set_texture_uniform(GL_TEXTURE_2D, Emission, "gEmission");
    rp.set_texture_uniform(GL_TEXTURE_2D, lastIllumination, "gPrevIllum");
    rp.set_texture_uniform(GL_TEXTURE_2D, last_Moments_HistoryLength, "gPrevMoments_HistoryLength");
    rp.set_texture_uniform(GL_TEXTURE_2D, init_normal_depth, "gNormalAndLinearZ");
    rp.set_texture_uniform(GL_TEXTURE_2D, last_normal_depth, "gPrevNormalAndLinearZ");
    rp.set_texture_uniform(GL_TEXTURE_2D, init_fwidth, "gNormalDepthFwidth");
    rp.draw();
    RenderPass& vp = variance_compute_pass;  // main.cpp:488-495
    vp.reset_texture_slot();
    vp.set_uniform_float("gPhiColor", config.sigma_l);
    vp.set_uniform_float("gPhiNormal", config.sigma_n);
    vp.set_texture_uniform(GL_TEXTURE_2D, curIllumination, "gIllumination");
    vp.set_texture_uniform(GL_TEXTURE_2D, curMomentHistory, "gMoments_HistoryLength");
    vp.set_texture_uniform(GL_TEXTURE_2D, init_normal_depth, "gNormalAndLinearZ");
    vp.set_texture_uniform(GL_TEXTURE_2D, init_fwidth, "gNormalDepthFwidth");
    vp.draw();
    for (int i = 0; i < config.num_atrous_iterations; ++i) {  // main.cpp:499-526
      atrous_pass.reset_texture_slot();
      atrous_pass.set_uniform_float("gPhiColor", config.sigma_l);
      atrous_pass.set_uniform_float("gPhiNormal", config.sigma_n);
      atrous_pass.set_uniform_int("gStepSize", 1 << i);
      atrous_pass.set_uniform_int("exact", atrous_exact ? 1 : 0);
      atrous_pass.set_texture_uniform(GL_TEXTURE_2D, init_normal_depth, "gNormalAndLinearZ");
      atrous_pass.set_texture_uniform(GL_TEXTURE_2D, init_fwidth, "gNormalDepthFwidth");
      atrous_pass.set_texture_uniform(GL_TEXTURE_2D, i == 0 ? variance_compute_illumination : tmp_atrous_result,
                                      "gIllumination");
      atrous_pass.draw();
      bilt_pass.reset_texture_slot();
      bilt_pass.set_texture_uniform(GL_TEXTURE_2D, atrous_output, "in_texture");
      bilt_pass.draw();
      if (i == 1) {
        save_next_frame_pass.reset_texture_slot();
        save_next_frame_pass.set_texture_uniform(GL_TEXTURE_2D, atrous_output, "in_texture");
        save_next_frame_pass.draw();
      }
    }
    svgf_modulate_pass.reset_texture_slot();  // main.cpp:530-535
    svgf_modulate_pass.set_texture_uniform(GL_TEXTURE_2D, Albedo, "gAlbedo");
    svgf_modulate_pass.set_texture_uniform(GL_TEXTURE_2D, Emission, "gEmission");
    svgf_modulate_pass.set_texture_uniform(GL_TEXTURE_2D, atrous_output, "gIllumination");
    svgf_modulate_pass.set_texture_uniform(GL_TEXTURE_2D, init_normal_depth, "gNormalAndLinearZ");
    svgf_modulate_pass.draw();
    pass_taa.reset_texture_slot();  // main.cpp:537-544
    pass_taa.set_texture_uniform(GL_TEXTURE_2D, modulate_color, "currentColor");
    pass_taa.set_texture_uniform(GL_TEXTURE_2D, last_taa_color, "previousColor");
    pass_taa.set_texture_uniform(GL_TEXTURE_2D, init_velocity, "velocityTexture");
    pass_taa.set_texture_uniform(GL_TEXTURE_2D, init_normal_depth, "normal_depth");
    pass_taa.set_uniform_uint("frameCounter", camera.frameCounter);
    pass_taa.draw();
    next_frame_input.reset_texture_slot();  // main.cpp:546-553
    next_frame_input.set_texture_uniform(GL_TEXTURE_2D, next_frame_color_input, "texPass0");
    next_frame_input.set_texture_uniform(GL_TEXTURE_2D, init_normal_depth, "texPass1");
    next_frame_input.set_texture_uniform(GL_TEXTURE_2D, curMomentHistory, "texPass2");
    next_frame_input.set_texture_uniform(GL_TEXTURE_2D, curColor, "accColor");
    next_frame_input.set_texture_uniform(GL_TEXTURE_2D, taa_output, "taaOutput");
    next_frame_input.draw();
    output_pass.reset_texture_slot();  // main.cpp:556-590, final view
    output_pass.set_uniform_bool("accumulate", config.accumulate_color);
    output_pass.set_texture_uniform(GL_TEXTURE_2D, taa_output, "texPass0");
    output_pass.draw();
    pt_check(pt_sync(), "sync");
    total_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    pre_viewproj = host::mul(projection, view);  // main.cpp:599-600
    camera.frameCounter++;
    if (fo)
      for (GLuint t : {curColor, Albedo, modulate_color, taa_output, output_tex}) write_plane(fo, t, W, H);
  }
  if (fo) std::fclose(fo);
  std::printf("{\"frames\": %d, \"width\": %d, \"height\": %d, \"ms_per_frame\": %.3f, \"triangles\": %d}\n", frames, W,
              H, total_ms / frames, scene.ntris);
  pt_shutdown();
  return 0;
}

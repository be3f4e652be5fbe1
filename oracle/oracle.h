/* oracle.h — CPU oracle for the path-tracing + SVGF hot path.
 *
 * TEST INFRASTRUCTURE ONLY. Nothing in the product (path-tracing-svgf_amd/)
 * links, loads or calls this; only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg do, and only as the checker.
 *
 * What it is: a pixel-for-pixel C++ restatement of the reference's GLSL
 * fragment shaders (each function cites the shader file:line it follows),
 * evaluated with the GLSL built-ins of path-tracing-svgf_amd/csrc/glsl_builtins.h
 * (the GL built-in library both sides share; the shader logic is restated here
 * independently of the HIP kernels).
 *
 * Pinning status (see DESIGN.md "Parity"):
 *  - host scene prep (readObj, buildBVHwithSAH, encodings): PINNED against the
 *    reference's own known-answer counts.
 *  - GLSL passes: PARITY UNPINNED. The reference publishes no golden vectors or
 *    tests, and its GL path cannot run in this container (no GL context, no GLSL
 *    compiler, no glm — absence of tooling, not a denial). The restatement is
 *    checked against hand-derived known answers of its building blocks
 *    (tests/test_oracle_units.py) and against analytic invariants.
 *
 * Frame images are full frames, RGBA32F, row-major, row 0 = GL window row 0.
 */
#ifndef PTSVGF_ORACLE_H
#define PTSVGF_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_scene orc_scene;

/* Scene buffers exactly as main.cpp uploads them (main.cpp:136-181):
 * tri_enc: ntris*45 floats (Triangle_encoded), node_enc: nnodes*12 floats
 * (BVHNode_encoded, node 0 dummy), lights: nlights*6 floats (PointLight),
 * hdr_rgb / cache_rgb: hdr_w*hdr_h*3 floats. */
orc_scene* orc_scene_create(const float* tri_enc, int ntris, const float* node_enc, int nnodes, const float* lights,
                            int nlights, const float* hdr_rgb, const float* cache_rgb, int hdr_w, int hdr_h);
void orc_scene_destroy(orc_scene* s);
/* material_array (main.cpp:184-205): RGBA8 texels, layer-major, rows of w texels; row 0 = GL t = 0. */
int orc_scene_set_material_array(orc_scene* s, const uint8_t* rgba, int w, int h, int layers);

typedef struct {
  uint32_t frameCounter;
  int width, height;
  float eye[3];
  float cameraRotate[16]; /* column-major mat4 = inverse(view) */
  int accumulate;
  float clamp_threshold;
  int max_tracing_depth;
  int aspect_corrected; /* 0: reference (pix.x unscaled), 1: pix.x * width/height */
  int y_begin, y_end;   /* rows to compute */
  int use_normal_map;   /* uniform use_normal_map (path_tracing.frag:338) */
} orc_pt_params;

/* path_tracing.frag main() (path_tracing.frag:1056-1128) for rows [y_begin, y_end).
 * last_frame may be NULL when accumulate == 0. Outputs are full frames. */
int orc_path_trace(const orc_scene* s, const orc_pt_params* p, const float* last_frame, float* out_color,
                   float* out_emission, float* out_albedo, int threads);

/* Ray-cast G-buffer: the build's definition of rasterize_vert/rasterize_frag
 * (DESIGN.md "G-buffer"). raster_verts: pos3+nrm3 per vertex, 3 vertices/tri. */
int orc_gbuffer(const float* raster_verts, int ntris, int width, int height, const float* view16, const float* proj16,
                const float* pre_viewproj16, float* out_world, float* out_normal_depth, float* out_motion,
                float* out_fwidth, int threads);

int orc_reproject(int W, int H, const float* motion, const float* color, const float* albedo, const float* emission,
                  const float* prev_illum, const float* prev_moments, const float* normal_depth,
                  const float* prev_normal_depth, const float* fwidth, float inv_w, float inv_h, float depth_thr,
                  float normal_thr, float* out_illum, float* out_moments, int threads);

int orc_variance(int W, int H, const float* illum, const float* moments, const float* normal_depth,
                 const float* fwidth, float phi_color, float phi_normal, float inv_w, float inv_h, float* out,
                 int threads);

int orc_atrous(int W, int H, const float* illum, const float* normal_depth, const float* fwidth, int step,
               float phi_color, float phi_normal, float inv_w, float inv_h, float* out, int threads);

int orc_modulate(int W, int H, const float* albedo, const float* emission, const float* illum,
                 const float* normal_depth, float* out, int threads);

/* taa.frag:123-153 — history clip in YCoCg-R, velocity-weighted blend */
int orc_taa(int W, int H, const float* cur, const float* prev, const float* velocity, const float* normal_depth,
            uint32_t frameCounter, float* out, int threads);

/* output_pass.frag:18-24 — Reinhard-like tonemap (limit 1.5) + gamma 1/2.2 */
int orc_output(int W, int H, const float* color, float* out, int threads);

/* individual GLSL helpers, for unit tests */
uint32_t orc_wang_hash(uint32_t seed);
float orc_sobol(uint32_t d, uint32_t i);
void orc_brdf_eval(const float* V, const float* N, const float* L, const float* material14, float* out3);
float orc_brdf_pdf(const float* V, const float* N, const float* L, const float* material14);
float orc_hit_aabb(const float* S, const float* d, const float* AA, const float* BB);
/* hitTriangle: returns 1 on hit; out5 = (t, normal.xyz, isInside) */
int orc_hit_triangle(const float* S, const float* d, const float* tri9, const float* n9, float* out5);
void orc_math(int fn, const float* in, int n, float* out); /* 0 sin 1 cos 2 atan2(in,in+n) 3 asin 4 log 5 exp */

#ifdef __cplusplus
}
#endif
#endif

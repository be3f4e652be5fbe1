/* ptsvgf.h — the drop-in boundary: a C ABI into HIP that replaces the
 * reference's OpenGL plumbing API (layer L2) for the path-tracing + SVGF hot
 * path. A main.cpp-shaped host issues the SAME call sequence it issues against
 * the reference classes; each entry point names the reference interface it
 * replaces (file:line under the reference tree):
 *
 *   getShaderProgram(frag, vert)            Utils/shader.h:21-67    -> pt_program_create
 *   getTextureRGB32F(w, h)                  Utils/help_func.h:22-32 -> pt_texture2d_create
 *   glTexImage2D(... RGB32F ...)            main.cpp:173-180        -> pt_texture2d_upload
 *   glTexBuffer(GL_TEXTURE_BUFFER, RGB32F)  main.cpp:136-168        -> pt_texbuffer_create
 *   glTexStorage3D / glTexSubImage3D        main.cpp:184-205,
 *                                           Utils/help_func.h:4-20  -> pt_texarray_create / _upload_layer
 *   RenderPass{program,colorAttachments,width,height}
 *                                           Utils/render_pass.h:82-90 -> pt_pass_create / _add_color_attachment
 *   RenderPass::bindData(finalPass)         render_pass.h:92-119    -> pt_pass_bind
 *   RenderPass::draw()                      render_pass.h:120-140   -> pt_pass_draw
 *   RenderPass::reset_texture_slot()        render_pass.h:141-143   -> pt_pass_reset_texture_slot
 *   RenderPass::set_texture_uniform(t,tex,n) render_pass.h:144-150  -> pt_pass_set_texture
 *   RenderPass::set_uniform_{mat4,float,int,uint,bool,vec3}
 *                                           render_pass.h:152-180   -> pt_pass_set_uniform_*
 *   Rasterize_RenderPass::bindData(verts)   render_pass.h:19-62     -> pt_raster_pass_bind
 *   Rasterize_RenderPass::draw()            render_pass.h:64-79     -> pt_pass_draw
 *   glUniform*(glGetUniformLocation(...))   main.cpp:223-226,243-247,436-441 -> pt_pass_set_uniform_* (same)
 *   buildBVHwithSAH + node/triangle encode  Utils/BVH.h:42-173, main.cpp:88-151 -> pt_bvh_build (GPU, dynamic
 *                                           scenes: a different tree in the same buffer formats)
 *
 * Conventions:
 *  - handles are opaque uint32 owned by the library (0 is never a valid handle);
 *  - every function returns int status: PT_OK (0) or a negative PT_ERR_*;
 *    pt_last_error() gives the message. Where the reference calls exit(-1)
 *    (missing shader file, shader.h:8-12) this returns PT_ERR_FILE instead;
 *  - an unknown uniform name is silently ignored (GL location -1 semantics);
 *  - textures are RGBA32F, row-major, row 0 = GL window row 0 (bottom);
 *  - mat4 arguments are 16 floats column-major (glm::value_ptr order);
 *  - texture targets / formats keep their GL enum values so call sites port 1:1;
 *  - draws are asynchronous on the library stream (GL orders passes the same
 *    way); pt_sync() / pt_texture_readback() synchronise.
 *
 * MI355X extensions (no GL counterpart): pt_init (device + rank), pt_set_stream
 * (run on the caller's HIP stream, e.g. torch's), pt_texture2d_wrap (adopt
 * external device memory), pt_set_band (screen-band sharding across GPUs:
 * textures hold rows [row0, row0+rows) of the global frame).
 */
#ifndef PTSVGF_H
#define PTSVGF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PT_OK 0
#define PT_ERR_INVALID_HANDLE (-1)
#define PT_ERR_UNKNOWN_PROGRAM (-2)
#define PT_ERR_FILE (-3)
#define PT_ERR_MISSING_TEXTURE (-4)
#define PT_ERR_HIP (-5)
#define PT_ERR_ARG (-6)
#define PT_ERR_FORMAT (-7)
#define PT_ERR_NO_DEVICE (-8)
#define PT_ERR_STATE (-9)

/* GL enum values (texture targets and formats) */
#define PT_TEXTURE_2D 0x0DE1
#define PT_TEXTURE_BUFFER 0x8C2A
#define PT_TEXTURE_2D_ARRAY 0x8C1A
#define PT_RGB32F 0x8815
#define PT_RGBA32F 0x8814
#define PT_RGB 0x1907
#define PT_RGBA 0x1908

/* ---- library / device ---------------------------------------------------- */
int pt_init(int device);                    /* select HIP device, create stream */
int pt_shutdown(void);                      /* free every handle and the stream */
int pt_set_stream(void* hip_stream);        /* run on this stream; NULL = HIP default (null) stream */
int pt_use_own_stream(void);                /* back to the library's own stream (the pt_init default) */
/* The caller draws no more on this stream (it may be destroyed, or its handle
 * reused): the library drops its per-stream state (the trace_fork side stream,
 * the merged environment's reader event) once that state's work is done, and
 * falls back to its own stream if this one is current. No GL counterpart. */
int pt_stream_release(void* hip_stream);
/* A new stream whose kernels run only on the CUs whose bits are set in
 * mask[0..words) (hipExtStreamCreateWithCUMask; bit i of word w = CU 32 w + i),
 * e.g. to keep a set of CUs free of long traversal launches for a latency-bound
 * chain on another stream. Destroy with pt_stream_destroy. No GL counterpart. */
int pt_stream_create_cu_masked(uint32_t words, const uint32_t* mask, void** out);
/* A new non-blocking stream at queue priority `priority` (hipStreamCreateWithPriority;
 * numerically lower = higher, clamped into pt_stream_priority_range), e.g. to
 * put long traversal launches below a latency-bound chain. A trace_fork side
 * stream takes its draw stream's priority. Destroy with pt_stream_destroy. */
int pt_stream_create_priority(int priority, void** out);
int pt_stream_priority_range(int* least, int* greatest);
int pt_stream_destroy(void* hip_stream);   /* release (above), wait for its work, destroy */
/* Host-only check of the trees the library derives from a reference tree
 * (node_enc / tri_enc as pts_scene_encode writes them), built with 4-wide
 * collapse mode `collapse` (0..3, PTSVGF_WIDE_COLLAPSE) and `treelet` passes of
 * treelet restructuring (PTSVGF_TREELET). Needs no device and no pt_init.
 * out[0..PT_TREE_CHECK_COUNT): 1/0 every reference-leaf triangle is held by
 * exactly one leaf of the binary any-hit tree / the any-hit 4-wide tree / the
 * closest-hit 4-wide tree (and no other triangle); 1/0 every child box lies
 * inside its parent's box and every leaf box holds its triangles (boxes under a
 * reference leaf's own box excepted: its fine boxes only cull); SAH cost / root
 * area before and after the treelet passes; summed 4-wide node area / root area
 * of the any-hit and closest-hit trees; 4-wide nodes (both trees); binary depth;
 * 4-wide stack need; 1 when the closest-hit tree is a separate one.
 * No GL counterpart: the reference walks its own tree only. */
#define PT_TREE_CHECK_COUNT 12
int pt_tree_check(const float* node_enc, int nnodes, const float* tri_enc, int ntris, int collapse, int treelet,
                  double* out, int nout);
int pt_device_cus(int* n);                 /* compute units of the library's device */
int pt_sync(void);                          /* wait for all queued draws */
const char* pt_last_error(void);
int pt_version(void);

/* Band sharding: this rank renders global rows [y_begin, y_end) of a
 * frame_w x frame_h frame; every 2-D texture of exactly that size created
 * afterwards stores global rows [row0, row0 + rows) (band + ghost rows).
 * Default (never called): one band covering the frame. */
int pt_set_band(int frame_w, int frame_h, int y_begin, int y_end, int row0, int rows);
/* Record HIP events around every draw so pt_pass_last_ms can report it. */
int pt_set_profiling(int on);

/* ---- programs (getShaderProgram) ------------------------------------------- */
/* The fragment shader's basename selects the HIP kernel: path_tracing.frag,
 * svgf_reproject.frag, svgf_variance.frag, svgf_Atrous.frag, svgf_modulate.frag,
 * bilt.frag, save_frame_data.frag, output_pass.frag, taa.frag (full-screen,
 * vert.vert) and rasterize_frag.frag (rasterize_vert.vert). The shader files are
 * not read (the kernels are compiled in); an unknown basename or a mismatched
 * vertex stage returns PT_ERR_UNKNOWN_PROGRAM where the reference exit(-1)s. */
int pt_program_create(const char* frag_path, const char* vert_path, uint32_t* out_program);

/* ---- textures -------------------------------------------------------------- */
int pt_texture2d_create(int width, int height, uint32_t* out_tex);                 /* RGBA32F, zeroed */
int pt_texture2d_upload(uint32_t tex, int width, int height, uint32_t fmt,         /* PT_RGB32F | PT_RGBA32F */
                        const float* host_data);
int pt_texture2d_wrap(void* device_ptr, int width, int height, uint32_t* out_tex); /* RGBA32F, not owned;
    the library does not see writes to wrapped memory: a wrapped hdrMap / hdrCache whose contents change must be
    wrapped again (a new handle) for the path tracer's merged environment to be rebuilt */
int pt_texbuffer_create(const void* host_data, size_t bytes, uint32_t fmt, uint32_t* out_tex); /* RGB32F */
/* GPU BVH builder for dynamic scenes. The reference builds once on the host
 * (buildBVHwithSAH, Utils/BVH.h:42-173, main.cpp:88-96) and encodes triangles and nodes (main.cpp:101-151);
 * this builds a Karras LBVH on the device from the DEVICE contents of tri_in (Triangle_encoded texels, e.g.
 * after moving vertices through pt_texture_device_ptr) and writes, in those same formats, the triangles in leaf
 * order into tri_out and BVHNode_encoded nodes (dummy node 0, root node 1, leaves of <= leaf_n triangles) into
 * node_out. ploc_radius > 0 (e.g. 16) rebuilds the tree above the LBVH leaves by PLOC clustering with that search
 * radius (a surface-area-driven top, cheaper to walk); 0 keeps the plain LBVH. tri_out / node_out are existing
 * texbuffers (any size, e.g. created empty), distinct from tri_in and each other; their device and host copies are
 * replaced, so passes bound to them draw the new scene next time. leaf_n in [1, 15], ploc_radius in [0, 256].
 * out_nodes: node count (dummy included); out_ms: device time of the build (NULL: skipped).
 * Synchronous (waits for the build on the library stream). */
int pt_bvh_build(uint32_t tri_in, int leaf_n, int ploc_radius, uint32_t tri_out, uint32_t node_out, int* out_nodes,
                 float* out_ms);
int pt_texarray_create(int width, int height, int layers, uint32_t* out_tex);     /* RGBA8 2-D array */
int pt_texarray_upload_layer(uint32_t tex, int layer, int width, int height, int channels,
                             const uint8_t* host_data);
int pt_texture_readback(uint32_t tex, float* host_out, size_t bytes);             /* syncs the device */
int pt_texture_upload_rgba(uint32_t tex, const float* host_rgba, size_t bytes);   /* raw RGBA32F rows */
int pt_texture_device_ptr(uint32_t tex, void** out_ptr);
int pt_texture_info(uint32_t tex, int* width, int* height, int* row0);
int pt_texture_destroy(uint32_t tex);

/* ---- passes (RenderPass / Rasterize_RenderPass) ---------------------------- */
int pt_pass_create(uint32_t program, int width, int height, uint32_t* out_pass);
int pt_pass_add_color_attachment(uint32_t pass, uint32_t tex);
int pt_pass_bind(uint32_t pass, int final_pass);
int pt_raster_pass_bind(uint32_t pass, const float* vertices, size_t n_floats);   /* pos3+nrm3 per vertex */
/* Dynamic scenes: pt_raster_pass_bind from a DEVICE vertex list (same layout), its G-buffer tree built by the GPU
 * builder (LBVH, PLOC top with ploc_radius > 0) and its records decoded on the device; the G-buffer does not depend
 * on the tree (closest t, ties to the lower original index), so the planes equal the host bind's bit for bit. */
int pt_raster_pass_bind_device(uint32_t pass, const void* device_vertices, size_t n_floats, int ploc_radius);
/* A rasterize pass drawing another (bound) rasterize pass's triangles and tree: the reference has one G-buffer pass;
 * a driver with several G-buffer targets (frames in flight) binds one and shares it. Rebinding `pass` ends the share;
 * destroying `src_pass` first makes `pass`'s draws fail with PT_ERR_STATE. */
int pt_raster_pass_share(uint32_t pass, uint32_t src_pass);
/* The G-buffer planes of a rasterize pass's attachments were written elsewhere for rows [y_begin, y_end) (multi-GPU:
 * another rank drew these rows of the same frame and sent them; the G-buffer is per pixel, so they equal a draw's):
 * derive what a draw makes beside its planes (the a-trous's compact depth-fwidth plane and per-tile surface flags,
 * "atrous_rows_begin" / "_end" as for a draw) on the current stream. No reference counterpart. */
int pt_raster_pass_adopt(uint32_t pass, int y_begin, int y_end);
/* Tile shard (multi-GPU, no GL counterpart): a path-tracing pass with "tile_stride" = S and "tile_offset" = o draws the
 * 16 x 16 tiles t = k * S + o of its rows, numbered row-major from its first row (tile_y0) with frame_w / 16 tiles per
 * row. pt_tiles_copy moves the pixels of such subsets between textures (RGBA32F, the same width, a multiple of 16) and
 * packed device buffers, one segment per (rows, subset, buffer): unpack = 0 writes the segment's packed block from the
 * textures, 1 writes the textures from it. A block holds, for each texture in order, each row of [y_begin, y_end) in
 * order, each row's subset tiles in x order: pt_tiles_count(...) pixels per texture (16 B each). Asynchronous on the
 * library stream; segment rows must lie in every texture's stored rows. */
typedef struct {
  int y_begin, y_end, offset;
  void* packed;
} PtTileSeg;
int pt_tiles_count(int frame_w, int tile_y0, int stride, int offset, int y_begin, int y_end, int64_t* out_pixels);
int pt_tiles_copy(const uint32_t* tex, int ntex, int tile_y0, int stride, const PtTileSeg* segs, int nseg, int unpack);
int pt_pass_reset_texture_slot(uint32_t pass);
int pt_pass_set_texture(uint32_t pass, uint32_t target, uint32_t tex, const char* name);
int pt_pass_set_uniform_mat4(uint32_t pass, const char* name, const float* m16);
int pt_pass_set_uniform_float(uint32_t pass, const char* name, float v);
int pt_pass_set_uniform_int(uint32_t pass, const char* name, int v);
int pt_pass_set_uniform_uint(uint32_t pass, const char* name, uint32_t v);
int pt_pass_set_uniform_bool(uint32_t pass, const char* name, int v);
int pt_pass_set_uniform_vec3(uint32_t pass, const char* name, const float* v3);
/* Rows this pass computes (global coords); default = the band. The G-buffer
 * pass uses it to compute ghost rows locally for multi-GPU halos. */
int pt_pass_set_rows(uint32_t pass, int y_begin, int y_end);
/* Load-balancing probe (path-tracing pass, wavefront kernel): while set, every
 * draw ADDS the BVH node + triangle visits of each pixel's rays into
 * device_counts[row - y_begin] (uint32 per computed row; caller zeroes it).
 * NULL disables. No reference counterpart (multi-GPU band planning). */
int pt_pass_set_row_cost(uint32_t pass, void* device_counts);
/* Motion bound (G-buffer pass): while set, every draw first zeroes *device_u32 and
 * then stores there the largest |motion.y| (UV units, the bits of a non-negative
 * float; +inf for a non-finite motion) over the surface pixels it computes. The
 * multi-GPU band renderer sizes its reprojection / TAA history exchange from it
 * (svgf_reproject.frag:45-156 reads the history at uv - motion). NULL disables.
 * No reference counterpart (the single-GPU reference reads the whole frame). */
int pt_pass_set_motion_bound(uint32_t pass, void* device_u32);
/* Traversal counters (path-tracing pass, wavefront kernel): while set, every
 * draw ADDS to device_u64[0..13] (caller zeroes): primary rays, primary node +
 * triangle visits, bounce rays, bounce visits, shadow rays, shadow visits,
 * exact-tie re-walks on the reference tree, primary rays retried unbounded after
 * the G-buffer bound, rays whose stack spilled past the LDS stack (reference
 * trees deeper than 32 levels), the lane slots of primary / bounce / shadow
 * waves (64 x the wave's largest visit count), and, counted from the shadow
 * verdicts, the shadow rays toward point lights and the occluded shadow rays.
 * device_u64 holds `count` counters: counters past count are not written
 * (pt_trace_stats_count() = how many this library has; count above it is
 * capped, count <= 0 with a buffer is PT_ERR_ARG).
 * Wave-aggregated atomics; NULL disables (the default). */
int pt_pass_set_trace_stats_n(uint32_t pass, void* device_u64, int count);
/* The first form of the call: a buffer of PT_TRACE_STATS_V1 (12) counters,
 * the first 12 above; the two shadow-split counters are not written. */
#define PT_TRACE_STATS_V1 12
int pt_pass_set_trace_stats(uint32_t pass, void* device_u64);
/* Number of traversal counters this library writes (14). */
int pt_trace_stats_count(void);
int pt_pass_draw(uint32_t pass);
/* Draw `count` (1..8) path-tracing passes — the frames of a batch, each with its
 * own uniforms, samplers and attachments, one scene, size and band — as one
 * wavefront run whose list-driven traversal launches trace every frame's rays at
 * once (no GL counterpart: the reference draws one frame at a time). Results are
 * those of drawing each pass alone. passes[0] owns the shared wavefront state,
 * sized for max(count, its "trace_batch" uniform) frames; the batch is timed as
 * its draw. Accumulation (lastFrame) is refused; tile subsets are batched when every pass traces the same one
 * ("tile_stride" / "tile_offset"). */
int pt_pass_draw_batch(const uint32_t* passes, int count);
/* Time the last draw of this pass (ms, HIP events on the library stream; syncs). */
int pt_pass_last_ms(uint32_t pass, float* ms);
int pt_pass_destroy(uint32_t pass);

#ifdef __cplusplus
}
#endif
#endif

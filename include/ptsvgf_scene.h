/* ptsvgf_scene.h — host-side scene preparation (layer L1 of the reference).
 *
 * C ABI over plain pointers and sizes. Each entry point restates one reference
 * host routine so a main.cpp-shaped driver (or the Python harness) produces the
 * exact buffers the reference uploads to its GL texture buffers:
 *
 *   pts_scene_add_obj        <- readObj            Utils/obj_loader.h:5-163
 *   pts_transform_matrix     <- getTransformMatrix Utils/obj_loader.h:166-182
 *   pts_scene_build_bvh      <- buildBVHwithSAH    Utils/BVH.h:42-173 (+ dummy node 0, main.cpp:88-96)
 *   pts_scene_encode         <- Triangle_encoded / BVHNode_encoded loops, main.cpp:101-133
 *   pts_hdr_cache            <- calculateHdrCache  Utils/hdr_compute.h:5-102
 *
 * plus deterministic synthetic stand-ins for the assets the reference lists as
 * missing (.MISSING_LARGE_BLOBS: plant.obj, teapot.obj, room.hdr):
 *   pts_scene_add_mesh, pts_gen_plant, pts_gen_teapot, pts_gen_cornell, pts_gen_env_map.
 *
 * Return convention: 0 = success, negative = error (see pts_last_error()).
 */
#ifndef PTSVGF_SCENE_H
#define PTSVGF_SCENE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Material — Utils/Material.h:8-22, as 18 floats in this order:
 * emissive[3], baseColor[3], subsurface, metallic, specular, specularTint,
 * roughness, anisotropic, sheen, sheenTint, clearcoat, clearcoatGloss, IOR, transmission.
 * A negative baseColor/metallic/roughness selects the texture-array layer
 * (path_tracing.frag:331-364), exactly as in the reference. */
#define PTS_MATERIAL_FLOATS 18
/* Triangle_encoded (Utils/Triangle.h:12-24): 15 x vec3 = 45 floats = 180 B. */
#define PTS_TRI_ENCODED_FLOATS 45
/* BVHNode_encoded (Utils/BVH.h:18-22): 4 x vec3 = 12 floats = 48 B. */
#define PTS_NODE_ENCODED_FLOATS 12
/* Raster vertex list entry (obj_loader.h:143-160): pos3 + nrm3 per vertex. */
#define PTS_RASTER_FLOATS_PER_TRI 18

typedef struct pts_scene pts_scene;

pts_scene* pts_scene_create(void);
void pts_scene_destroy(pts_scene* s);

/* readObj(filepath, verticesout, triangles, material, trans, smoothNormal, objIndex).
 * trans: column-major mat4 (glm::value_ptr order). */
int pts_scene_add_obj(pts_scene* s, const char* path, const float* material18, const float* trans16,
                      int smooth_normal, int obj_index);

/* Add an indexed mesh WITHOUT readObj's size normalisation (synthetic content).
 * positions: n_verts*3 floats; uvs: n_verts*2 floats or NULL; indices: n_tris*3.
 * trans16 applied with glm's mat4*vec4 evaluation order; normals as readObj. */
int pts_scene_add_mesh(pts_scene* s, const float* positions, const float* uvs, int n_verts, const int* indices,
                       int n_tris, const float* material18, const float* trans16, int smooth_normal, int obj_index);

/* Add raw triangles (p1,n1,p2,n2,p3,n3 = 18 floats each, the raster vertex list
 * layout) without normal recomputation. obj_index < 0: each triangle's objIndex
 * is its running index in this call (used to keep original order through the
 * BVH sort). */
int pts_scene_add_raw(pts_scene* s, const float* verts18, int n_tris, const float* material18, int obj_index);

/* buildBVHwithSAH(triangles, nodes{dummy}, 0, N-1, leaf_n); reorders triangles. */
int pts_scene_build_bvh(pts_scene* s, int leaf_n);

/* counts: [0]=triangles [1]=nodes (incl. dummy 0) [2]=leaves [3]=max depth (root=0)
 *         [4]=max leaf size [5]=raster floats */
int pts_scene_counts(const pts_scene* s, int64_t* out6);
/* Root AABB (node 1): out6 = AA.xyz, BB.xyz */
int pts_scene_root_aabb(const pts_scene* s, float* out6);

/* Encoded buffers exactly as uploaded by main.cpp:136-151 / obj_loader raster list.
 * Any output pointer may be NULL. Sizes: tris*45, nodes*12, raster floats. */
int pts_scene_encode(const pts_scene* s, float* tri_out, float* node_out, float* raster_out);

/* glm::mat4 getTransformMatrix(rotateCtrl(deg), translateCtrl, scaleCtrl) -> out16 column-major */
void pts_transform_matrix(const float* rot3_deg, const float* trans3, const float* scale3, float* out16);

/* calculateHdrCache(HDR, width, height): hdr RGB32F rows (w*h*3) -> cache RGB32F (w*h*3):
 * R = sample x, G = sample y, B = pdf (hdr_compute.h:88-99). */
int pts_hdr_cache(const float* hdr_rgb, int width, int height, float* cache_out);

/* HDRLoader::load (lib/hdrloader.cpp:28-97): Radiance RGBE file -> RGB32F rows, file scanline order (the
 * first scanline in the file is row 0, as the reference stores it), components (v / 256) * 2^(E - 128).
 * Call with rgb_out == NULL to get the size, then with a w*h*3 buffer. Differences, all on malformed input
 * only: the resolution is read into long and narrowed (the reference's "%ld" into int is undefined on LP64,
 * hdrloader.cpp:68), run lengths are bounds-checked, and a truncated file is an error instead of a
 * partially uninitialised image. */
int pts_load_hdr(const char* path, int* width, int* height, float* rgb_out);

/* ------------------------------------------------ synthetic stand-ins ---- */
/* Seeded procedural potted plant (stand-in for models/plant.obj): writes
 * positions/indices into caller buffers when non-NULL; returns counts. */
int pts_gen_plant(uint32_t seed, int leaves, int* n_verts, int* n_tris, float* positions, int* indices);
/* Procedural teapot-like body of revolution + spout + handle (stand-in for teapot.obj). */
int pts_gen_teapot(int segments, int* n_verts, int* n_tris, float* positions, int* indices);
/* Cornell-style box: 5 axis-aligned quads (floor, ceiling, back, left, right), extent [-1,1]^3. */
int pts_gen_cornell(int* n_verts, int* n_tris, float* positions, int* indices);
/* Synthetic equirect "room.hdr" stand-in: RGB32F rows (width x height), sky gradient
 * + ground + one Gaussian sun lobe, deterministic (GLSL built-in restatement). */
int pts_gen_env_map(int width, int height, float* rgb_out);

const char* pts_last_error(void);

#ifdef __cplusplus
}
#endif
#endif

// pt_device.h — parameter blocks and HBM layouts shared by the C-ABI layer
// (capi.hip) and the kernels. Everything here is plain data; no torch types.
//
// HBM layout (DESIGN.md "Data layout"):
//  * frame planes: RGBA32F (float4) row-major, one plane per GL texture, holding
//    global rows [row0, row0+rows) of a W x H frame (row0 = 0, rows = H on 1 GPU);
//  * optional compact side plane `aux` (float, 4 B/px) next to a plane whose only
//    consumer-visible channel is .y (the depth fwidth of gNormalDepthFwidth):
//    written by the G-buffer kernel, read by the a-trous kernel instead of the
//    16-B texel (52 B/px/iteration instead of 64). Its magnitude is .y (always
//    >= 0, or a NaN with the sign clear); its SIGN BIT flags zCenter == 1 (the
//    pixel's gNormalAndLinearZ.w, background sentinel), so the a-trous skips
//    reading the normal/depth texel of pixels it only copies;
//  * scene: tri_geom  4 x float4 / triangle  (p1,N.p1)(p2,-)(p3,-)(N,-)  intersection
//           tri_shade 9 x float4 / triangle  normals, material, uv, objIndex  closest hit only
//           bvh       4 x float4 / interior node: both children's AABBs + child refs
//    (children refs >= 0: interior index; < 0: leaf = -(first*16 + count) - 1);
//           bvh4      7 x float4 / node: the 4-wide collapse for any-hit (shadow) rays,
//                     lo.x[4] hi.x[4] lo.y[4] hi.y[4] lo.z[4] hi.z[4] refs[4];
//  * HDR map / importance cache: float4 per texel (RGB32F padded), row-major.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#else
struct float4 {
  float x, y, z, w;
};
struct int2 {
  int x, y;
};
#endif

namespace ptk {

#ifndef PT_KSTACK
#define PT_KSTACK 32
#endif
// float4s per node of the 4-wide tree (pack_wide): 7 hold the four child boxes and refs. PT_WIDE_STRIDE = 8 pads a
// node to one 128-B cache line (at 7, 112-B nodes straddle two lines for most indices): measured SLOWER, 211.5 ->
// 202.6 fps at 4K and 69.2 -> 62.9 on the surface view (three alternating repetitions, profiles/r04/wide_stride_ab.log).
#ifndef PT_WIDE_STRIDE
#define PT_WIDE_STRIDE 7
#endif
constexpr int kWideStride = PT_WIDE_STRIDE;
// PT_WIDE_ORDER = 1 (default): pack_wide stores a node's largest child first, i.e. right after the node, where the
// node's own fetch already brings most of it into L1 (capi.hip). Same box, three alternating repetitions
// (profiles/r04/wide_order_ab.log): 4K 210.6 / 212.2 / 210.4 -> 213.0 / 214.2 / 213.0 fps, surface view
// 68.6 / 68.9 / 68.5 -> 69.7 / 69.7 / 69.7.
#ifndef PT_WIDE_ORDER
#define PT_WIDE_ORDER 1
#endif
// PT_WIDE_SIGNED = 1 (default since round 5): the 4-wide walks pick each child's near / far planes by the ray's
// direction signs (which float4 is loaded) instead of slab's 6 min / max per child (pt_shading.h wide_step): 99 -> 92
// VALU per shadow node step in the ISA. Same bits. With the traversal kernels at 7 waves per SIMD (kernels_wavefront.hip
// PT_TRACE_WAVES_PER_EU), same box, two alternating repetitions (profiles/r05/wide_signed/): 4K 222.5 / 222.4 ->
// 225.3 / 225.2 fps, surface view 73.9 / 74.0 -> 78.1 / 78.0 (at 8 waves it spills 40-44 B per lane: 223.0, 77.1;
// at 6: 223.0, 76.6)
#ifndef PT_WIDE_SIGNED
#define PT_WIDE_SIGNED 1
#endif
constexpr int kStack = PT_KSTACK;  // traversal stack depth (host checks BVH depth < kStack)
// Traversal counters: a node visit counts PT_NODE_VISIT (1; a diagnostic build with 0 counts triangle tests only)
#ifndef PT_NODE_VISIT
#define PT_NODE_VISIT 1
#endif
constexpr int kStackSmall = 24;    // smaller LDS stack (more resident waves) for trees that fit it
// LDS entries of the spilling traversal stack (SpillStack): a tree deeper than this walks kSpillKS entries in LDS and
// the rest in global memory. Default kStack (spill only beyond the 32-entry stack); PT_SPILL_KS < kStackSmall trades
// rare global spills for more resident waves (A/B).
#ifndef PT_SPILL_KS
#define PT_SPILL_KS PT_KSTACK
#endif
constexpr int kSpillKS = PT_SPILL_KS;
constexpr int kBlock = 256;      // threads per block for per-pixel kernels
constexpr int kNoneRef = (int)0x80000000;
constexpr int kPointBins = 4;     // point-light shadow lists, one per light index mod 4 (coherent waves)
constexpr int kLiveBins = 1;  // live-ray lists (by direction octant, 8 of them, measured 4 % slower: one list)
// wavefront list counters per bounce (8 segments each): live bins, HDR shadow, point bins, straggler count
constexpr int kCtrHdr = 8 * kLiveBins, kCtrPoint = kCtrHdr + 8, kCtrStrag = kCtrPoint + 8 * kPointBins;
// per-XCD work-queue heads of the refill traversal kernels launched in bounce i: shadow rays, closest-hit rays
constexpr int kCtrQShadow = kCtrStrag + 1, kCtrQClosest = kCtrQShadow + 8, kCtrStragC = kCtrQClosest + 8;
constexpr int kWfCtr = (kCtrStragC + 1 + 63) / 64 * 64;
constexpr int kWfCounters = 4 * kWfCtr;  // 4 bounces  // "no node" (leaf refs are >= -(2^31 - 1))

struct Plane {          // banded RGBA32F plane
  float4* p;
  const float* aux;     // optional compact channel (see above), may be null
  int W;                // row width (pixels)
  int row0;             // global row of local row 0
  int rows;             // allocated rows
};

// Cost-ordered dispatch of a tiled traversal launch (kernels_sched.hip). The
// slowest waves of a traversal launch (rays through dense geometry: ~1000 node and
// triangle visits at ~0.7 us each) set its tail; started last in raster order they
// finish long after the bulk. Each launch records every tile's slowest wave and the
// next launch dispatches tiles in descending order of that cost, so the long waves
// start first and overlap the bulk. Dispatch order only: results are unchanged.
struct TileSched {
  const int* perm;      // launch slot -> tile index, may be null (raster order)
  int* perm_next;       // where the order from this launch's costs is written (the same buffer as perm)
  uint32_t* cost;       // per tile: max traversal steps of its waves in this launch, may be null
  int ntiles;
};

struct Tex {            // non-banded float4 image (HDR map / cache)
  const float4* p;
  int W, H;
};

struct SceneDev {
  const float4* tri_geom;
  const float4* tri_shade;
  const float4* bvh;
  int root_ref;         // >= 0 interior node index, < 0 leaf ref
  const float4* bvh4;   // 4-wide collapse of bvh for any-hit rays (7 x float4 / node), may be null
  int root4;
  int root4c;           // root of the closest-hit walks' 4-wide tree in bvh4 (= root4 unless PTSVGF_WIDE_COLLAPSE 2 / 3)
  const float4* bvh_any;  // binary any-hit tree over bvh's leaves (capi.hip build_anyhit_tree), may be null
  int root_any;
  int ntris;
  const float* lights;  // 6 floats per light (PointLight: position, radiance)
  int nlights_buf;      // lights actually present in the buffer
  // material_array (main.cpp:184-205): RGBA8 2-D array, layer-major rows of tex_w texels, may be null
  const uint32_t* texarr;
  int tex_w, tex_h, tex_layers;
  int use_normal_map;   // uniform use_normal_map (path_tracing.frag:338)
  // the reference tree's leaves (2 x float4 each: (box lo, leaf ref bits), (box hi, -)): the primary-ray tile
  // rasteriser's items (wf_primary_raster)
  const float4* leaves;
  int nleaves;
};

// Wavefront path-tracer state (kernels_wavefront.hip): SoA per band pixel.
struct WFState {
  float4 *ray_o, *ray_d;        // current ray (origin, direction)
  float4 *light, *red;          // radiance accumulator, path throughput ("reduction")
  float4 *pend0, *pend1, *pend2, *pend3;  // NEE terms awaiting the shadow verdicts
  float4 *sh_h, *sh_p;          // shadow directions (HDR; point light + distance in .w)
  int2* hit;                    // closest hit (triangle, t bits)
  uint32_t* seed;               // RNG state (path_tracing.frag:433)
  uint8_t *occ_h, *occ_p;       // shadow verdicts
  int *list0, *list1;           // compacted live-ray lists (ping-pong), kLiveBins bins of kSeg segments of `cap`
  int* shadow_list;             // compacted shadow rays of one bounce: HDR list, then kPointBins point-light
                                // lists (by light index), each kSeg segments of `cap`
  int* counters;                // per bounce i, base kWfCtr*i: [0, kCtrHdr) live-bin segment counts, then 8 HDR,
                                // 8 kPointBins point-light counts, [kCtrStrag] cooperative-walk stragglers,
                                // 8 + 8 work-queue heads (kCtrQShadow, kCtrQClosest)
  uint32_t* row_cost;           // optional: traversal steps per band row (load-balancing probe), may be null
  int* straggler;               // shadow rays past the step budget: pid | (point << 31), count at kCtrStrag
  uint32_t shadow_budget;       // node + triangle visits before a shadow ray is handed to the cooperative walk (0: never)
  int* strag_c;                 // bounce rays past closest_budget (count at kCtrStragC): the cooperative closest walk
  uint32_t closest_budget;      // node + triangle visits before a bounce ray is handed to it (0: never; refill kernel)
  unsigned long long* stats;    // optional traversal counters (kStat*), wave-aggregated atomics; may be null
  int stats_n;                  // counters the caller's buffer holds: counter k is written only when k < stats_n
  int* spill;                   // deep trees only: stack entries past the LDS stack, entry kStack + j of pixel pid at
  size_t spill_stride;          // spill[j * spill_stride + pid] (spill_stride = band pixels); null otherwise
};
// Traversal counters of one path-tracing draw (pt_pass_set_trace_stats): rays traced and node + triangle visits
// per traversal kind, tie re-walks on the reference tree, primary rays retried unbounded after the G-buffer bound, rays
// whose stack went past the LDS stack into the spill columns (deep reference trees), and per traversal kind the lane
// slots its waves occupied (64 x the wave's largest visit count, summed over waves): visits / slots is the share of
// SIMD lanes doing useful traversal work (divergence: a wave runs as long as its longest ray); of the shadow rays
// (lane-refill walks), those toward point lights and those found occluded.
enum { kStatPrimRays, kStatPrimVisits, kStatBounceRays, kStatBounceVisits, kStatShadowRays, kStatShadowVisits,
       kStatTieRewalks, kStatPrimRetries, kStatSpills, kStatPrimSlots, kStatBounceSlots, kStatShadowSlots,
       kStatShadowPoint, kStatShadowOccluded, kStatCount };

// A path-tracing draw over several frames' pixels (pt_pass_draw_batch): frame b's pixels are the pids
// [b * n, (b + 1) * n) of one shared per-pixel wavefront state; its lists hold frame-local pids. The list-driven
// traversal kernels take every frame's list of a bounce at once, so one launch traces the whole batch's rays.
constexpr int kMaxBatch = 8;
struct ListBatch {
  int nb;               // frames
  int n;                // pixels per frame (the pid offset of frame b is b * n)
  const int* list[kMaxBatch];
  const int* counts[kMaxBatch];
};

// Screen-tile binning of items (the G-buffer's triangles, the path tracer's BVH leaves) for the tile rasterisers:
// an item-specific setup kernel writes each item's pixel box and counts it into the 16 x 16 tiles of the band it
// covers (bins_count_item); launch_bins then bins the large items, scans and scatters (kernels_pt.hip).
constexpr int kRTile = 16;
constexpr int kLargeTiles = 8;   // items covering more tiles are binned by a whole block
constexpr int kBoxMargin = 2;    // pixels added around a projected box (projection vs ray arithmetic)
struct Bins {
  int n;                // items
  int4* box;            // per item: pixel box (x0, y0, x1, y1) of the pixels whose ray it can meet; empty: x0 > x1
  float* tmin;          // per item: lower bound of the ray parameter of any hit (0 when unknown)
  int* tile_count;      // per tile of the band: items binned to it; the scatter counts it back to zero
  int* tile_off;        // ntiles + 1: exclusive scan of tile_count
  int* pairs;           // item indices grouped by tile
  int pair_cap;
  int* large;           // items whose box covers more than kLargeTiles tiles (binned by whole blocks)
  int large_cap;
  int* ctr;             // [0] large items, [1] binned pairs, [2] overflow (the caller's fallback then runs)
  int W, y0, y1;        // band: tiles counted from row y0
};

struct PTParams {
  int W, H, y0, y1;     // frame size (global) and rows to compute
  Plane color, emission, albedo, last;  // outputs (+ lastFrame input)
  SceneDev scene;
  Tex hdr, cache;
  // hdrMap's radiance (.xyz) and hdrCache's pdf (.z) of each texel in one float4 (capi.hip hdr_merged), when both
  // textures have one size: the NEE's hdr_color + hdr_pdf at one direction then read one texture (null: two)
  Tex hdr_pdf;
  int hdrResolution;
  int pointLightSize;
  uint32_t frameCounter;
  float eye[3];
  float camRot[16];     // column-major inverse(view)
  int accumulate;
  float clamp_threshold;
  int max_depth;
  int aspect_corrected;
  int prune;            // closest-hit pruning (parity-safe margin)
  int closest_tree;     // closest-hit rays walk the SAH tree over the reference leaves (closest_hit, pt_shading.h)
  int stack_need;       // deepest interior level of the binary BVH (selects the LDS stack size)
  int refill;           // > 0: percent of each bounce/shadow list traced by lane-refill waves (kernels_wavefront.hip)
  int refill_waves;     // resident waves a refill launch is sized for (0: the whole chip, kResidentWaves)
  int refill_grid;      // most blocks of a refill launch (uniform refill_grid; 0: PTSVGF_REFILL_GRID / its default)
  int list_grid;        // most blocks of the list-driven shade / finish (uniform list_grid; 0: PTSVGF_LIST_BLOCKS)
  float sobol_u[4], sobol_v[4];  // sobolVec2(frameCounter+1, b): uniform across pixels
  WFState wf;
  // optional bound for the primary rays from this frame's G-buffer (world position + normal/linearZ planes,
  // drawn before on the same stream): see wf_primary. p == null: no bound
  Plane hint_pos, hint_nd;
  TileSched tiles;      // primary-ray tiles (16 x 16 px), indexed by subset slot (below)
  // Tile subset (wavefront path tracer only): trace the 16 x 16 tiles t = k * tile_stride + tile_offset of
  // the band (raster tile order), k = 0 .. tiles.ntiles - 1; other pixels are left untouched. Stride 1,
  // offset 0 = every tile. Interleaved subsets give every rank of a multi-GPU frame an equal share of the
  // expensive tiles (ptsvgf.dist, DESIGN.md "Multi-GPU").
  int tile_stride, tile_offset;
  // primary rays by tile rasterisation of the reference leaves (wf_primary_raster; primary_raster uniform): the
  // bins, and for the wf_primary launch that follows it the bins' counters (pr_fix non-null: that launch walks
  // only the pixels the rasteriser flagged — exact-t ties — or every pixel after a list overflow)
  Bins leaf_bins;
  int primary_raster;
  const int* pr_fix;
};

struct GBufParams {
  int W, H, y0, y1;
  Plane world, normal_depth, motion, fwidth;
  float* fwidth_aux;    // compact depth-fwidth plane (rows of fwidth), may be null
  unsigned char* tflags;  // a-trous per-tile surface flags (atrous_mark_tiles) of rows [tf_y0, tf_y1), may be null
  int tf_off[5];          // their per-step offsets (atrous_flag_offset)
  int tf_y0, tf_y1;       // the rows the a-trous passes draw (default: the G-buffer's own rows)
  const float4* geom;   // 4 x float4 per raster triangle (walk): (p1,idx)(e1,-)(e2,-)(Ng,-)
  const float4* nrm;    // 3 x float4 per raster triangle (closest hit only): n1, n2, n3
  const float4* bvh;
  int root_ref;
  int stack_need;       // deepest interior level of the raster BVH
  float eye[3];
  float invR[9];        // row-major R^T (camera-to-world rotation)
  float P00, P11;       // projection diagonal (pixel ray scale)
  float M[16];          // projection * view (column-major)
  float PV[16];         // pre_viewproj
  TileSched tiles;      // 16 x 16 px tiles
  uint32_t* motion_max; // optional: max |motion.y| (float bits) over the launch's surface pixels, zeroed by the host
  Bins bins;            // tile-binned rasterisation (gbuffer_mode 1): items = the raster triangles; bins.ctr null
                        // when the ray cast runs alone
};

struct ReprojParams {
  int W, H, y0, y1;
  Plane motion, color, albedo, emission, prev_illum, prev_moments, nd, prev_nd, fwidth;
  Plane out_illum, out_moments;
  float inv_w, inv_h, depth_thr, normal_thr;
  int block;  // 1: the four history taps from one 3x3 texel block per plane when they tile it (same texels, same bits)
};

struct VarianceParams {
  int W, H, y0, y1;
  Plane illum, moments, nd, fwidth, out;
  float phi_color, phi_normal;
};

struct AtrousParams {
  int W, H, y0, y1;
  Plane illum, nd, fwidth, out;
  int step;
  float phi_color, phi_normal;
  const unsigned char* tile_any;  // tiled kernel: per-tile "holds a surface pixel" flags of this step, or null
  // fused modulate (the last iteration of a frame, fast driver): mod.p != null writes modulate_kernel's output of
  // this draw's rows from `out`'s values, albedo and emission (every plane must store the draw's rows)
  Plane albedo, emission, mod;
};
// Tiles of the tiled a-trous (kernels_atrous.hip): 64 * NX columns x TJ rows of one residue class mod S, one wave
// per 64-column strip of a tile row (64 * TJ * NX <= 1024 threads); tile (g, b, bx) of step S has byte
// (g * S + b) * NXT + bx in that step's flags. The staged footprint is (TJ + 4) x (64 NX + 4S) texels for TJ x 64 NX
// pixels. PT_ATROUS_TJ (rows for S <= 8) / PT_ATROUS_TJ16, PT_ATROUS_NX16 (S = 16) choose the shape (A/B).
#ifndef PT_ATROUS_TJ
#define PT_ATROUS_TJ 8
#endif
#ifndef PT_ATROUS_TJ16
#define PT_ATROUS_TJ16 8
#endif
#ifndef PT_ATROUS_NX16
#define PT_ATROUS_NX16 2
#endif
__host__ __device__ constexpr int atrous_tile_tj(int S) { return S >= 16 ? PT_ATROUS_TJ16 : PT_ATROUS_TJ; }
__host__ __device__ constexpr int atrous_tile_nx(int S) { return S >= 16 ? PT_ATROUS_NX16 : 1; }
static_assert(64 * PT_ATROUS_TJ <= 1024 && 64 * PT_ATROUS_TJ16 * PT_ATROUS_NX16 <= 1024, "a-trous tile too large");
__device__ __forceinline__ void atrous_mark_tiles(unsigned char* flags, const int* off, int W, int x, int r) {
#pragma unroll
  for (int si = 0; si < 5; ++si) {
    const int S = 1 << si, nx = atrous_tile_nx(S), nxt = (W + 64 * nx - 1) / (64 * nx);
    const int g = r / (S * atrous_tile_tj(S)), b = r % S;
    flags[off[si] + (size_t)(g * S + b) * nxt + x / (64 * nx)] = 1;
  }
}
// per-tile surface flags of the tiled a-trous for the 5 steps (1, 2, 4, 8, 16) of rows [y0, y1), from the
// depth-fwidth plane's sign bits: atrous_flag_bytes() bytes, step si's flags at atrous_flag_offset(si)
size_t atrous_flag_bytes(int W, int y0, int y1);
size_t atrous_flag_offset(int si, int W, int y0, int y1);
int atrous_tile_flags(const Plane& fwidth, int W, int y0, int y1, unsigned char* flags, hipStream_t s);

struct ModulateParams {
  int W, H, y0, y1;
  Plane albedo, emission, illum, nd, out;
};

struct OutputParams {
  int W, H, y0, y1;
  Plane in, out;
};

struct TAAParams {
  int W, H, y0, y1;
  Plane cur, prev, vel, nd, out;
  uint32_t frameCounter;
};

// Tile-shard transfer (kernels_shard.hip): the pixels of the 16 x 16 tile subset (t = k * stride + seg.offset, tiles
// numbered row-major from row tile_y0, W / 16 per row) in rows [seg.y0, seg.y1) of each plane, to (unpack = 0) or from
// (1) the segment's packed block: plane-major, rows in order, each row's subset tiles in x order.
constexpr int kShardSegs = 16;
struct ShardSeg {
  int y0, y1, offset;
  float4* packed;
};
struct ShardCopy {
  int W, tile_y0, stride, nseg, nplanes, unpack;
  float4* plane[4];
  int row0[4];
  ShardSeg seg[kShardSegs];
};

}  // namespace ptk

#if defined(__HIPCC__)
namespace ptk {
// Launchers (kernels_*.hip). Return hipError_t as int.
int launch_shard_copy(const ShardCopy& c, hipStream_t s);
long long shard_pixels(int W, int tile_y0, int stride, int offset, int y0, int y1);  // per plane
int launch_pathtrace(const PTParams& p, hipStream_t s);
// A side stream for the wavefront's bounce-0 shadow rays: they and the bounce-1 closest-hit rays both come from the
// bounce-0 shade and touch disjoint buffers, so the two walks run at once and fill each other's launch tails.
// `fork` is recorded on the draw's stream after that shade, `join` on the side stream after the bounce-0 finish.
struct WfFork {
  hipStream_t side;
  hipEvent_t fork, join;
};
int launch_pathtrace_wavefront(const PTParams& p, hipStream_t s, const WfFork* fk = nullptr);
// 1 when the walk kernels' translation unit keeps f32 subnormals (max(0, least subnormal) > 0, evaluated on the device
// with the walk code's compile flags), as PT_WIDE_SIGNED's one-compare child test needs; 0 if it flushes; < 0 a HIP error
int subnormal_probe(hipStream_t s);
int wf_list_capacity(int W, int rows);  // per-segment capacity of the compacted ray lists (8 segments)
int wf_subset_tiles(int W, int rows, int stride, int offset);  // tiles of a PTParams tile subset (< 0: invalid)
int launch_gbuffer(const GBufParams& p, hipStream_t s);
int launch_gbuffer_raster(const GBufParams& p, hipStream_t s);
int launch_gbuffer_adopt(const GBufParams& p, hipStream_t s);  // side data of G-buffer planes written elsewhere  // bins, resolves, and the ray cast on overflow
int launch_bins(const Bins& b, hipStream_t s);  // after the item setup kernel: large items, scan, scatter
// nb frames' path tracing with batched traversal launches (ps[b]: frame b, its wavefront state at pid offset b * n)
int launch_pathtrace_wavefront_batch(const PTParams* ps, int nb, hipStream_t s, const WfFork* fk = nullptr);
int launch_reproject(const ReprojParams& p, hipStream_t s);
int launch_variance(const VarianceParams& p, hipStream_t s);
int launch_atrous_exact(const AtrousParams& p, hipStream_t s);
int launch_atrous_fast(const AtrousParams& p, hipStream_t s);   // LDS-tiled (production)
int launch_atrous_step(const AtrousParams& p, hipStream_t s);   // step-specialised, texture-path taps
int launch_atrous_simple(const AtrousParams& p, hipStream_t s);
int launch_modulate(const ModulateParams& p, hipStream_t s);
// the modulate an a-trous draw with AtrousParams::mod set asks for, as its own launch (kernels that do not fuse it)
int launch_modulate_after(const AtrousParams& p, hipStream_t s);
int launch_output(const OutputParams& p, hipStream_t s);
int launch_taa(const TAAParams& p, hipStream_t s);
int launch_tile_sort(uint32_t* cost, int* perm, int ntiles, hipStream_t s);  // cost -> perm, clears cost
int launch_hdr_merge(const float4* hdr, const float4* cache, float4* out, int n, hipStream_t s);  // (hdr.xyz, cache.z)
}  // namespace ptk

namespace ptk {
// The tree shadow (any-hit) rays walk: bvh_any when present (same verdicts), else the reference tree.
__device__ __forceinline__ SceneDev anyhit_scene(const SceneDev& s) {
  SceneDev r = s;
  if (s.bvh_any) {
    r.bvh = s.bvh_any;
    r.root_ref = s.root_any;
  }
  return r;
}
__device__ __forceinline__ int sched_tile(const TileSched& t, int slot) { return t.perm ? t.perm[slot] : slot; }

struct TileBox {
  int tx0, tx1, ty0, ty1;
  __device__ int area() const { return (tx1 - tx0 + 1) * (ty1 - ty0 + 1); }
};
__device__ __forceinline__ TileBox tile_box(const Bins& b, int4 box) {
  return TileBox{box.x / kRTile, box.z / kRTile, (box.y - b.y0) / kRTile, (box.w - b.y0) / kRTile};
}
// Pixel box of projected extents (pixel coordinates of the centre rays), widened by kBoxMargin, clipped to the band.
__device__ __forceinline__ int4 pixel_box(const Bins& b, float x0, float y0, float x1, float y1) {
  const float lim = 1.0e8f;  // keeps the float -> int conversion in range
  const int bx0 = (int)floorf(fmaxf(x0, -lim)) - kBoxMargin, bx1 = (int)ceilf(fminf(x1, lim)) + kBoxMargin;
  const int by0 = (int)floorf(fmaxf(y0, -lim)) - kBoxMargin, by1 = (int)ceilf(fminf(y1, lim)) + kBoxMargin;
  return make_int4(max(bx0, 0), max(by0, b.y0), min(bx1, b.W - 1), min(by1, b.y1 - 1));
}
// Sutherland-Hodgman against s * w + sgn * c[axis] >= 0 (homogeneous coordinates: x, y, w)
__device__ __forceinline__ int clip_plane(const float3* in, int n, float3* out, int axis, float sgn) {
  const float s = 1.01f;
  int m = 0;
  for (int i = 0; i < n; ++i) {
    const float3 a = in[i], b = in[(i + 1) % n];
    const float da = s * a.z + sgn * (axis == 0 ? a.x : a.y), db = s * b.z + sgn * (axis == 0 ? b.x : b.y);
    if (da >= 0.0f) out[m++] = a;
    if ((da >= 0.0f) != (db >= 0.0f)) {
      const float t = da / (da - db);
      out[m++] = make_float3(a.x + t * (b.x - a.x), a.y + t * (b.y - a.y), a.z + t * (b.z - a.z));
    }
  }
  return m;
}

// Screen box and nearest-t bound of a convex polygon given by n <= 8 vertices (x, y, w) in a frame whose centre
// rays have NDC ((2x+1)/W - 1, (2y+1)/H - 1) scaled by (sx, sy): clipped to the widened frustum first.
// Returns false when nothing of it lies in front of the camera inside the frustum.
__device__ __forceinline__ bool poly_box(const Bins& b, int H, float3* A, int n, float sx, float sy, int4* box,
                                         float* tmin) {
  float3 B[16];
  n = clip_plane(A, n, B, 0, 1.0f);
  n = clip_plane(B, n, A, 0, -1.0f);
  n = clip_plane(A, n, B, 1, 1.0f);
  n = clip_plane(B, n, A, 1, -1.0f);
  if (n <= 0) return false;
  float x0 = 3.0e38f, y0 = 3.0e38f, x1 = -3.0e38f, y1 = -3.0e38f, wmin = 3.0e38f;
  for (int k = 0; k < n; ++k) {
    if (!(A[k].z > 0.0f)) {  // on the camera plane: the whole band, no bound
      *box = make_int4(0, b.y0, b.W - 1, b.y1 - 1);
      *tmin = 0.0f;
      return true;
    }
    wmin = fminf(wmin, A[k].z);
    // pixel coordinate whose centre ray has this NDC: ndc = (2 x + 1) / W - 1
    const float px = ((A[k].x / (A[k].z * sx) + 1.0f) * (float)b.W - 1.0f) * 0.5f;
    const float py = ((A[k].y / (A[k].z * sy) + 1.0f) * (float)H - 1.0f) * 0.5f;
    if (!(px == px && py == py)) {
      *box = make_int4(0, b.y0, b.W - 1, b.y1 - 1);
      *tmin = 0.0f;
      return true;
    }
    x0 = fminf(x0, px); x1 = fmaxf(x1, px);
    y0 = fminf(y0, py); y1 = fmaxf(y1, py);
  }
  *box = pixel_box(b, x0, y0, x1, y1);
  *tmin = wmin;
  return true;
}

// Records item i's box and bound and counts it into its tiles (small items) or queues it (large ones).
__device__ __forceinline__ void bins_count_item(const Bins& b, int i, int4 box, float tmin) {
  b.box[i] = box;
  b.tmin[i] = tmin;
  if (box.x > box.z || box.y > box.w) return;
  const TileBox tb = tile_box(b, box);
  if (tb.area() > kLargeTiles) {
    const int slot = atomicAdd(&b.ctr[0], 1);
    if (slot < b.large_cap) b.large[slot] = i;
    else atomicOr(&b.ctr[2], 1);
    return;
  }
  const int ntx = (b.W + kRTile - 1) / kRTile;
  for (int ty = tb.ty0; ty <= tb.ty1; ++ty)
    for (int tx = tb.tx0; tx <= tb.tx1; ++tx) atomicAdd(&b.tile_count[ty * ntx + tx], 1);
}
// Call with every lane of the wave active (steps = 0 for lanes without a ray).
__device__ __forceinline__ void sched_cost(const TileSched& t, int tile, uint32_t steps) {
  if (!t.cost) return;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) steps = max(steps, (uint32_t)__shfl_xor((int)steps, o));
  if ((threadIdx.x & 63) == 0 && steps) atomicMax(t.cost + tile, steps);
}
// GPU LBVH builder (kernels_bvh.hip): Triangle_encoded texels in, triangles in leaf order + BVHNode_encoded
// nodes out (the reference's upload formats, main.cpp:101-151). Scratch grows on demand and is reused.
struct LbvhWork {
  void* base = nullptr;
  size_t bytes = 0;
  static size_t need(int n);
};
// Triangle_encoded texels (device) -> tri_geom (4 float4) / tri_shade (9 float4) records, as get_scene decodes them
int decode_tris(const float* te, int n, float4* geom, float4* shade, hipStream_t s);
// Raster vertex list (18 floats per triangle) -> the G-buffer's geom (4 float4) / nrm (3 float4) records in the
// given leaf order (order[k] = original triangle index), as pt_raster_pass_bind builds them on the host
int decode_raster(const float* verts, const int* order, int n, float4* geom, float4* nrm, hipStream_t s);
// Where a triangle record keeps its vertices: p1 at 0, p2 at o2, p3 at o3, records `stride` floats apart.
struct TriLayout {
  int stride, o2, o3;
};
constexpr TriLayout kTriEncoded{45, 3, 6};   // Triangle_encoded (Utils/Triangle.h:12-24)
constexpr TriLayout kRasterVerts{18, 6, 12};  // the raster vertex list (obj_loader.h:143-160)
// node_out needs room for 2n nodes (12 floats each); *nnodes = nodes written (dummy node 0 included).
// ploc_r > 0: the tree above the LBVH leaves is rebuilt by PLOC with search radius ploc_r. tri_out (45-float
// records only) may be null; order (may be null) receives the original index of each leaf-order position.
int lbvh_build(LbvhWork& w, const float* tri, TriLayout lay, int n, int leaf_n, int ploc_r, float* tri_out,
               float* node_out, int* order, int* nnodes, hipStream_t s);

}  // namespace ptk
#endif

// kernels_wavefront.hip — the production path tracer: path_tracing.frag's main()
// (:1056-1128) split into stages so that BVH traversal runs in small,
// high-occupancy kernels and shading runs without a traversal stack:
//
//   per bounce i:  trace_closest -> shade -> trace_shadow (HDR + point light) -> finish
//   then          finalize (clamp / NaN / accumulate / store)
//
// Rays that stay alive are compacted into a list with one wave-ballot atomic per
// wave, so traversal waves carry only live rays (58 % of the 4K frame is sky).
// The arithmetic per pixel is exactly the megakernel's (and the reference's):
// shade() evaluates both light contributions as if unoccluded, finish() applies
// the shadow verdicts with the reference's selection (hdriLight :934-937 zeroes
// pdf and value; calculatePointLight :905-909 zeroes the value only), so outputs
// stay bit-identical to the CPU oracle. RNG consumption order per pixel is
// unchanged: AA x2, then per bounce xi_3, r1, r2, light pick.
#include <hip/hip_runtime.h>

#include "glsl_builtins.h"
#include "pt_device.h"
#include "pt_shading.h"

using namespace glsl;

namespace ptk {

#ifndef PT_WIDE_SHADOW_SORT
#define PT_WIDE_SHADOW_SORT 0  // shadow rays' 4-wide walk: 1 = nearest child first, 0 = slot order
#endif
constexpr int kTB = 128;  // threads per traversal block (LDS stack: kStack*kTB*4 = 16 KiB)
// Resident waves per SIMD the traversal kernels are compiled for. Round 3 (SLP vectorizer on): 98 VGPRs left alone,
// 96 at 5 waves (4K 179.8 -> 185.8 fps, profiles/r03/occupancy_ab.log). With SLP off the 4-wide refill walks need
// 63-67 VGPRs; 8 waves fits them in 64 without spills, which pays once the LDS stack allows 8 waves (PT_WIDE_KS 16:
// 8 KiB per 2-wave block). Round 4, same box, two alternating repetitions (profiles/r04/occupancy_ab.log): default
// 24 entries / 5 waves 210.8 / 210.5 fps at 4K, 68.5 / 68.6 surface view; 16 / 5 waves 212.2 / 211.7, 68.9 / 68.6;
// 16 / 8 waves 214.7 / 212.3, 69.4 / 69.0; 12 / 8 waves 199.9 / 198.3, 59.9 / 59.2 (more rays overflow to the
// cooperative walk). Round 5: the sign-selected planes of the 4-wide step (PT_WIDE_SIGNED) need a few more VGPRs; at
// 8 waves they spill 40-44 B per lane, at 7 (72 VGPRs) 8-12 B outside the walk loop: 7 kept (pt_device.h PT_WIDE_SIGNED,
// profiles/r05/wide_signed/).
#ifndef PT_TRACE_WAVES_PER_EU
#define PT_TRACE_WAVES_PER_EU 7
#endif
#if PT_TRACE_WAVES_PER_EU > 0
#define PT_TRACE_ATTR __attribute__((amdgpu_waves_per_eu(PT_TRACE_WAVES_PER_EU)))
#else
#define PT_TRACE_ATTR
#endif

// LDS stack entries of the 4-wide lane-refill walks. Unlike the binary walks (sized by the tree's depth: kStack /
// kStackSmall), a 4-wide walk whose pushes would overflow hands its ray to the cooperative walk (wide_step), so the
// stack can be smaller than the deepest path: it bounds the resident waves (kTB x entries x 4 B of LDS per block).
// Re-measured at 7 waves per SIMD (round 5, profiles/r05/wide_ks/): 20 and 22 entries (both still 7 waves: 10 / 11 KB
// per 2-wave block) within noise of 16 at 4K and on the surface view.
#ifndef PT_WIDE_KS
#define PT_WIDE_KS 16
#endif
constexpr int kWideKS = PT_WIDE_KS;

__device__ __forceinline__ void pix_xy(const PTParams& p, int pid, int* x, int* y) {
  *x = pid % p.W;
  *y = p.y0 + pid / p.W;
}

// ---------------------------------------------------------- ray lists ---
// Compacted ray lists are split into kSeg segments, one per XCD group of
// blocks (blockIdx % kSeg), each with its own counter: a producer block makes
// ONE atomic per list (block-aggregated through LDS), and the 8 counters spread
// those atomics over 8 addresses (one word saturates near 90 atomics/us,
// MI355X_MICROARCH.md "dequeue"). Consumers map a dense index onto the
// segments with the 8 counts (scalar loads).
constexpr int kSeg = 8;

__device__ __forceinline__ int seg_total(const int* __restrict__ counts) {
  int t = 0;
#pragma unroll
  for (int s = 0; s < kSeg; ++s) t += counts[s];
  return t;
}
// A list of `nbins` bins (bin b: items + b * kSeg * cap, counts + b * kSeg), read as one dense range.
__device__ __forceinline__ bool bins_get(const int* __restrict__ items, const int* __restrict__ counts, int nbins,
                                         int cap, int k, int* v) {
  int base = 0;
  for (int b = 0; b < nbins; ++b) {
#pragma unroll
    for (int s = 0; s < kSeg; ++s) {
      const int c = counts[b * kSeg + s];
      if (k < base + c) {
        *v = items[((size_t)b * kSeg + s) * cap + (k - base)];
        return true;
      }
      base += c;
    }
  }
  return false;
}
__device__ __forceinline__ bool seg_get(const int* __restrict__ items, const int* __restrict__ counts, int cap, int k,
                                        int* v) {
  int base = 0;
#pragma unroll
  for (int s = 0; s < kSeg; ++s) {
    const int c = counts[s];
    if (k < base + c) {
      *v = items[s * cap + (k - base)];
      return true;
    }
    base += c;
  }
  return false;
}

// Block-wide append of up to one item to each of the shade lists: the live rays into kLiveBins lists by
// direction octant, the HDR shadow rays, and the point-light shadow rays into kPointBins lists by light index
// (rays of one bin traverse alike, so a trace wave holding one bin diverges less). Every thread of the
// 256-thread block must call it. One atomic per (list, bin) per block.
constexpr int kLists = kLiveBins + 1 + kPointBins;
__device__ __forceinline__ void block_push_shade(bool p_live, int lbin, bool p_h, bool p_p, int bin, int v,
                                                 int* __restrict__ live, int* live_counts, int* __restrict__ shadow,
                                                 int* shadow_counts, int cap, int chunk) {
  __shared__ int wc[kLists][4];
  __shared__ int base[kLists];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  unsigned long long m[kLists];
#pragma unroll
  for (int b = 0; b < kLiveBins; ++b) m[b] = __ballot(p_live && lbin == b);
  m[kLiveBins] = __ballot(p_h);
#pragma unroll
  for (int b = 0; b < kPointBins; ++b) m[kLiveBins + 1 + b] = __ballot(p_p && bin == b);
  if (lane == 0)
#pragma unroll
    for (int l = 0; l < kLists; ++l) wc[l][wv] = __popcll(m[l]);
  __syncthreads();
  const int seg = chunk % kSeg;  // the chunk's segment (wf_list_capacity: at most 256 items per chunk)
  if (threadIdx.x < kLists) {
    const int l = threadIdx.x;
    const int t = (wc[l][0] + wc[l][1]) + (wc[l][2] + wc[l][3]);
    int* c = l < kLiveBins ? live_counts + l * kSeg : shadow_counts + (l - kLiveBins) * kSeg;
    base[l] = t ? atomicAdd(c + seg, t) : 0;
  }
  __syncthreads();
  const unsigned long long lt = (1ull << lane) - 1ull;
  // this lane's masks by constant indices and selects: a per-lane index into m[] put it in scratch (or LDS) memory
  unsigned long long mlive = m[0], mpoint = m[kLiveBins + 1];
#pragma unroll
  for (int j = 1; j < kLiveBins; ++j) mlive = lbin == j ? m[j] : mlive;
#pragma unroll
  for (int j = 1; j < kPointBins; ++j) mpoint = bin == j ? m[kLiveBins + 1 + j] : mpoint;
  if (p_live) {
    int o = base[lbin];
    for (int w = 0; w < wv; ++w) o += wc[lbin][w];
    live[((size_t)lbin * kSeg + seg) * cap + o + __popcll(mlive & lt)] = v;
  }
  if (p_h) {
    int o = base[kLiveBins];
    for (int w = 0; w < wv; ++w) o += wc[kLiveBins][w];
    shadow[seg * cap + o + __popcll(m[kLiveBins] & lt)] = v;
  }
  if (p_p) {
    const int li = kLiveBins + 1 + bin;
    int o = base[li];
    for (int w = 0; w < wv; ++w) o += wc[li][w];
    shadow[(size_t)(1 + bin) * kSeg * cap + seg * cap + o + __popcll(mpoint & lt)] = v;
  }
}

// PT_WIDE_SIGNED's child test (wide_step) takes t1 > 0 as t1 >= the least f32 subnormal: compiled with this file's
// flags, max(x, least subnormal) must stay above 0 for x = 0 (x comes from memory, so nothing folds at compile time)
__global__ void __launch_bounds__(64) subnormal_probe_kernel(const float* zero, int* out) {
  if (threadIdx.x == 0) out[0] = fmaxf(zero[0], __builtin_bit_cast(float, 1u)) > 0.0f ? 1 : 0;
}
int subnormal_probe(hipStream_t s) {
  void* buf = nullptr;
  if (hipMalloc(&buf, 8) != hipSuccess) return -1;
  int host = -1;
  bool ok = hipMemsetAsync(buf, 0, 8, s) == hipSuccess;
  if (ok) hipLaunchKernelGGL(subnormal_probe_kernel, dim3(1), dim3(64), 0, s, (const float*)buf, (int*)buf + 1);
  ok = ok && hipGetLastError() == hipSuccess &&
       hipMemcpyAsync(&host, (int*)buf + 1, sizeof(int), hipMemcpyDeviceToHost, s) == hipSuccess &&
       hipStreamSynchronize(s) == hipSuccess;
  (void)hipFree(buf);
  return ok ? host : -1;
}

// traversal counters (PTParams::wf.stats, pt_pass_set_trace_stats): a wave sum, one 64-bit atomic per wave.
// Call with every lane of the wave active.
__device__ __forceinline__ void stat_add(const PTParams& p, int k, uint32_t v) {
  if (!p.wf.stats || k >= p.wf.stats_n) return;  // (a buffer of fewer counters: those past its end are skipped)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
  if ((threadIdx.x & 63) == 0 && v) atomicAdd(p.wf.stats + k, (unsigned long long)v);
}

__device__ __forceinline__ void stat_slots(const PTParams& p, int k, uint32_t v) {  // 64 x the wave maximum
  if (!p.wf.stats || k >= p.wf.stats_n) return;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
  if ((threadIdx.x & 63) == 0 && v) atomicAdd(p.wf.stats + k, 64ull * v);
}

// load-balancing probe: accumulate traversal steps per band row (only when requested)
#ifndef PT_STEP_MAX
__device__ __forceinline__ void add_row_cost(const PTParams& p, int local_row, int, uint32_t steps) {
  if (p.wf.row_cost) atomicAdd(p.wf.row_cost + local_row, steps);
}
#else  // investigation build (tools/exp_build.sh stepmax -DPT_STEP_MAX): per-pixel maximum of the steps
__device__ __forceinline__ void add_row_cost(const PTParams& p, int, int pid, uint32_t steps) {
  if (p.wf.row_cost) atomicMax(p.wf.row_cost + pid, steps);
}
#endif

// This lane's traversal stack: its LDS column, and with DEEP (a reference tree deeper than the LDS stack, launched
// only for such trees) the pixel's spill column for the entries beyond it.
template <int STRIDE, int KS, bool DEEP>
__device__ __forceinline__ auto ray_stack(int* lds_column, const PTParams& p, int pid) {
  if constexpr (DEEP) return SpillStack<STRIDE, KS>{lds_column, p.wf.spill + pid, p.wf.spill_stride};
  else return LdsStack<STRIDE>{lds_column};
}


__device__ __forceinline__ v3 primary_dir(const PTParams& p, int x, int y) {
  float pixx = (float)(2 * x + 1) / (float)p.W - 1.0f;
  float pixy = (float)(2 * y + 1) / (float)p.H - 1.0f;
  if (p.aspect_corrected) pixx = pixx * ((float)p.W / (float)p.H);
  const float* m = p.camRot;
  return normalize(mk((m[0] * pixx + m[4] * pixy) + (m[8] * -1.0f + m[12] * 0.0f),
                      (m[1] * pixx + m[5] * pixy) + (m[9] * -1.0f + m[13] * 0.0f),
                      (m[2] * pixx + m[6] * pixy) + (m[10] * -1.0f + m[14] * 0.0f)));
}

// ------------------------------------------------------------ primaries ---
constexpr int kTieFix = -2;  // hit.x of a pixel wf_primary_raster leaves to the walk (two triangles share its t)

// 16x16 screen tiles, each wave an 8x8 sub-tile: coherent camera rays.
// nslots: the subset's tiles; a block walks slots blockIdx.x, + gridDim.x, ... (launched with one slot per block)
template <int KS, bool DEEP>
__global__ void __launch_bounds__(256) PT_TRACE_ATTR wf_primary(PTParams p, int nslots) {
  __shared__ int stk[KS * 256];
  for (int slot = blockIdx.x; slot < nslots; slot += gridDim.x) {
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  const int tile = sched_tile(p.tiles, slot);  // cost-ordered dispatch (subset slot)
  const int gt = tile * p.tile_stride + p.tile_offset, ntx = (p.W + 15) / 16;
  const int tx = gt % ntx, ty = gt / ntx;
  const int x = tx * 16 + (wv & 1) * 8 + (ln & 7);
  const int y = p.y0 + ty * 16 + (wv >> 1) * 8 + (ln >> 3);
  bool valid = x < p.W && y < p.y1;
  const int pid = (y - p.y0) * p.W + x;
  bool count_ray = true;
  if (p.pr_fix) {  // after wf_primary_raster: walk only the pixels it flagged, or all of them after an overflow
    if (p.pr_fix[2]) {
      // the skipped scatter did not count the tiles back to zero: the block of subset slot `tile` clears the tiles of
      // its stride group (the last slot also the band's tail), so every band tile is cleared once
      if (threadIdx.x == 0) {
        const int all = ntx * ((p.y1 - p.y0 + 15) / 16), lo = tile * p.tile_stride;
        const int hi = tile + 1 == nslots ? all : min(all, lo + p.tile_stride);
        for (int j = lo; j < hi; ++j) p.leaf_bins.tile_count[j] = 0;
      }
    } else {
      if (p.closest_tree) return;  // the flagged pixels went to wf_primary_coop
      valid = valid && ldnt(&p.wf.hit[pid]).x == kTieFix;
      if (!__any(valid)) continue;
      count_ray = false;  // counted by the rasteriser
    }
  }
  uint32_t steps = 0;
  bool rewalk = false, retry = false, spill = false;
  if (valid) {
    v3 S = mk(p.eye[0], p.eye[1], p.eye[2]);
    v3 d = primary_dir(p, x, y);
    // Bound from the G-buffer: the surface this pixel rasterised lies at distance |P - eye|; the walk first seeks
    // only hits nearer than that (plus a margin). The closest hit, if it is nearer, lies in boxes the pruned walk
    // still visits in the reference's order (ties included), so the result is the unbounded walk's; when no hit
    // is found below the bound (a different ray, a grazing or culled surface) the walk is repeated unbounded.
    float bound = PT_INF;
    if (p.hint_pos.p && p.prune) {
      const float4 nd = pld(p.hint_nd, x, y);
      if (nd.w != 1.0f) {  // not background (zCenter == 1)
        const float4 P = pld(p.hint_pos, x, y);
        const float dist = length(sub(xyz(P), S));
        if (dist == dist) bound = dist * 1.001f + 1.0e-3f;
      }
    }
    float t;
    auto st = ray_stack<256, KS, DEEP>(stk + threadIdx.x, p, pid);
    int tri = closest_hit(p.scene, p.closest_tree, st, S, d, p.prune, &t, &steps, bound, &rewalk);
    if (tri < 0 && bound < PT_INF) {
      uint32_t more = 0;
      bool rw2 = false;
      tri = closest_hit(p.scene, p.closest_tree, st, S, d, p.prune, &t, &more, PT_INF, &rw2);
      steps += more;
      retry = true;
      rewalk = rewalk || rw2;
    }
    stnt(&p.wf.hit[pid], make_int2(tri, __float_as_int(t)));
    spill = st.spilled;
  }
  stat_add(p, kStatPrimRays, valid && count_ray ? 1u : 0u);
  stat_add(p, kStatPrimVisits, steps);
  stat_slots(p, kStatPrimSlots, steps);
  stat_add(p, kStatTieRewalks, rewalk ? 1u : 0u);
  stat_add(p, kStatPrimRetries, retry ? 1u : 0u);
  stat_add(p, kStatSpills, spill ? 1u : 0u);
  sched_cost(p.tiles, tile, steps);
  if (valid) add_row_cost(p, y - p.y0, pid, steps);
  }
}

// ------------------------------------------------ primaries by tile binning ---
// The primary rays' closest hits without a per-pixel BVH walk. The candidates of hitBVH for a ray are the
// triangles of the reference leaves whose own box the ray passes (hitAABB > 0: every reference ancestor box holds
// that box, so the walk reaches it — closest_hit's argument, pt_shading.h), the closest hit is the minimum t over
// them, and when one triangle alone attains it, that triangle. So each reference leaf is binned to the 16 x 16
// tiles whose pixels' primary rays can pass its box, and each pixel runs, over its tile's leaves, the walk's own
// leaf step: hitAABB on the leaf box with the walk's pruning bound, then hitTriangle on the leaf's triangles in
// order, seeking (as wf_primary) only hits nearer than this frame's G-buffer surface. A pixel whose minimum t two
// triangles share (the reference keeps the one its depth-first order meets first) or that finds nothing below the
// G-buffer bound is flagged and walked by wf_primary, as is every pixel if a list overflows. Same bits as wf_primary.
constexpr int kPChunk = 256;  // leaves staged in LDS per round
// per reference leaf: the pixel box of the primary rays that can pass its box — each face clipped to the widened
// frustum and projected; a box holding the eye covers the band — and the nearest t they can meet it at (t along
// the normalised ray is at least the camera-space depth w of the point)
__global__ void __launch_bounds__(256) pr_setup(PTParams p) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= p.scene.nleaves) return;
  const float4 lo4 = p.scene.leaves[2 * i], hi4 = p.scene.leaves[2 * i + 1];
  const float lo[3] = {lo4.x, lo4.y, lo4.z}, hi[3] = {hi4.x, hi4.y, hi4.z};
  const float* m = p.camRot;  // primary_dir: right = m[0..2], up = m[4..6], back = m[8..10]
  const float sx = p.aspect_corrected ? (float)p.W / (float)p.H : 1.0f;
  int4 box = make_int4(0, p.y0, p.W - 1, p.y1 - 1);
  float tmin = 0.0f;
  bool inside = true;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const float e = p.eye[a], tol = 1.0e-4f * (fabsf(e) + 1.0f);
    inside = inside && e >= lo[a] - tol && e <= hi[a] + tol;
  }
  if (!inside) {
    float3 C[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float X = (k & 1 ? hi[0] : lo[0]) - p.eye[0], Y = (k & 2 ? hi[1] : lo[1]) - p.eye[1],
                  Z = (k & 4 ? hi[2] : lo[2]) - p.eye[2];
      const float cx = (m[0] * X + m[1] * Y) + m[2] * Z, cy = (m[4] * X + m[5] * Y) + m[6] * Z,
                  cz = (m[8] * X + m[9] * Y) + m[10] * Z;
      C[k] = make_float3(cx / sx, cy, -cz);
    }
    // every corner inside the widened frustum (poly_box's clip planes) and in front: no clipping happens, and the
    // box's projection is the hull of its corners' projections (all w > 0)
    bool front = true;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      front = front && C[k].z > 0.0f && fabsf(C[k].x) <= 1.01f * C[k].z && fabsf(C[k].y) <= 1.01f * C[k].z;
    constexpr int F[6][4] = {{0, 2, 6, 4}, {1, 3, 7, 5}, {0, 1, 5, 4}, {2, 3, 7, 6}, {0, 1, 3, 2}, {4, 5, 7, 6}};
    int4 u = make_int4(1, 1, 0, 0);
    float w = 3.0e38f;
    bool any = false;
    if (front) {  // nothing to clip: the box of the corners' projections (poly_box's arithmetic, unrolled)
      float x0 = 3.0e38f, y0 = 3.0e38f, x1 = -3.0e38f, y1 = -3.0e38f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float px = ((C[k].x / C[k].z + 1.0f) * (float)p.W - 1.0f) * 0.5f;
        const float py = ((C[k].y / C[k].z + 1.0f) * (float)p.H - 1.0f) * 0.5f;
        x0 = fminf(x0, px); x1 = fmaxf(x1, px);
        y0 = fminf(y0, py); y1 = fmaxf(y1, py);
        w = fminf(w, C[k].z);
      }
      u = pixel_box(p.leaf_bins, x0, y0, x1, y1);
      any = !(u.x > u.z || u.y > u.w);
    }
#pragma unroll
    for (int f = 0; f < 6; ++f) {  // (unrolled: the corner indices stay compile-time, C in registers)
      if (front) break;
      float3 A[16];
#pragma unroll
      for (int k = 0; k < 4; ++k) A[k] = C[F[f][k]];
      int4 fb;
      float ft;
      if (!poly_box(p.leaf_bins, p.H, A, 4, 1.0f, 1.0f, &fb, &ft)) continue;
      if (fb.x > fb.z || fb.y > fb.w) continue;
      u = any ? make_int4(min(u.x, fb.x), min(u.y, fb.y), max(u.z, fb.z), max(u.w, fb.w)) : fb;
      w = fminf(w, ft);
      any = true;
    }
    box = any ? u : make_int4(1, 1, 0, 0);
    tmin = any ? w * 0.9999f : 0.0f;
  }
  bins_count_item(p.leaf_bins, i, box, tmin);
}

#ifndef PT_RASTER_WAVES
// waves/SIMD wf_primary_raster is compiled for (0: the compiler's choice, 67 VGPRs = 7 waves). 8 (64 VGPRs, no spill)
// measured the same (kernel trace, one frame at a time: 916.6 / 921.3 us, surface view 666.3 / 658.9; with PT_SHADE_WAVES
// 6 as well the frame rate fell 0.5 %: profiles/r05/occupancy_r8/)
#define PT_RASTER_WAVES 0
#endif
#if PT_RASTER_WAVES > 0
#define PT_RASTER_ATTR __attribute__((amdgpu_waves_per_eu(PT_RASTER_WAVES)))
#else
#define PT_RASTER_ATTR
#endif
__global__ void __launch_bounds__(256) PT_RASTER_ATTR wf_primary_raster(PTParams p) {
  __shared__ float4 slo[kPChunk], shi[kPChunk];
  __shared__ int4 sbox[kPChunk];
  __shared__ float stmin[kPChunk];
  __shared__ short wlist[4][kPChunk];  // per wave: the chunk's leaves that can meet its pixels
  const Bins& bn = p.leaf_bins;
  if (bn.ctr[2]) return;  // overflow: wf_primary walks every pixel
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  // subset slot -> band tile (PTParams::tile_stride: a pass may trace every tile_stride-th tile; the bins cover all)
  const int tile = blockIdx.x, gt = tile * p.tile_stride + p.tile_offset, ntx = (p.W + 15) / 16;
  const int x = (gt % ntx) * 16 + (wv & 1) * 8 + (ln & 7);
  const int y = p.y0 + (gt / ntx) * 16 + (wv >> 1) * 8 + (ln >> 3);
  const bool valid = x < p.W && y < p.y1;
  const int pid = (y - p.y0) * p.W + x;
  const v3 S = mk(p.eye[0], p.eye[1], p.eye[2]);
  const v3 d = primary_dir(p, x, y);
  const v3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  // the G-buffer bound of wf_primary: only hits nearer than the rasterised surface (plus a margin) are sought; a
  // pixel that finds none below it is flagged for the walk (which retries unbounded)
  float bound = PT_INF;
  if (valid && p.hint_pos.p && p.prune) {
    const float4 nd = pld(p.hint_nd, x, y);
    if (nd.w != 1.0f) {
      const float dist = length(sub(xyz(pld(p.hint_pos, x, y)), S));
      if (dist == dist) bound = dist * 1.001f + 1.0e-3f;
    }
  }
  float tbest = bound;
  int best = -1;
  bool tied = false;
  uint32_t steps = 0;
  // The tile's loosest pruning bound: a pixel's bound (tbest) only falls, so a leaf entered beyond the largest bound of
  // the tile's pixels, with a wider margin than the walk's (below), is skipped by every pixel — it is left out of the
  // staged chunk. Surface tiles drop the leaves hidden behind their surfaces; a tile with a background pixel keeps all.
  __shared__ float wmax[4];
  __shared__ int wcount[4];
  float tb = valid ? bound : 0.0f;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) tb = fmaxf(tb, __shfl_xor(tb, o));
  if (ln == 0) wmax[wv] = tb;
  __syncthreads();
  const float tile_lim = fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3])) * 1.0004f + 4.0e-4f;
  const int off = bn.tile_off[gt], total = bn.tile_off[gt + 1] - off;
  for (int base = 0; base < total; base += kPChunk) {
    __syncthreads();
    const int j = base + (int)threadIdx.x;
    int leaf = 0;
    float tm = 0.0f;
    if (j < total) {
      leaf = bn.pairs[off + j];
      tm = bn.tmin[leaf];
    }
    const bool keep = j < total && !(tm > tile_lim);
    const unsigned long long km = __ballot(keep);
    if (ln == 0) wcount[wv] = __popcll(km);
    __syncthreads();
    int n = 0, slot = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      slot += w < wv ? wcount[w] : 0;
      n += wcount[w];
    }
    if (keep) {  // compacted in thread order
      slot += __popcll(km & ((1ull << ln) - 1ull));
      slo[slot] = p.scene.leaves[2 * leaf];
      shi[slot] = p.scene.leaves[2 * leaf + 1];
      sbox[slot] = bn.box[leaf];
      stmin[slot] = tm;
    }
    __syncthreads();
    // this wave's share of the chunk: the staged leaves whose pixel box meets the wave's 8 x 8 pixels and that are not
    // entered beyond the loosest of its pixels' pruning bounds, in chunk order (the closest t, a unique closest
    // triangle and an exact tie met do not depend on the order the candidates are tested in); each lane then steps
    // through that list instead of the whole chunk
    float wl = valid ? tbest * 1.0002f + 2.0e-4f : 0.0f;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) wl = fmaxf(wl, __shfl_xor(wl, o));
    const int wx0 = x - (ln & 7), wy0 = y - (ln >> 3);
    int wn = 0;
    for (int k0 = 0; k0 < n; k0 += 64) {
      const int k = k0 + ln;
      bool ov = false;
      if (k < n) {
        const int4 b = sbox[k];
        ov = !(b.z < wx0 || b.x > wx0 + 7 || b.w < wy0 || b.y > wy0 + 7) && !(stmin[k] > wl);
      }
      const unsigned long long m = __ballot(ov);
      if (ov) wlist[wv][wn + __popcll(m & ((1ull << ln) - 1ull))] = (short)k;
      wn += __popcll(m);
    }
    __syncthreads();
    if (!valid) continue;
    for (int i = 0; i < wn; ++i) {
      const int k = wlist[wv][i];
      const int4 b = sbox[k];
      if (x < b.x || x > b.z || y < b.y || y > b.w) continue;  // no primary ray of this pixel passes the box
      const float lim = tbest * 1.0002f + 2.0e-4f;                // the walk's pruning bound (traverse<0>)
      if (stmin[k] > lim) continue;                               // entered beyond it
      const float4 lo = slo[k], hi = shi[k];
      float t0;
      const float dl = slab(S, inv, lo.x, lo.y, lo.z, hi.x, hi.y, hi.z, &t0);
      ++steps;
      if (!(dl > 0.0f) || t0 > lim) continue;
      const int ref = __float_as_int(lo.w), first = ref_leaf_first(ref), cnt = ref_leaf_count(ref);
      steps += (uint32_t)cnt;
      leaf_scan(p.scene.tri_geom, first, cnt, S, d, [&](int i, float t) {
        if (t < tbest) { tbest = t; best = i; tied = false; }
        else if (t == tbest && best >= 0) tied = true;
        return false;
      });
    }
  }
  const bool walk = valid && (tied || (best < 0 && bound < PT_INF));  // a tie, or nothing below the G-buffer bound
  if (valid) stnt(&p.wf.hit[pid], walk ? make_int2(kTieFix, 0) : make_int2(best, __float_as_int(tbest)));
  if (p.closest_tree) {  // flagged pixels: the wave-cooperative closest-hit walk (wf_primary_coop)
    const unsigned long long m = __ballot(walk);
    if (m) {
      int base = 0;
      if (ln == __ffsll((long long)m) - 1) base = atomicAdd(p.wf.counters + kCtrStragC, __popcll(m));
      base = __shfl(base, __ffsll((long long)m) - 1);
      if (walk) p.wf.strag_c[base + __popcll(m & ((1ull << ln) - 1ull))] = pid;
    }
  }
  stat_add(p, kStatPrimRays, valid ? 1u : 0u);
  stat_add(p, kStatPrimVisits, steps);
  stat_slots(p, kStatPrimSlots, steps);
  sched_cost(p.tiles, tile, steps);
  if (valid) add_row_cost(p, y - p.y0, pid, steps);
}

// ----------------------------------------------------------- bounce trace ---
template <int KS, bool DEEP>
__global__ void __launch_bounds__(kTB) PT_TRACE_ATTR wf_trace_closest(PTParams p, const int* __restrict__ list,
                                                                       const int* __restrict__ counts, int cap) {
  __shared__ int stk[KS * kTB];
  const int k = blockIdx.x * kTB + threadIdx.x;
  int pid;
  const bool valid = bins_get(list, counts, kLiveBins, cap, k, &pid);
  if (!p.wf.stats && !valid) return;  // (with counters on, every lane stays for the wave sums)
  uint32_t steps = 0;
  bool rewalk = false, spill = false;
  if (valid) {
    float4 o = ldnt(&p.wf.ray_o[pid]), dd = ldnt(&p.wf.ray_d[pid]);
    float t;
    auto st = ray_stack<kTB, KS, DEEP>(stk + threadIdx.x, p, pid);
    int tri = closest_hit(p.scene, p.closest_tree, st, xyz(o), xyz(dd), p.prune, &t, &steps, PT_INF, &rewalk);
    stnt(&p.wf.hit[pid], make_int2(tri, __float_as_int(t)));
    add_row_cost(p, pid / p.W, pid, steps);
    spill = st.spilled;
  }
  stat_add(p, kStatSpills, spill ? 1u : 0u);
  stat_add(p, kStatBounceRays, valid ? 1u : 0u);
  stat_add(p, kStatBounceVisits, steps);
  stat_slots(p, kStatBounceSlots, steps);
  stat_add(p, kStatTieRewalks, rewalk ? 1u : 0u);
}

// Shadow rays from the compacted lists wf_shade queued: HDR rays, then point-light rays.
template <int KS, bool WIDE, bool DEEP>
__global__ void __launch_bounds__(kTB) PT_TRACE_ATTR wf_trace_shadow(PTParams p, const int* __restrict__ list,
                                                                      const int* __restrict__ counts, int cap,
                                                                      int* __restrict__ strag_count) {
  __shared__ int stk[KS * kTB];
  const int k = blockIdx.x * kTB + threadIdx.x;
  const int nh = seg_total(counts);  // HDR list first, then the point-light lists bin by bin
  const bool point = k >= nh;
  int pid = -1;
  bool valid = true;
  if (!point) {
    seg_get(list, counts, cap, k, &pid);
  } else {
    int r = k - nh;
    valid = false;
#pragma unroll
    for (int b = 0; b < kPointBins; ++b) {
      const int nb = seg_total(counts + (1 + b) * kSeg);
      if (r < nb) {
        seg_get(list + (size_t)(1 + b) * kSeg * cap, counts + (1 + b) * kSeg, cap, r, &pid);
        valid = true;
        break;
      }
      r -= nb;
    }
  }
  bool deferred = false, spill = false;
  uint32_t steps = 0;
  if (valid) {
    float4 o = ldnt(&p.wf.ray_o[pid]);
    const float4 dir = point ? ldnt(&p.wf.sh_p[pid]) : ldnt(&p.wf.sh_h[pid]);  // point: (direction, distance)
    int occ = WIDE ? anyhit4<kTB, KS>(p.scene, stk + threadIdx.x, xyz(o), xyz(dir), point, dir.w, &steps) : -1;
    if (occ < 0) {  // binary walk (default), or the 4-wide stack overflowed
      auto st = ray_stack<kTB, KS, DEEP>(stk + threadIdx.x, p, pid);
      occ = anyhit2(anyhit_scene(p.scene), st, xyz(o), xyz(dir), point, dir.w, &steps, p.wf.shadow_budget, &deferred);
      spill = st.spilled;
    }
    if (!deferred) (point ? p.wf.occ_p : p.wf.occ_h)[pid] = occ;
    add_row_cost(p, pid / p.W, pid, steps);
  }
  stat_add(p, kStatShadowRays, valid && pid >= 0 ? 1u : 0u);
  stat_add(p, kStatSpills, spill ? 1u : 0u);
  stat_add(p, kStatShadowVisits, steps);
  stat_slots(p, kStatShadowSlots, steps);
  // rays past the step budget go to the cooperative walk (one wave-aggregated append per wave)
  const unsigned long long m = __ballot(deferred);
  if (m) {
    const int lane = threadIdx.x & 63;
    int base = 0;
    if (lane == __ffsll((long long)m) - 1) base = atomicAdd(strag_count, __popcll(m));
    base = __shfl(base, __ffsll((long long)m) - 1);
    if (deferred) p.wf.straggler[base + __popcll(m & ((1ull << lane) - 1ull))] = pid | (point ? (int)0x80000000 : 0);
  }
}

// Dense index k of the shadow lists (HDR list, then the point-light lists bin by bin) -> pixel, kind.
__device__ __forceinline__ bool shadow_item(const int* __restrict__ list, const int* __restrict__ counts, int cap,
                                            int nh, int k, int* pid, bool* point) {
  if (k < nh) {
    *point = false;
    return seg_get(list, counts, cap, k, pid);
  }
  *point = true;
  int r = k - nh;
#pragma unroll
  for (int b = 0; b < kPointBins; ++b) {
    const int nb = seg_total(counts + (1 + b) * kSeg);
    if (r < nb) return seg_get(list + (size_t)(1 + b) * kSeg * cap, counts + (1 + b) * kSeg, cap, r, pid);
    r -= nb;
  }
  return false;
}

// Dense index k over a batch's frames (per-frame totals tot[b]) -> frame b and its local index (wave-uniform data).
__device__ __forceinline__ int batch_frame(const int* tot, int nb, int* k) {
  for (int b = 0; b < nb; ++b) {
    if (*k < tot[b]) return b;
    *k -= tot[b];
  }
  return -1;
}

// Work queue of the refill traversal kernels: the list's dense index range is cut into 8 regions, one per XCD,
// each with its own head word (one returning atomic per grab of kGrab items; a per-XCD head keeps the grabs of
// 256 CUs off one word, MI355X_MICROARCH.md "dequeue"). A wave drains its XCD's region first, then the others;
// regions seen exhausted (a relaxed load of the head) are skipped without an atomic. Wave-uniform.
#ifndef PT_REFILL_QUEUE
#define PT_REFILL_QUEUE 0
#endif
constexpr int kGrab = 64;
struct WaveQueue {
  int* heads;
  int total, xcd;
  unsigned done;  // regions known exhausted
  int next, end;  // current grab [next, end)
  // static chunks (PT_REFILL_QUEUE 0): this wave's virtual wave index, the grid's waves, chunk rounds, big waves
  int vw, gw, R, big;
  __device__ __forceinline__ void chunk() {
    if (vw < big) {
      next = vw * 64 * R;
      end = next + 64 * R;
    } else {
      next = min(big * 64 * R + (vw - big) * 64, total);
      end = min(next + 64, total);
    }
  }
  __device__ __forceinline__ bool grab() {
    if (!PT_REFILL_QUEUE) {  // static chunks: the chunk of virtual wave vw + the grid's waves, if any
      vw += gw;
      chunk();
      return next < end;
    }
    for (int t = 0; t < 8; ++t) {
      const int r = (xcd + t) & 7;
      if ((done >> r) & 1u) continue;
      const int rs = (int)(((long long)total * r) >> 3), re = (int)(((long long)total * (r + 1)) >> 3);
      if (rs + __hip_atomic_load(heads + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= re) {
        done |= 1u << r;
        continue;
      }
      int base = 0;
      if ((threadIdx.x & 63) == 0) base = atomicAdd(heads + r, kGrab);
      base = __builtin_amdgcn_readfirstlane(__shfl(base, 0));
      if (rs + base < re) {
        next = rs + base;
        end = min(next + kGrab, re);
        return true;
      }
      done |= 1u << r;
    }
    return false;
  }
};
// Resident blocks the refill kernels launch with the queue: enough to fill the chip at their occupancy (5 waves/SIMD
// at 86 VGPRs, 2-wave blocks); waves beyond the work exit at their first grab.
constexpr int kRefillBlocks = 256 * 10;
// Static chunks (default), guided: the first PTParams::refill percent of the list goes out in chunks of 64 * R items
// (R = kRefillRounds) to the first waves, the rest in chunks of 64 (one item per lane) to the waves after them, so
// the launch does not end on long refill waves; idle lanes take new items only once at least kRefillMin lanes of
// the wave are idle (a refill stalls the whole wave for the new rays' loads). PT_REFILL_QUEUE=1: the per-XCD work
// queue above instead (measured slower: 109 fps against 148 without refill at 4K).
// Measured at 4K (tools/lib_ab.sh, R = 4, kRefillMin = 16): refill 0 / 50 / 75 / 85 % -> 147.7 / 156.0 / 159.3 /
// 158.7 fps with 4 frames in flight, 117.1 / 116.0 / 110.0 / 108.1 fps serial: the refill waves raise the share of
// busy lanes (shadow 0.42 -> 0.65) but lengthen the launch's tail, which other frames in flight fill.
// The cap on R (end of round 2, same box, K = 4, tools/lib_ab.sh + lib_ab_views.sh): 4 / 8 / 12 / 16 -> 179.6 / 182.6 /
// 183.1 / 182.6 fps at 4K, surface view 53.1 -> 57.2 fps with 12, 1080p unchanged (its lists give R < 4 anyway);
// kRefillMin 8 / 16 / 32: 180.1 / 179.6 / 178.0.
#ifndef PT_REFILL_ROUNDS
#define PT_REFILL_ROUNDS 24  // round 4 (every item refilled, 8 waves per SIMD): 8 / 12 / 16 / 24 / 32 / 48 -> surface
#endif                       // view 73.1 / 74.9 / 75.1 / 75.6 / 75.7 / 75.7 fps, 4K 221-222 throughout
#ifndef PT_REFILL_MIN
#define PT_REFILL_MIN 16
#endif
constexpr int kRefillRounds = PT_REFILL_ROUNDS, kRefillMin = PT_REFILL_MIN;
// Chunk rounds per big wave, from the list length: a big wave lasts about R one-ray waves, which pays only when the
// launch spans several rounds of resident waves anyway (at 1080p the lists are too short: refill there measured
// 367 -> 312 fps with R = 4 everywhere; with R from the length 380 fps at 1080p, 156.6 at 4K). kResidentWaves: 256 CUs
// x 20 waves (86 VGPRs: 5 waves per SIMD). Estimates of 16 / 12 / 8 waves per CU (more rounds per wave) measured
// 182.8 / 181.2 / 177.5 fps against 183.7 at 4K, the surface view unchanged (end of round 2).
// Round 4: the refill kernels now run 8 waves per SIMD (32 per CU); re-measured with that occupancy, 26 per CU gave
// 221.4 / 221.1 fps at 4K against 219.1 / 218.7 for 20 and 220.7 / 220.4 for 32, the surface view within noise
// (profiles/r04/refill_waves_ab.log).
#ifndef PT_RESIDENT_WAVES
#define PT_RESIDENT_WAVES (256 * 26)
#endif
constexpr int kResidentWaves = PT_RESIDENT_WAVES;
#ifndef PT_REFILL_DIV
#define PT_REFILL_DIV 1
#endif
// `waves`: the resident waves the launch may count on (0: the chip, kResidentWaves). A band renderer's launches are
// small and share the chip with the other frames in flight: sized for the whole chip they get one round per wave
// (no refill at all); sized for a share of it they keep refilling.
__device__ __forceinline__ int refill_rounds(int total, int waves) {
  const int r = total / (64 * (waves > 0 ? waves : kResidentWaves) * PT_REFILL_DIV);
  return r < 1 ? 1 : (r > kRefillRounds ? kRefillRounds : r);
}
__device__ __forceinline__ WaveQueue refill_queue(int* heads, int total, int big_pct, int waves) {
  WaveQueue q{heads, total, (int)(blockIdx.x & 7), 0u, 0, 0, 0, 0, 1, 0};
  if (PT_REFILL_QUEUE) {
    q.grab();
  } else {
    q.vw = blockIdx.x * (kTB / 64) + (threadIdx.x >> 6);
    q.gw = gridDim.x * (kTB / 64);
    q.R = refill_rounds(total, waves);
    q.big = q.R > 1 ? (int)((long long)total * big_pct / 100) / (64 * q.R) : 0;  // waves with big chunks
    q.chunk();
    q.done = 0xffu;
  }
  return q;
}
// The static chunks' grid. Until round 6 it had a wave for every 64 items the lists could hold (2 per pixel for the
// shadow rays: 129 600 blocks at 4K) while the frame's lists hold a fraction of that: every wave past the work read
// the list counts and left, ~250 000 of them per shadow launch, at the launch's end. Now at most
// PTSVGF_REFILL_GRID blocks (read once; default 256 CUs x 26 waves x 2 rounds / 2 waves per block; 0 = unbounded),
// and a wave whose chunk is done takes the chunk of its virtual wave + the grid's waves (WaveQueue::grab): the same
// chunks, hence the same per-ray walks and results.
inline int refill_blocks(int items_max, int grid = 0) {
  static const int cap = [] {
    const char* e = getenv("PTSVGF_REFILL_GRID");
    return e ? std::max(0, atoi(e)) : kResidentWaves * 2 / (kTB / 64);
  }();
  const int need = (items_max + kTB - 1) / kTB;
  if (PT_REFILL_QUEUE) return need < kRefillBlocks ? need : kRefillBlocks;
  const int c = grid > 0 ? grid : cap;
  return c > 0 && need > c ? c : need;
}

// Traversal counters only (PTParams::wf.stats set): of one frame's shadow rays of a bounce, those toward point lights
// and those found occluded, from the verdicts.
__global__ void __launch_bounds__(256) wf_shadow_stats(PTParams p, const int* __restrict__ list,
                                                       const int* __restrict__ counts, int cap) {
  const int nh = seg_total(counts);
  int tot = nh;
#pragma unroll
  for (int c = 0; c < kPointBins; ++c) tot += seg_total(counts + (1 + c) * kSeg);
  uint32_t npoint = 0, nocc = 0;
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < tot; k += gridDim.x * blockDim.x) {
    int pid;
    bool point;
    if (!shadow_item(list, counts, cap, nh, k, &pid, &point)) continue;
    npoint += point ? 1u : 0u;
    nocc += (point ? p.wf.occ_p : p.wf.occ_h)[pid] != 0 ? 1u : 0u;
  }
  stat_add(p, kStatShadowPoint, npoint);
  stat_add(p, kStatShadowOccluded, nocc);
}

// Shadow rays with lane refill. In wf_trace_shadow a wave lives as long as its longest ray while lanes whose rays
// ended idle: only ~42 % of the lane slots of shadow waves do traversal work on the 4K bench frame (35 % on the
// surface view; trace counters, bench.py "lane_efficiency"). Here waves stay resident and, between two leaf phases
// of their while-while walks, hand list items from the work queue to their idle lanes, so lanes stay busy until the
// queue runs dry. Per ray the walk is anyhit2's (same boxes, same pruning bound, same triangle tests, visit order
// per ray unchanged); any-hit verdicts do not depend on which lane or when.
// With a visit budget (PTParams::wf.shadow_budget) a ray still undecided past it is handed to the wave-cooperative
// walk (wf_shadow_coop) and its lane takes the next item, as in wf_trace_shadow.
// WIDE: the walk runs on the 4-wide form of the any-hit tree (pack_wide: the same candidate triangles); a ray whose
// pushes would overflow the LDS stack goes to the cooperative walk like a ray past the visit budget.
template <int KS, bool DEEP, bool WIDE>
__global__ void __launch_bounds__(kTB) PT_TRACE_ATTR wf_trace_shadow_refill(PTParams p, ListBatch lb, int cap,
                                                                             int* __restrict__ heads,
                                                                             int* __restrict__ strag_count) {
  __shared__ int stk[KS * kTB];
  const int lane = threadIdx.x & 63;
  int nh[kMaxBatch], tot[kMaxBatch];
  int total = 0;
  for (int b = 0; b < lb.nb; ++b) {
    nh[b] = seg_total(lb.counts[b]);
    tot[b] = nh[b];
#pragma unroll
    for (int c = 0; c < kPointBins; ++c) tot[b] += seg_total(lb.counts[b] + (1 + c) * kSeg);
    total += tot[b];
  }
  WaveQueue q = refill_queue(heads, total, p.refill, p.refill_waves);
  if (q.next >= q.end) return;
  const SceneDev sc = anyhit_scene(p.scene);
  const unsigned long long below = (1ull << lane) - 1ull;
  auto st = ray_stack<kTB, KS, DEEP>(stk + threadIdx.x, p, 0);
  bool have = false, point = false, spill = false, ovf = false;
  int pid = 0, sp = 0, node = kNone, leaf = kNone;
  v3 S = splat(0.0f), d = splat(0.0f), inv = splat(0.0f);
  float lim = 0.0f, maxd = 0.0f;
  uint32_t nvis = 0, nray = 0, rvis = 0;
  const uint32_t budget = p.wf.shadow_budget;
  while (true) {
    const unsigned long long idle = __ballot(!have);
    if (__popcll(idle) >= (__ballot(have) ? kRefillMin : 1) && (q.next < q.end || q.grab())) {
      // refill: the next items go to the idle lanes in lane order
      int k = q.next + __popcll(idle & below);
      const int fb = k < q.end ? batch_frame(tot, lb.nb, &k) : -1;
      if (!have && fb >= 0 && shadow_item(lb.list[fb], lb.counts[fb], cap, nh[fb], k, &pid, &point)) {
        pid += fb * lb.n;
        rvis = 0;
        const float4 o = ldnt(&p.wf.ray_o[pid]);
        const float4 dir = point ? ldnt(&p.wf.sh_p[pid]) : ldnt(&p.wf.sh_h[pid]);  // point: (direction, distance)
        S = xyz(o);
        d = xyz(dir);
        inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
        maxd = dir.w;
        lim = point ? maxd * 1.0002f + 2.0e-4f : __builtin_inff();
        sp = 0;
        node = WIDE ? p.scene.root4 : sc.root_ref;
        leaf = kNone;
        ovf = WIDE && PT_WIDE_SIGNED && !finite3(inv);  // axis-parallel (wide_step's signed planes): the coop walk
        if (node < 0) { leaf = node; node = kNone; }
        if (ovf) node = leaf = kNone;
        if constexpr (DEEP) st = ray_stack<kTB, KS, DEEP>(stk + threadIdx.x, p, pid);
        have = true;
        ++nray;
      }
      q.next = min(q.next + __popcll(idle), q.end);
    }
    if (!__any(have)) break;
    while (node >= 0) {  // anyhit2's descent (only lanes holding a ray have node >= 0)
      nvis += PT_NODE_VISIT;
      ++rvis;
      if constexpr (WIDE) {
        if (!wide_step<KS, PT_WIDE_SHADOW_SORT>(p.scene.bvh4, node, st, sp, S, inv, lim)) {  // stack full: coop walk
          ovf = true;
          node = leaf = kNone;
        }
        if (node < 0 && node != kNone && leaf == kNone) {
          leaf = node;
          node = sp > 0 ? st.get(--sp) : kNone;
        }
        if (!__any(leaf == kNone)) break;
        continue;
      }
      const float4* nd = sc.bvh + 4 * node;
      const float4 q0 = nd[0], q1 = nd[1], q2 = nd[2], q3 = nd[3];
      float t0l, t0r;
      const float dl = slab(S, inv, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, &t0l);
      const float dr = slab(S, inv, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, &t0r);
      const bool hl = dl > 0.0f && !(t0l > lim), hr = dr > 0.0f && !(t0r > lim);
      const int cl = __float_as_int(q3.x), cr = __float_as_int(q3.y);
      if (hl && hr) {
        const bool lnear = dl < dr;
        st.put(sp++, lnear ? cr : cl);
        node = lnear ? cl : cr;
      } else if (hl) {
        node = cl;
      } else if (hr) {
        node = cr;
      } else {
        node = sp > 0 ? st.get(--sp) : kNone;
      }
      if (node < 0 && node != kNone && leaf == kNone) {
        leaf = node;
        node = sp > 0 ? st.get(--sp) : kNone;
      }
      if (!__any(leaf == kNone)) break;
    }
    bool hit = false;
    while (leaf != kNone) {  // anyhit2's leaf phase
      const int first = ref_leaf_first(leaf), cnt = ref_leaf_count(leaf);
      nvis += (uint32_t)cnt;
      rvis += (uint32_t)cnt;
      if (leaf_scan(sc.tri_geom, first, cnt, S, d, [&](int, float t) {
            return t < PT_INF && (!point || length(sub(add(S, muls(d, t)), S)) < maxd);
          })) {
        hit = true;
        break;
      }
      leaf = kNone;
      if (node < 0 && node != kNone) {
        leaf = node;
        node = sp > 0 ? st.get(--sp) : kNone;
      }
    }
    if (have && !ovf && (hit || (node == kNone && leaf == kNone))) {  // this lane's ray is decided
      (point ? p.wf.occ_p : p.wf.occ_h)[pid] = hit;
      have = false;
      node = leaf = kNone;
      spill = spill || st.spilled;
    }
    // past the budget, or the 4-wide walk's stack full: the cooperative walk decides it
    const bool defer = have && (ovf || (budget && rvis > budget));
    const unsigned long long m = __ballot(defer);
    if (m) {
      int base = 0;
      if (lane == __ffsll((long long)m) - 1) base = atomicAdd(strag_count, __popcll(m));
      base = __shfl(base, __ffsll((long long)m) - 1);
      if (defer) {
        p.wf.straggler[base + __popcll(m & below)] = pid | (point ? (int)0x80000000 : 0);
        have = false;
        node = leaf = kNone;
        spill = spill || st.spilled;
      }
    }
  }
  stat_add(p, kStatShadowRays, nray);
  stat_add(p, kStatSpills, spill ? 1u : 0u);
  stat_add(p, kStatShadowVisits, nvis);
  stat_slots(p, kStatShadowSlots, nvis);
}

// Bounce rays (closest hit) with lane refill, as wf_trace_shadow_refill: per ray closest_hit's walk on the SAH tree
// over the reference leaves (pruned), and for a ray whose best t was met exactly by a second triangle the walk again
// on the reference tree in the reference's order (traverse<0>; the same lane restarts it before taking a new ray).
// Production switches only (closest_tree = prune = 1); the host keeps wf_trace_closest otherwise.
// With a visit budget (PTParams::wf.closest_budget) a ray still walking past it goes to the cooperative closest-hit
// walk (wf_closest_coop) and its lane takes the next item.
// WIDE: the walk runs on the 4-wide form of the SAH tree (pack_wide: the same candidate triangles, so the same
// minimum t); a ray whose best t was met exactly by a second triangle, or whose pushes would overflow the LDS stack,
// goes to the cooperative walk (wf_closest_coop), which re-walks ties on the reference tree.
template <int KS, bool DEEP, bool WIDE>
__global__ void __launch_bounds__(kTB) PT_TRACE_ATTR wf_trace_closest_refill(PTParams p, ListBatch lb, int cap,
                                                                              int* __restrict__ heads,
                                                                              int* __restrict__ strag_count) {
  __shared__ int stk[KS * kTB];
  const int lane = threadIdx.x & 63;
  int tot[kMaxBatch];
  int total = 0;
  for (int b = 0; b < lb.nb; ++b) {
    tot[b] = 0;
#pragma unroll
    for (int c = 0; c < kLiveBins * kSeg; ++c) tot[b] += lb.counts[b][c];
    total += tot[b];
  }
  WaveQueue q = refill_queue(heads, total, p.refill, p.refill_waves);
  if (q.next >= q.end) return;
  const unsigned long long below = (1ull << lane) - 1ull;
  auto st = ray_stack<kTB, KS, DEEP>(stk + threadIdx.x, p, 0);
  bool have = false, rewalk = false, tied = false, spill = false, ovf = false;
  int pid = 0, sp = 0, node = kNone, leaf = kNone, best = -1;
  const float4* tree = p.scene.bvh_any;  // this lane's tree: the SAH tree, or the reference tree for a re-walk
  v3 S = splat(0.0f), d = splat(0.0f), inv = splat(0.0f);
  float tbest = PT_INF;
  uint32_t nvis = 0, nray = 0, nrewalk = 0, rvis = 0;
  const uint32_t budget = p.wf.closest_budget;
  while (true) {
    const unsigned long long idle = __ballot(!have);
    if (__popcll(idle) >= (__ballot(have) ? kRefillMin : 1) && (q.next < q.end || q.grab())) {
      int k = q.next + __popcll(idle & below);
      const int fb = k < q.end ? batch_frame(tot, lb.nb, &k) : -1;
      if (!have && fb >= 0 && bins_get(lb.list[fb], lb.counts[fb], kLiveBins, cap, k, &pid)) {
        pid += fb * lb.n;
        const float4 o = ldnt(&p.wf.ray_o[pid]), dd = ldnt(&p.wf.ray_d[pid]);
        S = xyz(o);
        d = xyz(dd);
        inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
        tree = p.scene.bvh_any;
        node = WIDE ? p.scene.root4c : p.scene.root_any;
        rewalk = false;
        ovf = WIDE && PT_WIDE_SIGNED && !finite3(inv);  // axis-parallel (wide_step's signed planes): the coop walk
        tbest = PT_INF;
        best = -1;
        tied = false;
        sp = 0;
        leaf = kNone;
        if (node < 0) { leaf = node; node = kNone; }
        if (ovf) node = leaf = kNone;
        if constexpr (DEEP) st = ray_stack<kTB, KS, DEEP>(stk + threadIdx.x, p, pid);
        have = true;
        rvis = 0;
        ++nray;
      }
      q.next = min(q.next + __popcll(idle), q.end);
    }
    if (!__any(have)) break;
    while (node >= 0) {  // traverse<0>'s descent, pruned by the current best t
      nvis += PT_NODE_VISIT;
      ++rvis;
      if constexpr (WIDE) {
        if (!wide_step<KS, true>(p.scene.bvh4, node, st, sp, S, inv, tbest * 1.0002f + 2.0e-4f)) {
          ovf = true;  // stack full: the cooperative walk
          node = leaf = kNone;
        }
        if (node < 0 && node != kNone && leaf == kNone) {
          leaf = node;
          node = sp > 0 ? st.get(--sp) : kNone;
        }
        if (!__any(leaf == kNone)) break;
        continue;
      }
      const float4* nd = tree + 4 * node;
      const float4 q0 = nd[0], q1 = nd[1], q2 = nd[2], q3 = nd[3];
      float t0l, t0r;
      const float dl = slab(S, inv, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, &t0l);
      const float dr = slab(S, inv, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, &t0r);
      const float lim = tbest * 1.0002f + 2.0e-4f;
      const bool hl = dl > 0.0f && !(t0l > lim), hr = dr > 0.0f && !(t0r > lim);
      const int cl = __float_as_int(q3.x), cr = __float_as_int(q3.y);
      if (hl && hr) {
        const bool lnear = dl < dr;
        st.put(sp++, lnear ? cr : cl);
        node = lnear ? cl : cr;
      } else if (hl) {
        node = cl;
      } else if (hr) {
        node = cr;
      } else {
        node = sp > 0 ? st.get(--sp) : kNone;
      }
      if (node < 0 && node != kNone && leaf == kNone) {
        leaf = node;
        node = sp > 0 ? st.get(--sp) : kNone;
      }
      if (!__any(leaf == kNone)) break;
    }
    while (leaf != kNone) {  // traverse<0>'s leaf phase: strict '<' keeps the first triangle at a given t
      const int first = ref_leaf_first(leaf), cnt = ref_leaf_count(leaf);
      nvis += (uint32_t)cnt;
      rvis += (uint32_t)cnt;
      leaf_scan(p.scene.tri_geom, first, cnt, S, d, [&](int i, float t) {
        if (t < tbest) {
          tbest = t;
          best = i;
          tied = false;
        } else if (t == tbest && best >= 0) {
          tied = true;
        }
        return false;
      });
      leaf = kNone;
      if (node < 0 && node != kNone) {
        leaf = node;
        node = sp > 0 ? st.get(--sp) : kNone;
      }
    }
    if (have && !ovf && node == kNone && leaf == kNone && !(WIDE && tied)) {  // this lane's walk is complete
      if (!WIDE && !rewalk && tied) {  // exact tie: walk the ray again on the reference tree, in the reference's order
        rewalk = true;
        ++nrewalk;
        tree = p.scene.bvh;
        node = p.scene.root_ref;
        tbest = PT_INF;
        best = -1;
        tied = false;
        sp = 0;
        if (node < 0) { leaf = node; node = kNone; }
      } else {
        stnt(&p.wf.hit[pid], make_int2(best, __float_as_int(tbest)));
        have = false;
        spill = spill || st.spilled;
      }
    }
    // past the budget, the 4-wide walk's stack full, or (4-wide) an exact tie met: the cooperative walk finishes it
    const bool defer = have && (ovf || (budget && rvis > budget) ||
                                (WIDE && tied && node == kNone && leaf == kNone));
    const unsigned long long m = __ballot(defer);
    if (m) {
      int base = 0;
      if (lane == __ffsll((long long)m) - 1) base = atomicAdd(strag_count, __popcll(m));
      base = __shfl(base, __ffsll((long long)m) - 1);
      if (defer) {
        p.wf.strag_c[base + __popcll(m & below)] = pid;
        have = false;
        node = leaf = kNone;
        spill = spill || st.spilled;
      }
    }
  }
  stat_add(p, kStatBounceRays, nray);
  stat_add(p, kStatSpills, spill ? 1u : 0u);
  stat_add(p, kStatBounceVisits, nvis);
  stat_slots(p, kStatBounceSlots, nvis);
  stat_add(p, kStatTieRewalks, nrewalk);
}

// The shadow rays wf_trace_shadow deferred: one wave per ray walks cooperatively (shadow_coop_walk). A fixed
// grid strides over the straggler list (its length is known only on the device).
constexpr int kCoopWaves = 4;          // waves per block
#ifndef PT_COOP_BLOCKS
#define PT_COOP_BLOCKS 512
#endif
// 2048 waves in flight; 1024 / 2048 blocks measured within noise (profiles/r05/coop_blocks/: 4K 229.1 / 229.6 / 229.5 fps,
// surface view 78.8 / 78.9 / 79.0, one frame at a time 166.3 / 166.4 / 167.1)
constexpr int kCoopBlocks = PT_COOP_BLOCKS;
constexpr int kCoopCap = 1024;         // LDS stack entries per wave
__global__ void __launch_bounds__(64 * kCoopWaves) wf_shadow_coop(PTParams p, const int* __restrict__ strag_count) {
  __shared__ int st[kCoopWaves][kCoopCap];
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int n = *strag_count;
  for (int r = blockIdx.x * kCoopWaves + wv; r < n; r += gridDim.x * kCoopWaves) {
    const int item = p.wf.straggler[r];
    const bool point = item < 0;
    const int pid = item & 0x7fffffff;
    const float4 o = ldnt(&p.wf.ray_o[pid]);
    const float4 dir = point ? ldnt(&p.wf.sh_p[pid]) : ldnt(&p.wf.sh_h[pid]);
    const bool occ = shadow_coop_walk(anyhit_scene(p.scene), st[wv], kCoopCap, xyz(o), xyz(dir), point, dir.w);
    if ((threadIdx.x & 63) == 0) (point ? p.wf.occ_p : p.wf.occ_h)[pid] = occ;
  }
}

// The bounce rays wf_trace_closest_refill deferred: one wave per ray (closest_coop_walk).
__global__ void __launch_bounds__(64 * kCoopWaves) wf_closest_coop(PTParams p, const int* __restrict__ strag_count) {
  __shared__ int st[kCoopWaves][kCoopCap];
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int n = *strag_count;
  uint32_t nrewalk = 0;
  for (int r = blockIdx.x * kCoopWaves + wv; r < n; r += gridDim.x * kCoopWaves) {
    const int pid = p.wf.strag_c[r];
    const float4 o = ldnt(&p.wf.ray_o[pid]), dd = ldnt(&p.wf.ray_d[pid]);
    float t;
    bool rw;
    const int tri = closest_coop_walk(p.scene, st[wv], kCoopCap, xyz(o), xyz(dd), &t, &rw);
    if ((threadIdx.x & 63) == 0) {
      stnt(&p.wf.hit[pid], make_int2(tri, __float_as_int(t)));
      nrewalk += rw ? 1u : 0u;
    }
  }
  stat_add(p, kStatTieRewalks, nrewalk);
}

// The primary rays wf_primary_raster flagged (an exact-t tie, or no hit below the G-buffer bound): one wave per ray
// (closest_coop_walk: closest_hit's answer, unbounded, ties walked on the reference tree).
// After a pair-list overflow (leaf_bins.ctr[2]: the rasteriser skipped the frame) every pixel of the subset's tiles is
// walked here the same way, and the tile counts the skipped scatter left are cleared; until round 6 a wf_primary
// launch of one block per tile did that, and every frame paid for its launch.
__global__ void __launch_bounds__(64 * kCoopWaves) wf_primary_coop(PTParams p, const int* __restrict__ strag_count) {
  __shared__ int st[kCoopWaves][kCoopCap];
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (p.leaf_bins.ctr && p.leaf_bins.ctr[2]) {
    const int ntx = (p.W + 15) / 16, all = ntx * ((p.y1 - p.y0 + 15) / 16);
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < all; j += gridDim.x * blockDim.x)
      p.leaf_bins.tile_count[j] = 0;
    const int nsub = all / p.tile_stride + (all % p.tile_stride > p.tile_offset ? 1 : 0);  // the subset's tiles
    uint32_t nrays = 0, nrewalk = 0;
    for (int r = blockIdx.x * kCoopWaves + wv; r < nsub * 256; r += gridDim.x * kCoopWaves) {
      const int gt = (r >> 8) * p.tile_stride + p.tile_offset, i = r & 255;
      const int x = (gt % ntx) * 16 + (i & 15), y = p.y0 + (gt / ntx) * 16 + (i >> 4);
      if (x >= p.W || y >= p.y1) continue;  // wave-uniform
      const int pid = (y - p.y0) * p.W + x;
      float t;
      bool rw;
      const int tri = closest_coop_walk(p.scene, st[wv], kCoopCap, mk(p.eye[0], p.eye[1], p.eye[2]),
                                        primary_dir(p, x, y), &t, &rw);
      if ((threadIdx.x & 63) == 0) {
        stnt(&p.wf.hit[pid], make_int2(tri, __float_as_int(t)));
        nrewalk += rw ? 1u : 0u;
        ++nrays;
      }
    }
    stat_add(p, kStatPrimRays, nrays);
    stat_add(p, kStatTieRewalks, nrewalk);
    return;
  }
  const int n = *strag_count;
  uint32_t nrewalk = 0, nretry = 0;
  for (int r = blockIdx.x * kCoopWaves + wv; r < n; r += gridDim.x * kCoopWaves) {
    const int pid = p.wf.strag_c[r];
    const int x = pid % p.W, y = p.y0 + pid / p.W;
    const v3 S = mk(p.eye[0], p.eye[1], p.eye[2]);
    float t;
    bool rw;
    const int tri = closest_coop_walk(p.scene, st[wv], kCoopCap, S, primary_dir(p, x, y), &t, &rw);
    if ((threadIdx.x & 63) == 0) {
      stnt(&p.wf.hit[pid], make_int2(tri, __float_as_int(t)));
      nrewalk += rw ? 1u : 0u;
      ++nretry;
    }
  }
  stat_add(p, kStatTieRewalks, nrewalk);
  stat_add(p, kStatPrimRetries, nretry);
}

// shade()'s MIS combination (:950-966) for given shadow verdicts: hdriLight zeroes
// its value and pdf when occluded, calculatePointLight only its value.
struct NeeTerms {
  v3 hcalc, pcalc, bcalc;
  float hpdf, ppdf, bpdf;
};
__device__ __forceinline__ v3 nee_hit_light(v3 red, const NeeTerms& t, bool occ_h, bool occ_p) {
  v3 hcalc = t.hcalc, pcalc = t.pcalc;
  float hpdf = t.hpdf;
  if (occ_h) { hpdf = 0.0f; hcalc = splat(0.0f); }  // :934-937
  if (occ_p) pcalc = splat(0.0f);                   // :905-909 (pdf kept)
  float sw = ((hpdf + t.ppdf) + t.bpdf) + 1e-6f;
  float w1 = hpdf / sw, w2 = t.ppdf / sw, w3 = t.bpdf / sw;
  return mul(red, add(add(muls(hcalc, w1), muls(pcalc, w2)), muls(t.bcalc, w3)));
}
__device__ __forceinline__ bool zero_bits(v3 a) {  // all three exactly +0.0f
  return (__float_as_uint(a.x) | __float_as_uint(a.y) | __float_as_uint(a.z)) == 0u;
}

// ------------------------------------------------------------------ shade ---
// Bounce i: consume the closest hit of the ray in (ray_o, ray_d); on a hit,
// sample the next direction and prepare both NEE contributions (:948-968).
// Shadow rays whose verdict cannot change a bit of the result (a light below the
// surface: zero BRDF) are not queued; the others go to one compacted list.
#ifndef PT_SHADE_WAVES
#define PT_SHADE_WAVES 0  // waves/SIMD wf_shade is compiled for (0: the compiler's choice, 93 VGPRs = 5 waves)
#endif
#if PT_SHADE_WAVES > 0
#define PT_SHADE_ATTR __attribute__((amdgpu_waves_per_eu(PT_SHADE_WAVES)))
#else
#define PT_SHADE_ATTR
#endif
__global__ void __launch_bounds__(256) PT_SHADE_ATTR wf_shade(PTParams p, int bounce, const int* __restrict__ list_in,
                                                const int* __restrict__ counts_in, int* __restrict__ list_out,
                                                int* __restrict__ counts_out, int* __restrict__ shadow_out,
                                                int* __restrict__ shadow_counts, int cap) {
  // bounce 0: one tile per block. Later bounces: 256 list items per chunk, a block taking chunks blockIdx.x,
  // + gridDim.x, ... (a grid a multiple of kSeg: chunk c appends to segment c % kSeg, as one block per chunk did)
  int total = 0;
  if (bounce > 0)
    for (int i = 0; i < kLiveBins * kSeg; ++i) total += counts_in[i];
  for (int c = blockIdx.x; bounce == 0 || c * 256 < total; c += gridDim.x) {
    const int k = c * 256 + threadIdx.x;
    int pid = 0;
    bool valid;
    if (bounce == 0) {
      // one 16 x 16 primary tile per block, in descending order of this frame's primary-ray cost
      // (tiles.perm_next, sorted right after wf_primary): the rays of expensive tiles are appended to
      // the lists first, so every later list-driven trace launch starts its slowest rays first
      const int ntx = (p.W + 15) / 16;
      const int tile = (p.tiles.cost ? p.tiles.perm_next[blockIdx.x] : (int)blockIdx.x) * p.tile_stride + p.tile_offset;
      const int x = (tile % ntx) * 16 + (threadIdx.x & 15), ly = (tile / ntx) * 16 + (threadIdx.x >> 4);
      valid = x < p.W && ly < p.y1 - p.y0;
      pid = ly * p.W + x;
    } else {
      valid = bins_get(list_in, counts_in, kLiveBins, cap, k, &pid);
    }
    bool push = false, need_h = false, need_p = false;
    int pbin = 0;  // point-light list of this ray (light index mod kPointBins)
    int lbin = 0;  // live list of the continuing ray (direction octant)
    if (valid) {
      int x, y;
      pix_xy(p, pid, &x, &y);
      int2 hr = ldnt(&p.wf.hit[pid]);
      v3 S, d;
      uint32_t seed;
      v3 light, red;
      if (bounce == 0) {
        S = mk(p.eye[0], p.eye[1], p.eye[2]);
        d = primary_dir(p, x, y);
        seed = ((uint32_t)x * 1973u + (uint32_t)y * 9277u + p.frameCounter * 26699u) | 1u;  // :433-436
        wang_hash(&seed);  // AA jitter rand() x2 (:1060), never applied
        wang_hash(&seed);
        light = splat(0.0f);
        red = splat(1.0f);
      } else {
        S = xyz(ldnt(&p.wf.ray_o[pid]));
        d = xyz(ldnt(&p.wf.ray_d[pid]));
        seed = ldnt(&p.wf.seed[pid]);
        light = xyz(ldnt(&p.wf.light[pid]));
        red = xyz(ldnt(&p.wf.red[pid]));
      }
      if (hr.x < 0) {  // miss (:1084-1087)
        light = add(light, mul(hdr_color(p, d), red));
        if (bounce == 0) {
          pst(p.emission, x, y, f4(0.0f, 0.0f, 0.0f, 1.0f));
          pst(p.albedo, x, y, f4(0.0f, 0.0f, 0.0f, 1.0f));
        }
      } else {
        Hit h = decode_hit(p.scene, hr.x, __int_as_float(hr.y), S, d);
        if (bounce == 0) {
          pst(p.emission, x, y, f4(h.m.emissive.x, h.m.emissive.y, h.m.emissive.z, 1.0f));
          pst(p.albedo, x, y, f4(h.m.baseColor.x, h.m.baseColor.y, h.m.baseColor.z, 1.0f));
        }
        uint32_t ps = ((uint32_t)x * 1973u + (uint32_t)y * 9277u + (uint32_t)(114514 / 1919) * 26699u) | 1u;
        float cpu = u32_to_unit(wang_hash(&ps));
        float cpv = u32_to_unit(wang_hash(&ps));
        float xi1 = p.sobol_u[bounce] + cpu;
        if (xi1 > 1.0f) xi1 -= 1.0f;
        if (xi1 < 0.0f) xi1 += 1.0f;
        float xi2 = p.sobol_v[bounce] + cpv;
        if (xi2 > 1.0f) xi2 -= 1.0f;
        if (xi2 < 0.0f) xi2 += 1.0f;
        float xi3 = u32_to_unit(wang_hash(&seed));
        v3 V = neg(h.viewDir);
        v3 L = sample_brdf(xi1, xi2, xi3, V, h.normal, h.m);
        if (dot(h.normal, L) > 0.0f) {
          push = true;
                  v3 brdf = brdf_eval(V, h.normal, L, h.m);
          float bpdf = brdf_pdf(V, h.normal, L, h.m);
          // hdriLight, evaluated as if unoccluded (:922-946)
          float r1 = u32_to_unit(wang_hash(&seed));
          float r2 = u32_to_unit(wang_hash(&seed));
          v3 hd = sample_hdr(p, r1, r2);
          float hpdf;
          v3 hv = hdr_color_pdf(p, hd, &hpdf);
          v3 hb = brdf_eval(V, h.normal, hd, h.m);
          v3 hcalc = divs(mul(muls(hb, f_abs(dot(hd, h.normal))), hv), hpdf);
          // calculatePointLight, as if unoccluded (:884-919)
          v3 pcalc = splat(0.0f);
          float4 shp = f4(0.0f, 0.0f, 0.0f, -1.0f);
          if (p.pointLightSize != 0) {
            float ppdf = (2.0f * PT_PI) / (float)p.pointLightSize;
            int li = (int)(u32_to_unit(wang_hash(&seed)) * (float)p.pointLightSize);
            pbin = li & (kPointBins - 1);
            v3 lpos = splat(0.0f), lrad = splat(0.0f);
            if (li >= 0 && li < p.scene.nlights_buf) {
              const float* lp = p.scene.lights + 6 * li;
              lpos = mk(lp[0], lp[1], lp[2]);
              lrad = mk(lp[3], lp[4], lp[5]);
            }
            v3 ld = normalize(sub(lpos, h.P));
            float dist = length(sub(lpos, h.P));
            v3 plv = divs(lrad, dist * dist);
            v3 pb = brdf_eval(V, h.normal, ld, h.m);
            pcalc = divs(muls(mul(plv, pb), f_abs(dot(ld, h.normal))), ppdf);
            shp = f4(ld.x, ld.y, ld.z, dist);
          }
          v3 cosb = muls(brdf, f_abs(dot(L, h.normal)));
          v3 bcalc = divs(mul(h.m.emissive, cosb), bpdf);
          // A verdict only zeroes terms: with the point value exactly +0 (light below the
          // surface: zero BRDF) its ray cannot change a bit; the HDR verdict also moves the
          // MIS weights, so it is dropped only when every term is +0 and every pdf finite.
          const bool pz = zero_bits(pcalc);
          need_p = shp.w >= 0.0f && !pz;
          need_h = !(pz && zero_bits(hcalc) && zero_bits(bcalc) && __builtin_isfinite(hpdf) && __builtin_isfinite(bpdf));
          stnt(&p.wf.pend0[pid], f4(hcalc.x, hcalc.y, hcalc.z, hpdf));
          stnt(&p.wf.pend1[pid], f4(pcalc.x, pcalc.y, pcalc.z, bpdf));
          stnt(&p.wf.pend2[pid], f4(bcalc.x, bcalc.y, bcalc.z, 0.0f));
          stnt(&p.wf.pend3[pid], f4(cosb.x, cosb.y, cosb.z, 0.0f));
          stnt(&p.wf.sh_h[pid], f4(hd.x, hd.y, hd.z, 0.0f));
          stnt(&p.wf.sh_p[pid], shp);
          stnt(&p.wf.ray_o[pid], f4(h.P.x, h.P.y, h.P.z, 0.0f));
          stnt(&p.wf.ray_d[pid], f4(L.x, L.y, L.z, 0.0f));
          stnt(&p.wf.red[pid], f4(red.x, red.y, red.z, 0.0f));
          stnt(&p.wf.occ_h[pid], (uint8_t)0);
          stnt(&p.wf.occ_p[pid], (uint8_t)0);
        }
      }
      stnt(&p.wf.seed[pid], seed);
      stnt(&p.wf.light[pid], f4(light.x, light.y, light.z, 0.0f));
    }
    // HDR and point-light shadow rays go to separate lists so trace waves stay homogeneous

    block_push_shade(push, lbin, need_h, need_p, pbin, pid, list_out, counts_out, shadow_out, shadow_counts, cap, c);
    if (bounce == 0) break;
    __syncthreads();  // the next chunk's push reuses block_push_shade's shared counters
  }
}

// ----------------------------------------------------------------- finish ---
__global__ void __launch_bounds__(256) wf_finish(PTParams p, const int* __restrict__ list,
                                                 const int* __restrict__ counts, int cap) {
  int total = 0;
  for (int i = 0; i < kLiveBins * kSeg; ++i) total += counts[i];
  for (int k = blockIdx.x * 256 + threadIdx.x; k < total; k += gridDim.x * 256) {
  int pid;
  if (!bins_get(list, counts, kLiveBins, cap, k, &pid)) continue;
  float4 q0 = ldnt(&p.wf.pend0[pid]), q1 = ldnt(&p.wf.pend1[pid]), q2 = ldnt(&p.wf.pend2[pid]), q3 = ldnt(&p.wf.pend3[pid]);
  NeeTerms nt;
  nt.hcalc = xyz(q0); nt.pcalc = xyz(q1); nt.bcalc = xyz(q2);
  nt.hpdf = q0.w; nt.bpdf = q1.w;
  nt.ppdf = p.pointLightSize != 0 ? (2.0f * PT_PI) / (float)p.pointLightSize : 0.0f;
  v3 cosb = xyz(q3);
  v3 red = xyz(ldnt(&p.wf.red[pid])), light = xyz(ldnt(&p.wf.light[pid]));
  v3 hitLight = nee_hit_light(red, nt, p.wf.occ_h[pid] != 0, p.wf.occ_p[pid] != 0);
  red = mul(red, divs(cosb, nt.bpdf));
  light = add(light, hitLight);
  stnt(&p.wf.red[pid], f4(red.x, red.y, red.z, 0.0f));
  stnt(&p.wf.light[pid], f4(light.x, light.y, light.z, 0.0f));
  }
}

// --------------------------------------------------------------- finalize ---
__global__ void __launch_bounds__(256) wf_finalize(PTParams p) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= p.W * (p.y1 - p.y0)) return;
  int x, y;
  pix_xy(p, k, &x, &y);
  if (p.tile_stride > 1) {  // pixels of tiles outside the subset keep their contents
    const int t = ((y - p.y0) >> 4) * ((p.W + 15) / 16) + (x >> 4);
    if (t % p.tile_stride != p.tile_offset) return;
  }
  v3 light = vclamp(xyz(ldnt(&p.wf.light[k])), 0.0f, p.clamp_threshold);  // :1110-1113
  v3 color = splat(0.0f);
  if (!f_isnan(light.x) && !f_isnan(light.y) && !f_isnan(light.z)) color = light;
  if (p.accumulate && p.last.p) {  // :1116-1119
    float4 lc = pld(p.last, x, y);
    color = mixv(xyz(lc), color, 1.0f / (float)(p.frameCounter + 1u));
  }
  pst(p.color, x, y, f4(color.x, color.y, color.z, 1.0f));
}

// A producer block appends at most 256 items to the segment blockIdx % kSeg; the most blocks
// an appending launch has is the larger of the per-pixel grid and the bounce-0 tile grid.
int wf_list_capacity(int W, int rows) {
  const int blocks = std::max((W * rows + 255) / 256, ((W + 15) / 16) * ((rows + 15) / 16));
  return (blocks + kSeg - 1) / kSeg * 256;
}

// Tiles of the subset k * stride + offset among the band's 16 x 16 tiles (PTParams::tile_stride).
int wf_subset_tiles(int W, int rows, int stride, int offset) {
  const int n = ((W + 15) / 16) * ((rows + 15) / 16);
  if (stride < 1 || offset < 0 || offset >= stride) return -1;
  return offset < n ? (n - offset + stride - 1) / stride : 0;
}

// Launch order of one frame. With a WfFork (uniform trace_fork) the closest-hit trace of bounce 1 (it needs only the
// rays and live list the bounce-0 shade wrote) runs beside the bounce-0 shadow trace and finish on the side stream;
// the join comes before the bounce-1 shade, which reuses the shadow list and reads the finished throughput. The two
// traversal launches then fill each other's tails. Without `fk` the launches are serial.
// nb > 1: a batch of frames (pt_pass_draw_batch) — per-frame launches for the primaries, shades and finishes, ONE
// launch per bounce for the list-driven traversals of every frame's rays (lane-refill kernels; the one-ray-per-lane
// kernels run per frame). Frame b's wavefront state lies at pid offset b * N of ps[0]'s, its counters at
// ps[0].wf.counters + b * kWfCounters; the batched launches use frame 0's work-queue heads and straggler lists.
// Grid of the list-driven shade (bounces > 0) and finish launches: until round 6 one block per 256 pixels (32 400 at
// 4K), most of them past the list's end, reading its counts and leaving. Now at most PTSVGF_LIST_BLOCKS (read once;
// default 2 048, a multiple of kSeg; 0 = one per 256 pixels) striding over 256-item chunks.
static int list_blocks(int n_items_max, int grid = 0) {
  static const int cap = [] {
    const char* e = getenv("PTSVGF_LIST_BLOCKS");
    const int v = e ? std::max(0, atoi(e)) : 2048;
    return (v + kSeg - 1) / kSeg * kSeg;
  }();
  const int need = (n_items_max + 255) / 256;
  const int c = grid > 0 ? (grid + kSeg - 1) / kSeg * kSeg : cap;
  return c > 0 && need > c ? c : need;
}
template <int KS, bool DEEP>
int launch_wavefront(const PTParams* ps, int nb, hipStream_t s, const WfFork* fk) {
  const PTParams& p = ps[0];
  const int rows = p.y1 - p.y0;
  if (rows <= 0) return 0;
  const int N = p.W * rows;
  const int cap = wf_list_capacity(p.W, rows);  // per segment; the host sized the lists with the same function
  hipError_t e = hipMemsetAsync(p.wf.counters, 0, (size_t)nb * kWfCounters * sizeof(int), s);
  if (e != hipSuccess) return (int)e;
  const int ntiles = wf_subset_tiles(p.W, rows, p.tile_stride, p.tile_offset);
  if (ntiles <= 0) return 0;
  for (int b = 0; b < nb; ++b) {
    const PTParams& f = ps[b];
    if (f.primary_raster) {  // leaves binned to every tile of the band; the subset's tiles rasterised
      if (f.scene.nleaves > 0) hipLaunchKernelGGL(pr_setup, dim3((f.scene.nleaves + 255) / 256), dim3(256), 0, s, f);
      const int rc = launch_bins(f.leaf_bins, s);
      if (rc) return rc;
      hipLaunchKernelGGL(wf_primary_raster, dim3(ntiles), dim3(256), 0, s, f);
      if (f.closest_tree)
        hipLaunchKernelGGL(wf_primary_coop, dim3(kCoopBlocks), dim3(64 * kCoopWaves), 0, s, f,
                           (const int*)(f.wf.counters + kCtrStragC));
      static const bool fix_launch = [] {  // A/B only: PTSVGF_PRIMARY_FIX_LAUNCH=1 launches it anyway (512 blocks)
        const char* e = getenv("PTSVGF_PRIMARY_FIX_LAUNCH");
        return e && atoi(e) != 0;
      }();
      if (!f.closest_tree || fix_launch) {  // the flagged pixels (and, after an overflow, all) by the per-pixel walk
        PTParams q = f;
        q.pr_fix = f.leaf_bins.ctr;
        hipLaunchKernelGGL((wf_primary<KS, DEEP>), dim3(f.closest_tree ? std::min(ntiles, 512) : ntiles), dim3(256), 0,
                           s, q, ntiles);
      }
    } else {
      hipLaunchKernelGGL((wf_primary<KS, DEEP>), dim3(ntiles), dim3(256), 0, s, f, ntiles);
    }
    if (f.tiles.cost) {  // this frame's primary costs -> tile order of the bounce-0 shade and the next frame
      const int rc = launch_tile_sort(f.tiles.cost, f.tiles.perm_next, f.tiles.ntiles, s);
      if (rc) return rc;
    }
  }
  const int gN = (N + 255) / 256, gT = (N + kTB - 1) / kTB, gT2 = (2 * N + kTB - 1) / kTB;
  const int gL = list_blocks(N, p.list_grid);  // list-driven shade / finish: at most list_blocks() blocks striding
  const int gS0 = ntiles;  // bounce-0 shade: one block per primary tile
  auto lst = [&](const PTParams& f, int i) { return (i & 1) ? f.wf.list1 : f.wf.list0; };  // bounce i's live list
  const bool refill_closest = p.refill && p.closest_tree && p.prune && p.scene.bvh_any;
  const bool wide = !DEEP && p.refill && p.scene.bvh4;  // the refill walks on the 4-wide any-hit tree
  auto closest = [&](int i) {
    hipStream_t st = s;
    if (refill_closest) {
      ListBatch lb{nb, N, {}, {}};
      for (int b = 0; b < nb; ++b) {
        lb.list[b] = lst(ps[b], i + 1);
        lb.counts[b] = ps[b].wf.counters + kWfCtr * (i - 1);
      }
      int* strag = p.wf.counters + kWfCtr * i + kCtrStragC;
      if constexpr (!DEEP)
        if (wide) {
          hipLaunchKernelGGL((wf_trace_closest_refill<kWideKS, false, true>), dim3(refill_blocks(nb * N, p.refill_grid)), dim3(kTB), 0, st,
                             p, lb, cap, p.wf.counters + kWfCtr * i + kCtrQClosest, strag);
        }
      if (!wide)
        hipLaunchKernelGGL((wf_trace_closest_refill<KS, DEEP, false>), dim3(refill_blocks(nb * N, p.refill_grid)), dim3(kTB), 0, st,
                           p, lb, cap, p.wf.counters + kWfCtr * i + kCtrQClosest, strag);
      if (p.wf.closest_budget || wide)  // (4-wide: ties and stack overflows go there too)
        hipLaunchKernelGGL(wf_closest_coop, dim3(kCoopBlocks), dim3(64 * kCoopWaves), 0, st, p, (const int*)strag);
    } else {
      for (int b = 0; b < nb; ++b)
        hipLaunchKernelGGL((wf_trace_closest<KS, DEEP>), dim3(gT), dim3(kTB), 0, st, ps[b], lst(ps[b], i + 1),
                           (const int*)(ps[b].wf.counters + kWfCtr * (i - 1)), cap);
    }
  };
  // deep trees keep one stream: both walks would use the pixel's spill columns
  const bool split = fk && !DEEP && p.max_depth > 1;
  for (int i = 0; i < p.max_depth; ++i) {
    if (i > 0) closest(i);
    if (i == 1 && split) {
      const hipError_t e = hipStreamWaitEvent(s, fk->join, 0);
      if (e != hipSuccess) return (int)e;
    }
    for (int b = 0; b < nb; ++b) {
      const PTParams& f = ps[b];
      const int* live_in = f.wf.counters + kWfCtr * (i > 0 ? i - 1 : 0);
      hipLaunchKernelGGL(wf_shade, dim3(i == 0 ? gS0 : gL), dim3(256), 0, s, f, i, (const int*)lst(f, i + 1), live_in,
                         lst(f, i), f.wf.counters + kWfCtr * i, f.wf.shadow_list, f.wf.counters + kWfCtr * i + kCtrHdr,
                         cap);
    }
    hipStream_t ss = s;  // the shadow walk's and finish's stream
    if (i == 0 && split) {
      hipError_t e = hipEventRecord(fk->fork, s);
      if (e == hipSuccess) e = hipStreamWaitEvent(fk->side, fk->fork, 0);
      if (e != hipSuccess) return (int)e;
      ss = fk->side;
    }
    if (p.refill) {
      ListBatch lb{nb, N, {}, {}};
      for (int b = 0; b < nb; ++b) {
        lb.list[b] = ps[b].wf.shadow_list;
        lb.counts[b] = ps[b].wf.counters + kWfCtr * i + kCtrHdr;
      }
      int* strag = p.wf.counters + kWfCtr * i + kCtrStrag;  // shadow rays handed to the cooperative walk
      if constexpr (!DEEP)
        if (wide) {
          hipLaunchKernelGGL((wf_trace_shadow_refill<kWideKS, false, true>), dim3(refill_blocks(2 * nb * N, p.refill_grid)), dim3(kTB), 0,
                             ss, p, lb, cap, p.wf.counters + kWfCtr * i + kCtrQShadow, strag);
        }
      if (!wide)
        hipLaunchKernelGGL((wf_trace_shadow_refill<KS, DEEP, false>), dim3(refill_blocks(2 * nb * N, p.refill_grid)), dim3(kTB), 0, ss,
                           p, lb, cap, p.wf.counters + kWfCtr * i + kCtrQShadow, strag);
      if (p.wf.shadow_budget || wide)
        hipLaunchKernelGGL(wf_shadow_coop, dim3(kCoopBlocks), dim3(64 * kCoopWaves), 0, ss, p, (const int*)strag);
    } else {
      for (int b = 0; b < nb; ++b) {
        const PTParams& f = ps[b];
        const int* shadow = f.wf.counters + kWfCtr * i + kCtrHdr;
        int* strag = f.wf.counters + kWfCtr * i + kCtrStrag;
        if (f.scene.bvh4)
          hipLaunchKernelGGL((wf_trace_shadow<KS, true, DEEP>), dim3(gT2), dim3(kTB), 0, ss, f,
                             (const int*)f.wf.shadow_list, shadow, cap, strag);
        else
          hipLaunchKernelGGL((wf_trace_shadow<KS, false, DEEP>), dim3(gT2), dim3(kTB), 0, ss, f,
                             (const int*)f.wf.shadow_list, shadow, cap, strag);
        if (f.wf.shadow_budget)
          hipLaunchKernelGGL(wf_shadow_coop, dim3(kCoopBlocks), dim3(64 * kCoopWaves), 0, ss, f, (const int*)strag);
      }
    }
    if (p.wf.stats)
      for (int b = 0; b < nb; ++b)
        hipLaunchKernelGGL(wf_shadow_stats, dim3(gN), dim3(256), 0, ss, ps[b], (const int*)ps[b].wf.shadow_list,
                           (const int*)(ps[b].wf.counters + kWfCtr * i + kCtrHdr), cap);
    for (int b = 0; b < nb; ++b)
      hipLaunchKernelGGL(wf_finish, dim3(gL), dim3(256), 0, ss, ps[b], (const int*)lst(ps[b], i),
                         (const int*)(ps[b].wf.counters + kWfCtr * i), cap);
    if (i == 0 && split) {
      const hipError_t e = hipEventRecord(fk->join, ss);
      if (e != hipSuccess) return (int)e;
    }
  }
  for (int b = 0; b < nb; ++b) hipLaunchKernelGGL(wf_finalize, dim3(gN), dim3(256), 0, s, ps[b]);
  return (int)hipGetLastError();
}

int launch_pathtrace_wavefront(const PTParams& p, hipStream_t s, const WfFork* fk) {
  // the LDS stack bounds resident waves: a tree that fits the small stack gets more of them
  if (p.wf.spill) return launch_wavefront<kSpillKS, true>(&p, 1, s, fk);  // deep tree
  return p.stack_need <= kStackSmall ? launch_wavefront<kStackSmall, false>(&p, 1, s, fk)
                                     : launch_wavefront<kStack, false>(&p, 1, s, fk);
}

int launch_pathtrace_wavefront_batch(const PTParams* ps, int nb, hipStream_t s, const WfFork* fk) {
  if (nb < 1 || nb > kMaxBatch) return (int)hipErrorInvalidValue;
  if (ps[0].wf.spill) return launch_wavefront<kSpillKS, true>(ps, nb, s, fk);
  return ps[0].stack_need <= kStackSmall ? launch_wavefront<kStackSmall, false>(ps, nb, s, fk)
                                         : launch_wavefront<kStack, false>(ps, nb, s, fk);
}

}  // namespace ptk

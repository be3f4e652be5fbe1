// kernels_pt.hip — per-pixel path tracer with next-event estimation and the
// ray-cast G-buffer, for gfx950 (wave64, no RT hardware: traversal is VALU).
//
// Behaviour restated from shaders/path_tracing.frag (file:line cited per
// function). Engineering differences from the GLSL, all result-preserving:
//  * scene decoded once at bind time into float4 SoA records (pt_device.h) —
//    one 64-B node fetch tests both children, one 64-B record per triangle test;
//  * short traversal stack in LDS (column layout: conflict-free), near child
//    visited first exactly as hitBVH's push order (:407-420);
//  * closest-hit rays prune boxes whose entry lies beyond the current hit
//    (with a safety margin; the reference visits every intersected box, which
//    can only change the result through its strict '<' tie rule — a pruned box
//    holds no triangle nearer than the current hit);
//  * shadow rays are any-hit: the HDR test only asks isHit (:934), the point
//    test asks whether the closest hit is nearer than the light (:905-909);
//  * material/normal of the closest hit are decoded once after traversal (the
//    reference decodes per leaf; the values are a function of the triangle and
//    the hit point only).
// Built with -ffp-contract=off and the shared GLSL built-ins: the CPU oracle's
// restatement of the same shader reproduces these outputs bit for bit.
#include <hip/hip_runtime.h>

#include "glsl_builtins.h"
#include "pt_device.h"
#include "pt_shading.h"

using namespace glsl;

namespace ptk {

// ------------------------------------------------------------ path tracer ---
__global__ void __launch_bounds__(kBlock) pathtrace_kernel(PTParams p) {
  __shared__ int stk[kStack * kBlock];
  LdsStack<kBlock> s{stk + threadIdx.x};
  // 16x16 pixel tile per block; each wave owns an 8x8 sub-tile (ray coherence).
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  const int x = blockIdx.x * 16 + (wv & 1) * 8 + (ln & 7);
  const int y = p.y0 + blockIdx.y * 16 + (wv >> 1) * 8 + (ln >> 3);
  if (x >= p.W || y >= p.y1) return;

  uint32_t seed = ((uint32_t)x * 1973u + (uint32_t)y * 9277u + p.frameCounter * 26699u) | 1u;  // :433-436
  wang_hash(&seed);  // AA jitter rand() x2 (:1060), never applied
  wang_hash(&seed);
  // Cranley-Patterson shift (:497-515): per-pixel constant
  uint32_t ps = ((uint32_t)x * 1973u + (uint32_t)y * 9277u + (uint32_t)(114514 / 1919) * 26699u) | 1u;
  float cpu = u32_to_unit(wang_hash(&ps));
  float cpv = u32_to_unit(wang_hash(&ps));

  float pixx = (float)(2 * x + 1) / (float)p.W - 1.0f;
  float pixy = (float)(2 * y + 1) / (float)p.H - 1.0f;
  if (p.aspect_corrected) pixx = pixx * ((float)p.W / (float)p.H);
  const float* m = p.camRot;
  v3 S = mk(p.eye[0], p.eye[1], p.eye[2]);
  v3 d = normalize(mk((m[0] * pixx + m[4] * pixy) + (m[8] * -1.0f + m[12] * 0.0f),
                      (m[1] * pixx + m[5] * pixy) + (m[9] * -1.0f + m[13] * 0.0f),
                      (m[2] * pixx + m[6] * pixy) + (m[10] * -1.0f + m[14] * 0.0f)));
  v3 light = splat(0.0f), red = splat(1.0f);
  v3 firstE = splat(0.0f), firstA = splat(0.0f);

  for (int i = 0; i < p.max_depth; ++i) {
    float t;
    int tri = traverse<0>(p.scene, s, S, d, 0.0f, p.prune, &t);
    if (tri < 0) {
      light = add(light, mul(hdr_color(p, d), red));
      break;
    }
    Hit h = decode_hit(p.scene, tri, t, S, d);
    if (i == 0) { firstE = h.m.emissive; firstA = h.m.baseColor; }
    float xi1 = p.sobol_u[i] + cpu;
    if (xi1 > 1.0f) xi1 -= 1.0f;
    if (xi1 < 0.0f) xi1 += 1.0f;
    float xi2 = p.sobol_v[i] + cpv;
    if (xi2 > 1.0f) xi2 -= 1.0f;
    if (xi2 < 0.0f) xi2 += 1.0f;
    float xi3 = u32_to_unit(wang_hash(&seed));
    v3 V = neg(h.viewDir);
    v3 L = sample_brdf(xi1, xi2, xi3, V, h.normal, h.m);
    if (dot(h.normal, L) <= 0.0f) break;

    // shade (:948-968)
    v3 brdf = brdf_eval(V, h.normal, L, h.m);
    float bpdf = brdf_pdf(V, h.normal, L, h.m);
    // hdriLight (:922-946)
    float r1 = u32_to_unit(wang_hash(&seed));
    float r2 = u32_to_unit(wang_hash(&seed));
    v3 hd = sample_hdr(p, r1, r2);
    float hpdf = 0.0f;
    v3 hcalc = splat(0.0f);
    {
      float ts;
      if (traverse<1>(p.scene, s, h.P, hd, 0.0f, 0, &ts) < 0) {
        v3 hv = hdr_color(p, hd);
        v3 hb = brdf_eval(V, h.normal, hd, h.m);
        hpdf = hdr_pdf(p, hd);
        hcalc = divs(mul(muls(hb, f_abs(dot(hd, h.normal))), hv), hpdf);
      }
    }
    // calculatePointLight (:884-919)
    float ppdf = 0.0f;
    v3 pcalc = splat(0.0f);
    if (p.pointLightSize != 0) {
      ppdf = (2.0f * PT_PI) / (float)p.pointLightSize;
      int li = (int)(u32_to_unit(wang_hash(&seed)) * (float)p.pointLightSize);
      v3 lpos = splat(0.0f), lrad = splat(0.0f);
      if (li >= 0 && li < p.scene.nlights_buf) {  // out-of-range texelFetch reads 0
        const float* lp = p.scene.lights + 6 * li;
        lpos = mk(lp[0], lp[1], lp[2]);
        lrad = mk(lp[3], lp[4], lp[5]);
      }
      v3 ld = normalize(sub(lpos, h.P));
      float dist = length(sub(lpos, h.P));
      float ts;
      if (traverse<2>(p.scene, s, h.P, ld, dist, 0, &ts) < 0) {
        v3 plv = divs(lrad, dist * dist);
        v3 pb = brdf_eval(V, h.normal, ld, h.m);
        pcalc = divs(muls(mul(plv, pb), f_abs(dot(ld, h.normal))), ppdf);
      }
    }
    v3 cosb = muls(brdf, f_abs(dot(L, h.normal)));
    v3 bcalc = divs(mul(h.m.emissive, cosb), bpdf);
    float sw = ((hpdf + ppdf) + bpdf) + 1e-6f;
    float w1 = hpdf / sw, w2 = ppdf / sw, w3 = bpdf / sw;
    v3 hitLight = mul(red, add(add(muls(hcalc, w1), muls(pcalc, w2)), muls(bcalc, w3)));
    red = mul(red, divs(cosb, bpdf));
    light = add(light, hitLight);
    S = h.P;
    d = L;
  }
  light = vclamp(light, 0.0f, p.clamp_threshold);
  v3 color = splat(0.0f);
  if (!f_isnan(light.x) && !f_isnan(light.y) && !f_isnan(light.z)) color = light;
  if (p.accumulate && p.last.p) {  // :1116-1119
    float4 lc = pld(p.last, x, y);
    color = mixv(xyz(lc), color, 1.0f / (float)(p.frameCounter + 1u));
  }
  pst(p.color, x, y, f4(color.x, color.y, color.z, 1.0f));
  pst(p.emission, x, y, f4(firstE.x, firstE.y, firstE.z, 1.0f));
  pst(p.albedo, x, y, f4(firstA.x, firstA.y, firstA.z, 1.0f));
}

// --------------------------------------------------------------- G-buffer ---
struct MTr {
  float t, u, v;
  bool ok;
};
__device__ __forceinline__ MTr moller(v3 p1, v3 e1, v3 e2, v3 o, v3 d, bool bounds) {
  MTr r;
  r.ok = false;
  r.t = r.u = r.v = 0.0f;
  v3 pvec = cross(d, e2);
  float det = dot(e1, pvec);
  if (det > -1e-12f && det < 1e-12f) return r;
  float inv = 1.0f / det;
  v3 tvec = sub(o, p1);
  r.u = dot(tvec, pvec) * inv;
  v3 qvec = cross(tvec, e1);
  r.v = dot(d, qvec) * inv;
  r.t = dot(e2, qvec) * inv;
  if (bounds) {
    if (r.u < 0.0f || r.u > 1.0f) return r;
    if (r.v < 0.0f || r.u + r.v > 1.0f) return r;
    if (!(r.t > 0.0f)) return r;
  }
  r.ok = true;
  return r;
}
__device__ __forceinline__ bool gb_box(v3 o, v3 inv, float ax, float ay, float az, float bx, float by, float bz,
                                       float lim, float* t0o) {
  // NaN slabs (0 * inf) leave the interval unchanged, as in the oracle's test
  float t0 = 0.0f, t1 = lim;
  const float lo[3] = {ax, ay, az}, hi[3] = {bx, by, bz}, oo[3] = {o.x, o.y, o.z}, ii[3] = {inv.x, inv.y, inv.z};
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    float ta = (lo[a] - oo[a]) * ii[a], tb = (hi[a] - oo[a]) * ii[a];
    if (ta > tb) { float tt = ta; ta = tb; tb = tt; }
    ta -= 1e-4f * (f_abs(ta) + 1.0f);
    tb += 1e-4f * (f_abs(tb) + 1.0f);
    t0 = ta > t0 ? ta : t0;
    t1 = tb < t1 ? tb : t1;
  }
  *t0o = t0;
  return t0 <= t1;
}
__device__ __forceinline__ v3 gb_dir(const GBufParams& p, int x, int y) {
  float px = (float)(2 * x + 1) / (float)p.W - 1.0f;
  float py = (float)(2 * y + 1) / (float)p.H - 1.0f;
  float dc0 = px / p.P00, dc1 = py / p.P11, dc2 = -1.0f;
  const float* R = p.invR;
  return mk((R[0] * dc0 + R[1] * dc1) + R[2] * dc2, (R[3] * dc0 + R[4] * dc1) + R[5] * dc2,
            (R[6] * dc0 + R[7] * dc1) + R[8] * dc2);
}
__device__ __forceinline__ void mat_vec4(const float* m, v3 P, float* o) {
  for (int r = 0; r < 4; ++r) o[r] = (m[r] * P.x + m[4 + r] * P.y) + (m[8 + r] * P.z + m[12 + r] * 1.0f);
}
__device__ __forceinline__ float lin_z(const GBufParams& p, v3 P) {
  float c[4];
  mat_vec4(p.M, P, c);
  float zw = (c[2] / c[3]) * 0.5f + 0.5f;
  float fw = 1.0f / c[3];
  return zw / fw;
}

// The G-buffer texels of pixel (x, y) from its closest front-facing hit (bests: geom index, best: t, (bu, bv):
// barycentrics; bests < 0: background) and the wave's motion bound. Called by the whole wave (invalid lanes too).
__device__ __forceinline__ void gb_finish(const GBufParams& p, int x, int y, bool valid, int ln, v3 o, v3 d,
                                          float best, int bests, float bu, float bv) {
  if (p.motion_max) {  // band planning (pt_pass_set_motion_bound): wave max of |motion.y|, one atomic per wave
    float mv = 0.0f;
    if (valid && bests >= 0) {  // the motion written below, recomputed for this lane
      const v3 P = add(o, muls(d, best));
      float c[4], pc[4];
      mat_vec4(p.M, P, c);
      mat_vec4(p.PV, P, pc);
      mv = f_abs(((c[1] / c[3]) * 0.5f + 0.5f) - ((pc[1] / pc[3]) * 0.5f + 0.5f));
      if (!(mv <= 3.0e38f)) mv = __builtin_inff();  // NaN / inf: unbounded
    }
    uint32_t mb = __float_as_uint(mv);  // non-negative floats order as their bits
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) mb = max(mb, (uint32_t)__shfl_xor((int)mb, s));
    if (ln == 0 && mb) atomicMax(p.motion_max, mb);
  }
  if (!valid) return;
  if (bests < 0) {
    float4 bg = f4(0.2f, 0.3f, 0.3f, 1.0f);  // glClearColor (main.cpp:62)
    pst(p.world, x, y, bg);
    pst(p.normal_depth, x, y, bg);
    pst(p.motion, x, y, bg);
    pst(p.fwidth, x, y, bg);
    if (p.fwidth_aux) p.fwidth_aux[(size_t)prow(p.fwidth, y) * p.W + x] = -0.3f;  // .y with the zCenter == 1 flag
    return;
  }
  const float4* g = p.geom + 4 * bests;
  const float4* gn = p.nrm + 3 * bests;
  v3 p1 = xyz(g[0]), e1 = xyz(g[1]), e2 = xyz(g[2]);
  v3 n1 = xyz(gn[0]), n2 = xyz(gn[1]), n3 = xyz(gn[2]);
  auto interp = [&](float u, float v) {
    float w0 = (1.0f - u) - v;
    return add(add(muls(n1, w0), muls(n2, u)), muls(n3, v));
  };
  v3 P = add(o, muls(d, best));
  v3 N = interp(bu, bv);
  float lz = lin_z(p, P);
  float c[4], pc[4];
  mat_vec4(p.M, P, c);
  mat_vec4(p.PV, P, pc);
  float nowx = (c[0] / c[3]) * 0.5f + 0.5f, nowy = (c[1] / c[3]) * 0.5f + 0.5f;
  float prex = (pc[0] / pc[3]) * 0.5f + 0.5f, prey = (pc[1] / pc[3]) * 0.5f + 0.5f;
  v3 dx = gb_dir(p, x ^ 1, y), dy = gb_dir(p, x, y ^ 1);
  MTr hx = moller(p1, e1, e2, o, dx, false), hy = moller(p1, e1, e2, o, dy, false);
  v3 Nx = interp(hx.u, hx.v), Ny = interp(hy.u, hy.v);
  float zx = lin_z(p, add(o, muls(dx, hx.t)));
  float zy = lin_z(p, add(o, muls(dy, hy.t)));
  v3 fwN = add(mk(f_abs(Nx.x - N.x), f_abs(Nx.y - N.y), f_abs(Nx.z - N.z)),
               mk(f_abs(Ny.x - N.x), f_abs(Ny.y - N.y), f_abs(Ny.z - N.z)));
  float fwz = f_max(f_abs(zx - lz), f_abs(zy - lz));
  pst(p.world, x, y, f4(P.x, P.y, P.z, 1.0f));
  pst(p.normal_depth, x, y, f4(N.x, N.y, N.z, lz));
  pst(p.motion, x, y, f4(nowx - prex, nowy - prey, 0.0f, 1.0f));
  pst(p.fwidth, x, y, f4(length(fwN), fwz, lz, 1.0f));
  if (p.fwidth_aux)  // .y, sign bit = (linearZ == 1.0): the a-trous background test (svgf_Atrous.frag:77)
    p.fwidth_aux[(size_t)prow(p.fwidth, y) * p.W + x] =
        __uint_as_float(__float_as_uint(fwz) | (lz == 1.0f ? 0x80000000u : 0u));
  // the a-trous tiles holding this surface pixel (their background-only peers copy without reading their flags)
  if (p.tflags && lz != 1.0f && y >= p.tf_y0 && y < p.tf_y1) atrous_mark_tiles(p.tflags, p.tf_off, p.W, x, y - p.tf_y0);
}

// One 16 x 16 tile per slot; a block takes slots blockIdx.x, + gridDim.x, ... (ntx tiles per row, nslots tiles). As
// the rasteriser's overflow fallback (p.bins.ctr set) it has work only after an overflow and launches a few hundred
// blocks (launch_gbuffer): one block per tile, each reading one flag and leaving, held its stream for ~0.14 ms of a
// 4K frame.
template <int KS>
__global__ void __launch_bounds__(kBlock) gbuffer_kernel(GBufParams p, int ntx, int nslots) {
  __shared__ int stk[KS * kBlock];
  if (p.bins.ctr && p.bins.ctr[2] == 0) return;  // the rasteriser's fallback, not needed
  for (int b = blockIdx.x; b < nslots; b += gridDim.x) {
  // the overflowed frame skipped the scatter, which returns every tile count to zero: clear them here
  if (p.bins.ctr && threadIdx.x == 0) p.bins.tile_count[b] = 0;
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  const int tile = sched_tile(p.tiles, b);  // cost-ordered dispatch
  const int tx = tile % ntx, ty = tile / ntx;
  const int x = tx * 16 + (wv & 1) * 8 + (ln & 7);
  const int y = p.y0 + ty * 16 + (wv >> 1) * 8 + (ln >> 3);
  const bool valid = x < p.W && y < p.y1;
  v3 o = mk(p.eye[0], p.eye[1], p.eye[2]);
  v3 d = gb_dir(p, x, y);
  v3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  float best = 3.0e38f;
  int besti = -1, bests = -1;
  float bu = 0.f, bv = 0.f;
  uint32_t steps = 0;
  // while-while walk with one postponed leaf per lane (as traverse<>): the result
  // (closest t, ties to the lower original index) does not depend on visit order
  int sp = 0, node = valid ? p.root_ref : kNone, leaf = kNone;
  if (node < 0) { leaf = node; node = kNone; }
  while (node != kNone || leaf != kNone) {
    while (node >= 0) {
      ++steps;
      const float4* nd = p.bvh + 4 * node;
      float4 q0 = nd[0], q1 = nd[1], q2 = nd[2], q3 = nd[3];
      // conservative (widened) slab test: the box only culls, Moller-Trumbore decides
      float lim = best * 1.0002f + 2.0e-4f;
      float t0l, t0r;
      bool hl = gb_box(o, inv, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, lim, &t0l);
      bool hr = gb_box(o, inv, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, lim, &t0r);
      int cl = __float_as_int(q3.x), cr = __float_as_int(q3.y);
      if (hl && hr) {
        int nearc = (t0l < t0r) ? cl : cr, farc = (t0l < t0r) ? cr : cl;
        stk[sp * kBlock + threadIdx.x] = farc;
        ++sp;
        node = nearc;
      } else if (hl) {
        node = cl;
      } else if (hr) {
        node = cr;
      } else {
        node = sp > 0 ? stk[--sp * kBlock + threadIdx.x] : kNone;
      }
      if (node < 0 && node != kNone && leaf == kNone) {
        leaf = node;
        node = sp > 0 ? stk[--sp * kBlock + threadIdx.x] : kNone;
      }
      if (!__any(leaf == kNone)) break;
    }
    while (leaf != kNone) {
      int first = ref_leaf_first(leaf), cnt = ref_leaf_count(leaf);
      steps += (uint32_t)cnt;
      for (int i = first; i < first + cnt; ++i) {
        const float4* g = p.geom + 4 * i;
        float4 a = g[0], e1 = g[1], e2 = g[2], ng = g[3];
        v3 p1 = xyz(a);
        if (!(dot(xyz(ng), sub(p1, o)) < 0.0f)) continue;  // back face culled (GL_BACK, CCW front)
        MTr h = moller(p1, xyz(e1), xyz(e2), o, d, true);
        if (!h.ok) continue;
        int oi = __float_as_int(a.w);
        if (h.t < best || (h.t == best && oi < besti)) {
          best = h.t;
          besti = oi;
          bests = i;
          bu = h.u;
          bv = h.v;
        }
      }
      leaf = kNone;
      if (node < 0 && node != kNone) {
        leaf = node;
        node = sp > 0 ? stk[--sp * kBlock + threadIdx.x] : kNone;
      }
    }
  }
  sched_cost(p.tiles, tile, steps);
  gb_finish(p, x, y, valid, ln, o, d, best, bests, bu, bv);
  }
}

// ------------------------------------------------------- tile binning ---
// Generic stages of the tile rasterisers (Bins, pt_device.h); the item-specific setup kernel runs first.
constexpr int kRChunk = 256;     // items staged in LDS per round of a resolve
constexpr int kLargeBlocks = 512;

// large items: one block strides over each one's tiles. SCATTER 0 counts, 1 writes the list entries.
template <int SCATTER>
__global__ void __launch_bounds__(256) bins_large(Bins b) {
  if (SCATTER && b.ctr[2]) return;
  const int nlarge = min(b.ctr[0], b.large_cap);
  const int ntx = (b.W + kRTile - 1) / kRTile;
  for (int q = blockIdx.x; q < nlarge; q += gridDim.x) {
    const int i = b.large[q];
    const TileBox tb = tile_box(b, b.box[i]);
    const int w = tb.tx1 - tb.tx0 + 1, n = tb.area();
    for (int k = threadIdx.x; k < n; k += 256) {
      const int tile = (tb.ty0 + k / w) * ntx + tb.tx0 + k % w;
      if (SCATTER) b.pairs[b.tile_off[tile] + atomicSub(&b.tile_count[tile], 1) - 1] = i;
      else atomicAdd(&b.tile_count[tile], 1);
    }
  }
}

// one block: exclusive scan of the per-tile counts (tile_off[ntiles] = pairs); overflow if they exceed the list.
// 4096 counts per round: 4 consecutive per thread, wave prefix sums by shuffles, 16 wave totals through LDS, a
// carry between rounds.
__global__ void __launch_bounds__(1024) bins_scan(Bins bn, int ntiles) {
  __shared__ int wsum[16];
  __shared__ int carry_s;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (t == 0) carry_s = 0;
  __syncthreads();
  for (int base = 0; base < ntiles; base += 4096) {
    const int i0 = base + 4 * t;
    int c[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) c[k] = i0 + k < ntiles ? bn.tile_count[i0 + k] : 0;
    const int mine = c[0] + c[1] + c[2] + c[3];
    int inc = mine;  // inclusive wave scan
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(inc, o);
      if (lane >= o) inc += v;
    }
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    int before = carry_s;
    for (int w = 0; w < wv; ++w) before += wsum[w];
    int run = before + inc - mine;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (i0 + k < ntiles) bn.tile_off[i0 + k] = run;
      run += c[k];
    }
    __syncthreads();
    if (t == 1023) carry_s = run;  // the last thread's running sum: this round's total plus the carry
    __syncthreads();
  }
  if (t == 0) {
    const int total = carry_s;
    bn.tile_off[ntiles] = total;
    bn.ctr[1] = total;
    if (total > bn.pair_cap) atomicOr(&bn.ctr[2], 1);
  }
}

// per small item: its index into each covered tile's list (slot order within a tile is arbitrary)
__global__ void __launch_bounds__(256) bins_scatter(Bins b) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= b.n || b.ctr[2]) return;
  const int4 box = b.box[i];
  if (box.x > box.z || box.y > box.w) return;
  const TileBox tb = tile_box(b, box);
  if (tb.area() > kLargeTiles) return;
  const int ntx = (b.W + kRTile - 1) / kRTile;
  for (int ty = tb.ty0; ty <= tb.ty1; ++ty)
    for (int tx = tb.tx0; tx <= tb.tx1; ++tx) {
      const int tile = ty * ntx + tx;
      b.pairs[b.tile_off[tile] + atomicSub(&b.tile_count[tile], 1) - 1] = i;
    }
}

int launch_bins(const Bins& b, hipStream_t s) {
  const int ntiles = ((b.W + kRTile - 1) / kRTile) * ((b.y1 - b.y0 + kRTile - 1) / kRTile);
  if (b.n > 0) hipLaunchKernelGGL(bins_large<0>, dim3(kLargeBlocks), dim3(256), 0, s, b);
  hipLaunchKernelGGL(bins_scan, dim3(1), dim3(1024), 0, s, b, ntiles);
  if (b.n > 0) {
    hipLaunchKernelGGL(bins_scatter, dim3((b.n + 255) / 256), dim3(256), 0, s, b);
    hipLaunchKernelGGL(bins_large<1>, dim3(kLargeBlocks), dim3(256), 0, s, b);
  }
  return (int)hipGetLastError();
}

// ------------------------------------------------- G-buffer by tile binning ---
// The same G-buffer (closest front-facing Moller hit of the pixel-centre ray, ties to the lower triangle index;
// gb_finish for the texels) computed without a per-pixel BVH walk: every front-facing triangle is binned to the
// 16 x 16 tiles its screen box covers, and each pixel runs the exact Moller test of gbuffer_kernel against the
// triangles of its tile. The winner is the lexicographic minimum of (t, original index) over every triangle whose
// Moller test accepts the ray — the ray cast's answer whatever the order, provided each such triangle reaches the
// pixel's tile. The box: the triangle clipped in clip space to the view frustum's four side planes (widened by
// 1 %; every pixel-centre ray with t > 0 lies inside, so the clipped-away part meets no such ray — and a triangle
// with nothing left is dropped), projected, widened by kBoxMargin pixels (projection and ray arithmetic agree
// to far below a pixel). A clipped vertex on the camera plane (the triangle passes through the eye) makes the
// box the whole band. No walk means no tail: a tile costs about as much as it holds triangles.

// per triangle: back-face cull, box, bound, binning counts
__global__ void __launch_bounds__(256) rast_setup(GBufParams p) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= p.bins.n) return;
  const float4* g = p.geom + 4 * i;
  const float4 a = g[0], e1 = g[1], e2 = g[2], ng = g[3];
  const v3 o = mk(p.eye[0], p.eye[1], p.eye[2]);
  const v3 p1 = xyz(a);
  int4 box = make_int4(1, 1, 0, 0);  // empty
  float tmin = 0.0f;
  if (dot(xyz(ng), sub(p1, o)) < 0.0f) {  // front-facing: gbuffer_kernel's back-face cull
    const v3 v[3] = {p1, add(p1, xyz(e1)), add(p1, xyz(e2))};
    float3 A[16];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      float c[4];
      mat_vec4(p.M, v[k], c);
      A[k] = make_float3(c[0], c[1], c[3]);
    }
    // the pixel rays' direction has camera-space z = -1, so a hit's t is its clip w, which is linear over the
    // (clipped) triangle: no hit lies nearer than the smallest vertex w (margin for the rounding of both)
    if (poly_box(p.bins, p.H, A, 3, 1.0f, 1.0f, &box, &tmin)) tmin *= 0.9999f;
  }
  bins_count_item(p.bins, i, box, tmin);
}

// one block per tile: the tile's list staged through LDS, every pixel's Moller tests, gb_finish
__global__ void __launch_bounds__(kBlock) gbuffer_raster_kernel(GBufParams p) {
  __shared__ float4 sg[kRChunk * 3];
  __shared__ int4 sbox[kRChunk];
  __shared__ int sidx[kRChunk];
  __shared__ float stmin[kRChunk];
  const Bins& bn = p.bins;
  if (bn.ctr[2]) return;  // overflow: gbuffer_kernel (the ray cast) writes the frame
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  const int tile = blockIdx.y * gridDim.x + blockIdx.x;
  const int x = blockIdx.x * 16 + (wv & 1) * 8 + (ln & 7);
  const int y = p.y0 + blockIdx.y * 16 + (wv >> 1) * 8 + (ln >> 3);
  const bool valid = x < p.W && y < p.y1;
  const v3 o = mk(p.eye[0], p.eye[1], p.eye[2]);
  const v3 d = gb_dir(p, x, y);
  float best = 3.0e38f, bu = 0.0f, bv = 0.0f;
  int besti = -1, bests = -1;
  const int off = bn.tile_off[tile], total = bn.tile_off[tile + 1] - off;
  for (int base = 0; base < total; base += kRChunk) {
    __syncthreads();
    const int j = base + (int)threadIdx.x;
    if (j < total) {
      const int tri = bn.pairs[off + j];
      const float4* g = p.geom + 4 * tri;
      sg[3 * threadIdx.x] = g[0];
      sg[3 * threadIdx.x + 1] = g[1];
      sg[3 * threadIdx.x + 2] = g[2];
      sbox[threadIdx.x] = bn.box[tri];
      sidx[threadIdx.x] = tri;
      stmin[threadIdx.x] = bn.tmin[tri];
    }
    __syncthreads();
    const int n = min(kRChunk, total - base);
    if (!valid) continue;
    for (int k = 0; k < n; ++k) {
      const int4 b = sbox[k];
      if (x < b.x || x > b.z || y < b.y || y > b.w) continue;  // outside the triangle's widened screen box
      if (stmin[k] > best) continue;                             // wholly behind this pixel's closest hit so far
      const float4 a = sg[3 * k];
      const MTr h = moller(xyz(a), xyz(sg[3 * k + 1]), xyz(sg[3 * k + 2]), o, d, true);
      if (!h.ok) continue;
      const int oi = __float_as_int(a.w);
      if (h.t < best || (h.t == best && oi < besti)) {
        best = h.t;
        besti = oi;
        bests = sidx[k];
        bu = h.u;
        bv = h.v;
      }
    }
  }
  gb_finish(p, x, y, valid, ln, o, d, best, bests, bu, bv);
}

// A G-buffer whose planes another process wrote (multi-GPU frame shard: the rank tracing the frame drew these rows of
// it and sent them): the side data a draw makes beside its planes, from the planes — the compact depth-fwidth plane
// (fwidth.y with the sign bit = linearZ == 1, exactly as gb_finish writes it) and the a-trous tile flags of rows
// [tf_y0, tf_y1). One thread per pixel of rows [y0, y1).
__global__ void __launch_bounds__(256) gbuffer_adopt_kernel(GBufParams p) {
  const int x = blockIdx.x * 64 + (int)(threadIdx.x & 63);
  const int y = p.y0 + (int)blockIdx.y * 4 + (int)(threadIdx.x >> 6);
  if (x >= p.W || y >= p.y1) return;
  const float lz = pld(p.normal_depth, x, y).w;
  const float fwz = pld(p.fwidth, x, y).y;
  if (p.fwidth_aux)
    p.fwidth_aux[(size_t)prow(p.fwidth, y) * p.W + x] = __uint_as_float(__float_as_uint(fwz) | (lz == 1.0f ? 0x80000000u : 0u));
  if (p.tflags && lz != 1.0f && y >= p.tf_y0 && y < p.tf_y1) atrous_mark_tiles(p.tflags, p.tf_off, p.W, x, y - p.tf_y0);
}

int launch_gbuffer_adopt(const GBufParams& p, hipStream_t s) {
  if (p.y1 <= p.y0) return 0;
  hipLaunchKernelGGL(gbuffer_adopt_kernel, dim3((p.W + 63) / 64, (p.y1 - p.y0 + 3) / 4), dim3(256), 0, s, p);
  return (int)hipGetLastError();
}

int launch_gbuffer_raster(const GBufParams& p, hipStream_t s) {
  if (p.y1 <= p.y0) return 0;
  const int ntx = (p.W + kRTile - 1) / kRTile, nty = (p.y1 - p.y0 + kRTile - 1) / kRTile;
  if (p.bins.n > 0) hipLaunchKernelGGL(rast_setup, dim3((p.bins.n + 255) / 256), dim3(256), 0, s, p);
  int rc = launch_bins(p.bins, s);
  if (rc) return rc;
  hipLaunchKernelGGL(gbuffer_raster_kernel, dim3(ntx, nty), dim3(kBlock), 0, s, p);
  // the ray cast runs only if a list overflowed (it reads the flag and returns otherwise)
  return launch_gbuffer(p, s);
}

// The merged environment texture (PTParams::hdr_pdf): per texel hdrMap's radiance and hdrCache's pdf channel.
__global__ void __launch_bounds__(256) hdr_merge_kernel(const float4* __restrict__ hdr, const float4* __restrict__ cache,
                                                        float4* __restrict__ out, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float4 h = hdr[i];
  out[i] = make_float4(h.x, h.y, h.z, cache[i].z);
}
int launch_hdr_merge(const float4* hdr, const float4* cache, float4* out, int n, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(hdr_merge_kernel, dim3((n + 255) / 256), dim3(256), 0, s, hdr, cache, out, n);
  return (int)hipGetLastError();
}

int launch_pathtrace(const PTParams& p, hipStream_t s) {
  if (p.y1 <= p.y0) return 0;
  dim3 grid((p.W + 15) / 16, (p.y1 - p.y0 + 15) / 16);
  hipLaunchKernelGGL(pathtrace_kernel, grid, dim3(kBlock), 0, s, p);
  return (int)hipGetLastError();
}
// the fallback's grid (PTSVGF_GBUFFER_FIX_BLOCKS, read once; 0 = one block per tile, as until round 6)
static int gbuffer_fix_blocks() {
  static const int n = [] {
    const char* e = getenv("PTSVGF_GBUFFER_FIX_BLOCKS");
    return e ? std::max(0, atoi(e)) : 512;
  }();
  return n;
}
int launch_gbuffer(const GBufParams& p, hipStream_t s) {
  if (p.y1 <= p.y0) return 0;
  const int ntx = (p.W + 15) / 16, nslots = ntx * ((p.y1 - p.y0 + 15) / 16);
  const int fix = p.bins.ctr ? gbuffer_fix_blocks() : 0;
  const dim3 grid(fix > 0 ? std::min(nslots, fix) : nslots);
  if (p.stack_need <= kStackSmall)
    hipLaunchKernelGGL(gbuffer_kernel<kStackSmall>, grid, dim3(kBlock), 0, s, p, ntx, nslots);
  else hipLaunchKernelGGL(gbuffer_kernel<kStack>, grid, dim3(kBlock), 0, s, p, ntx, nslots);
  return (int)hipGetLastError();
}

}  // namespace ptk

// kernels_svgf.hip — SVGF denoise chain for gfx950: reprojection, variance
// estimate, edge-stopping a-trous (x5 by the caller), albedo re-modulation and
// the output tonemap. One thread per pixel; planes are RGBA32F (16-B loads).
//
// Reference shaders (behaviour restated, GLSL file:line):
//   reproject  shaders/svgf_reproject.frag:26-204
//   variance   shaders/svgf_variance.frag:18-117
//   a-trous    shaders/svgf_Atrous.frag:20-126
//   modulate   shaders/svgf_modulate.frag:18-29
//   output     shaders/output_pass.frag:12-24
//
// Exactness: built with -ffp-contract=off and the GLSL built-ins of
// glsl_builtins.h, so these kernels reproduce the CPU oracle bit for bit. The
// production a-trous (atrous_fast_kernel, kernels_atrous.hip) trades the
// built-in pow/exp for the hardware exp2/log2 and is checked within tolerance.
#include <hip/hip_runtime.h>

#include "glsl_builtins.h"
#include "pt_device.h"

using namespace glsl;

namespace ptk {

__device__ __forceinline__ int row_of(const Plane& P, int y) {
  int ly = y - P.row0;
  return ly < 0 ? 0 : (ly >= P.rows ? P.rows - 1 : ly);
}
__device__ __forceinline__ float4 ldp(const Plane& P, int x, int y) {
  return P.p[(size_t)row_of(P, y) * P.W + x];
}
__device__ __forceinline__ void stp(const Plane& P, int x, int y, float4 v) {
  P.p[(size_t)row_of(P, y) * P.W + x] = v;
}
// texture2D(LINEAR, CLAMP_TO_EDGE) on a banded plane in global uv.
__device__ __forceinline__ float4 lin(const Plane& P, int W, int H, float u, float v) {
  Bilin b = bilin_setup(u, v, W, H);
  float4 c00 = ldp(P, b.x0, b.y0), c10 = ldp(P, b.x1, b.y0), c01 = ldp(P, b.x0, b.y1), c11 = ldp(P, b.x1, b.y1);
  float4 r;
  r.x = bilin_mix(b, c00.x, c10.x, c01.x, c11.x);
  r.y = bilin_mix(b, c00.y, c10.y, c01.y, c11.y);
  r.z = bilin_mix(b, c00.z, c10.z, c01.z, c11.z);
  r.w = bilin_mix(b, c00.w, c10.w, c01.w, c11.w);
  return r;
}
__device__ __forceinline__ float uv_of(int x, int W) {
  float pix = (float)(2 * x + 1) / (float)W - 1.0f;  // vert.vert: pix = NDC of the pixel centre
  return pix * 0.5f + 0.5f;
}
__device__ __forceinline__ float lum(float r, float g, float b) { return (0.2125f * r + 0.7154f * g) + 0.0721f * b; }

__device__ __forceinline__ bool reprj_valid(float cx, float cy, float Z, float Zprev, float fwZ, v3 n, v3 np,
                                            float fwN, float dthr, float nthr) {
  if (cx < 0.0f || cx > 1.0f || cy < 0.0f || cy > 1.0f) return false;
  if (f_abs(Zprev - Z) / (fwZ + 1e-2f) > dthr) return false;
  if (distance(n, np) / (fwN + 1e-2f) > nthr) return false;
  return true;
}

// computeWeight (svgf_variance.frag:23-35, svgf_Atrous.frag:43-55)
__device__ __forceinline__ float edge_weight(float zc, float zp, float phiDepth, v3 nc, v3 np, float phiNormal,
                                             float lc, float lp, float phiIllum) {
  float wN = g_pow(f_clamp(dot(nc, np), 0.0f, 1.0f), phiNormal);
  float wZ = (phiDepth == 0.0f) ? 0.0f : f_abs(zc - zp) / phiDepth;
  float wL = f_abs(lc - lp) / phiIllum;
  return g_exp((0.0f - f_max(wL, 0.0f)) - f_max(wZ, 0.0f)) * wN;
}

// ------------------------------------------------------------ reproject ---
#ifndef PT_REPROJ_WAVES
#define PT_REPROJ_WAVES 0  // waves/SIMD reproject_kernel is compiled for (0: the compiler's choice, 94 VGPRs = 5 waves)
#endif
#if PT_REPROJ_WAVES > 0
#define PT_REPROJ_ATTR __attribute__((amdgpu_waves_per_eu(PT_REPROJ_WAVES)))
#else
#define PT_REPROJ_ATTR
#endif
// The bilinear fetch of tap (OX, OY) from a 3x3 texel block B whose top-left texel is the tap (0, 0)'s (x0, y0):
// the texels lin() reads, mixed with the tap's own weights.
template <int OX, int OY>
__device__ __forceinline__ float4 lin_blk(const float4 (&B)[3][3], const Bilin& b) {
  const float4 c00 = B[OY][OX], c10 = B[OY][OX + 1], c01 = B[OY + 1][OX], c11 = B[OY + 1][OX + 1];
  float4 r;
  r.x = bilin_mix(b, c00.x, c10.x, c01.x, c11.x);
  r.y = bilin_mix(b, c00.y, c10.y, c01.y, c11.y);
  r.z = bilin_mix(b, c00.z, c10.z, c01.z, c11.z);
  r.w = bilin_mix(b, c00.w, c10.w, c01.w, c11.w);
  return r;
}
__device__ __forceinline__ void load_blk(const Plane& P, int X, int Y, float4 (&B)[3][3]) {
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int i = 0; i < 3; ++i) B[j][i] = ldp(P, X + i, Y + j);
}
template <int K>
__device__ __forceinline__ float4 lin_tap(const float4 (&B)[3][3], const Bilin& b) {
  return lin_blk<(K & 1), (K >> 1)>(B, b);
}

__global__ void __launch_bounds__(256) PT_REPROJ_ATTR reproject_kernel(ReprojParams p) {
  int x = blockIdx.x * 16 + (threadIdx.x & 15);
  int y = p.y0 + blockIdx.y * 16 + (threadIdx.x >> 4);
  if (x >= p.W || y >= p.y1) return;
  const int W = p.W, H = p.H;
  float uvx = uv_of(x, W), uvy = uv_of(y, H);
  float4 cnd = ldp(p.nd, x, y);
  if (cnd.w == 1.0f) {  // background sentinel (glClearColor .w = 1)
    stp(p.out_illum, x, y, ldp(p.color, x, y));
    stp(p.out_moments, x, y, ldp(p.prev_moments, x, y));
    return;
  }
  float4 c = ldp(p.color, x, y), e = ldp(p.emission, x, y), a = ldp(p.albedo, x, y);
  v3 illum = mk((c.x - e.x) / f_max(a.x, 0.001f), (c.y - e.y) / f_max(a.y, 0.001f), (c.z - e.z) / f_max(a.z, 0.001f));
  if (f_isnan(illum.x) || f_isnan(illum.y) || f_isnan(illum.z)) illum = splat(0.0f);

  float4 mo = ldp(p.motion, x, y);
  float4 fw = ldp(p.fwidth, x, y);
  float ipx = uvx - mo.x, ipy = uvy - mo.y;
  v3 n = mk(cnd.x, cnd.y, cnd.z);
  float z = cnd.w;
  float pI[4] = {0.f, 0.f, 0.f, 0.f}, pM[2] = {0.f, 0.f};
  const float ox[4] = {0.0f, p.inv_w, 0.0f, p.inv_w};
  const float oy[4] = {0.0f, 0.0f, p.inv_h, p.inv_h};
  // the four history taps (+0/+1 texel in x and y, svgf_reproject.frag:99-125): lin()'s setups, once
  Bilin bt[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) bt[k] = bilin_setup(ipx + ox[k], ipy + oy[k], W, H);
  // when they tile one 3x3 block (no clamping, each tap one texel on from tap 0), every plane's 16 texel reads are
  // its 9 block texels: load them once (same texels, same weights, same bits as lin per tap)
  const int X = bt[0].x0, Y = bt[0].y0;
  const bool blk = p.block && bt[0].x1 == X + 1 && bt[0].y1 == Y + 1 && X + 2 < W && Y + 2 < H &&
                   bt[1].x0 == X + 1 && bt[1].y0 == Y && bt[2].x0 == X && bt[2].y0 == Y + 1 &&
                   bt[3].x0 == X + 1 && bt[3].y0 == Y + 1;
  bool v[4];
  bool valid = false;
  float4 hq;  // the history length tap (lin(prev_moments, ipx, ipy)), from the moments block when it is loaded
  bool have_hq = false;
  if (blk) {
    {
      float4 B[3][3];
      load_blk(p.prev_nd, X, Y, B);
      const float4 q[4] = {lin_tap<0>(B, bt[0]), lin_tap<1>(B, bt[1]), lin_tap<2>(B, bt[2]), lin_tap<3>(B, bt[3])};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[k] = reprj_valid(ipx + ox[k], ipy + oy[k], z, q[k].w, fw.y, n, mk(q[k].x, q[k].y, q[k].z), fw.x,
                           p.depth_thr, p.normal_thr);
        valid = valid || v[k];
      }
    }
    if (valid) {
      float sumw = 0.0f;
      float bx = ipx - (float)f2i(ipx / p.inv_w) * p.inv_w;
      float by = ipy - (float)f2i(ipy / p.inv_h) * p.inv_h;
      const float w[4] = {(1.0f - bx) * (1.0f - by), bx * (1.0f - by), (1.0f - bx) * by, bx * by};
      {
        float4 B[3][3];
        load_blk(p.prev_illum, X, Y, B);
        const float4 q[4] = {lin_tap<0>(B, bt[0]), lin_tap<1>(B, bt[1]), lin_tap<2>(B, bt[2]), lin_tap<3>(B, bt[3])};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (!v[k]) continue;
          pI[0] += w[k] * q[k].x; pI[1] += w[k] * q[k].y; pI[2] += w[k] * q[k].z; pI[3] += w[k] * q[k].w;
        }
      }
      {
        float4 B[3][3];
        load_blk(p.prev_moments, X, Y, B);
        const float4 q[4] = {lin_tap<0>(B, bt[0]), lin_tap<1>(B, bt[1]), lin_tap<2>(B, bt[2]), lin_tap<3>(B, bt[3])};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (!v[k]) continue;
          pM[0] += w[k] * q[k].x; pM[1] += w[k] * q[k].y;
          sumw += w[k];
        }
        hq = q[0];
        have_hq = true;
      }
      valid = (sumw >= 0.01f);
      for (int q = 0; q < 4; ++q) pI[q] = valid ? pI[q] / sumw : 0.0f;
      for (int q = 0; q < 2; ++q) pM[q] = valid ? pM[q] / sumw : 0.0f;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float lx = ipx + ox[k], ly = ipy + oy[k];
      float4 q = lin(p.prev_nd, W, H, lx, ly);
      v[k] = reprj_valid(lx, ly, z, q.w, fw.y, n, mk(q.x, q.y, q.z), fw.x, p.depth_thr, p.normal_thr);
      valid = valid || v[k];
    }
    if (valid) {
      float sumw = 0.0f;
      float bx = ipx - (float)f2i(ipx / p.inv_w) * p.inv_w;
      float by = ipy - (float)f2i(ipy / p.inv_h) * p.inv_h;
      const float w[4] = {(1.0f - bx) * (1.0f - by), bx * (1.0f - by), (1.0f - bx) * by, bx * by};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (!v[k]) continue;
        float lx = ipx + ox[k], ly = ipy + oy[k];
        float4 qi = lin(p.prev_illum, W, H, lx, ly);
        float4 qm = lin(p.prev_moments, W, H, lx, ly);
        pI[0] += w[k] * qi.x; pI[1] += w[k] * qi.y; pI[2] += w[k] * qi.z; pI[3] += w[k] * qi.w;
        pM[0] += w[k] * qm.x; pM[1] += w[k] * qm.y;
        sumw += w[k];
      }
      valid = (sumw >= 0.01f);
      for (int q = 0; q < 4; ++q) pI[q] = valid ? pI[q] / sumw : 0.0f;
      for (int q = 0; q < 2; ++q) pM[q] = valid ? pM[q] / sumw : 0.0f;
    }
  }
  if (!valid) {
    float nValid = 0.0f;
    for (int yy = -1; yy <= 1; ++yy)
      for (int xx = -1; xx <= 1; ++xx) {
        float lx = ipx + (float)xx * p.inv_w, ly = ipy + (float)yy * p.inv_h;
        float4 q = lin(p.prev_nd, W, H, lx, ly);
        if (reprj_valid(lx, ly, z, q.w, fw.y, n, mk(q.x, q.y, q.z), fw.x, p.depth_thr, p.normal_thr)) {
          float4 qi = lin(p.prev_illum, W, H, lx, ly);
          float4 qm = lin(p.prev_moments, W, H, lx, ly);
          pI[0] += qi.x; pI[1] += qi.y; pI[2] += qi.z; pI[3] += qi.w;
          pM[0] += qm.x; pM[1] += qm.y;
          nValid += 1.0f;
        }
      }
    if (nValid > 0.0f) {
      valid = true;
      for (int q = 0; q < 4; ++q) pI[q] /= nValid;
      for (int q = 0; q < 2; ++q) pM[q] /= nValid;
    }
  }
  float hist;
  if (valid) {
    hist = (have_hq ? hq : lin(p.prev_moments, W, H, ipx, ipy)).z;  // tap 0's fetch: the same setup, the same texels
  } else {
    for (int q = 0; q < 4; ++q) pI[q] = 0.0f;
    pM[0] = pM[1] = 0.0f;
    hist = 0.0f;
  }
  hist = f_min(32.0f, valid ? hist + 1.0f : 1.0f);
  float alpha = valid ? f_max(0.2f, 1.0f / hist) : 1.0f;
  float m0 = lum(illum.x, illum.y, illum.z);
  float m1 = m0 * m0;
  m0 = (1.0f - alpha) * pM[0] + alpha * m0;
  m1 = (1.0f - alpha) * pM[1] + alpha * m1;
  float var = f_max(0.0f, m1 - m0 * m0);
  float4 oi, om;
  oi.x = (1.0f - alpha) * pI[0] + alpha * illum.x;
  oi.y = (1.0f - alpha) * pI[1] + alpha * illum.y;
  oi.z = (1.0f - alpha) * pI[2] + alpha * illum.z;
  oi.w = var;
  om.x = m0; om.y = m1; om.z = hist; om.w = 0.0f;
  stp(p.out_illum, x, y, oi);
  stp(p.out_moments, x, y, om);
}

// -------------------------------------------------------------- variance ---
// Per 16 x 16 block: a pixel with a long history (or the background) copies its illumination (32 B read, 16 B
// written); the 7x7 spatial estimate (svgf_variance.frag:58-110, young histories) reads its taps from the block's
// illumination, moments and normal/depth staged once in LDS with a 3-texel apron — only in blocks where some pixel
// needs it. Same taps in the same order as the per-pixel form.
constexpr int kVT = 16 + 2 * 3;
__global__ void __launch_bounds__(256) variance_kernel(VarianceParams p) {
  __shared__ float4 s_il[kVT * kVT], s_mo[kVT * kVT], s_nd[kVT * kVT];
  const int bx = blockIdx.x * 16, by = p.y0 + blockIdx.y * 16;
  const int x = bx + (threadIdx.x & 15), y = by + (threadIdx.x >> 4);
  const bool valid = x < p.W && y < p.y1;
  float h = 4.0f;
  float4 ic = make_float4(0.0f, 0.0f, 0.0f, 0.0f), nd = ic;
  bool need = false;
  if (valid) {
    h = ldp(p.moments, x, y).z;
    ic = ldp(p.illum, x, y);
    if (h < 4.0f) {
      nd = ldp(p.nd, x, y);
      need = nd.w != 1.0f;
    }
  }
  if (!__syncthreads_or(need)) {  // nothing to filter in this block
    if (valid) stp(p.out, x, y, ic);
    return;
  }
  for (int i = threadIdx.x; i < kVT * kVT; i += 256) {  // texels outside the frame are never read
    const int tx = bx - 3 + i % kVT, ty = by - 3 + i / kVT;
    if (tx >= 0 && tx < p.W && ty >= 0 && ty < p.H) {
      s_il[i] = ldp(p.illum, tx, ty);
      s_mo[i] = ldp(p.moments, tx, ty);
      s_nd[i] = ldp(p.nd, tx, ty);
    }
  }
  __syncthreads();
  if (!valid) return;
  if (!need) {
    stp(p.out, x, y, ic);
    return;
  }
  float lc = lum(ic.x, ic.y, ic.z);
  v3 nc = mk(nd.x, nd.y, nd.z);
  float phiDepth = f_max(ldp(p.fwidth, x, y).y, 1e-8f) * 3.0f;
  float sumW = 0.0f, s0 = 0.f, s1 = 0.f, s2 = 0.f, m0 = 0.f, m1 = 0.f;
  for (int yy = -3; yy <= 3; ++yy) {
    int py = y + yy;
    if (py < 0 || py >= p.H) continue;
    for (int xx = -3; xx <= 3; ++xx) {
      int px = x + xx;
      if (px < 0 || px >= p.W) continue;
      const int li = (py - (by - 3)) * kVT + (px - (bx - 3));
      float4 ip = s_il[li];
      float4 mp = s_mo[li];
      float4 q = s_nd[li];
      float len = f_sqrt((float)(xx * xx) + (float)(yy * yy));
      float w = edge_weight(nd.w, q.w, phiDepth * len, nc, mk(q.x, q.y, q.z), p.phi_normal, lc,
                            lum(ip.x, ip.y, ip.z), p.phi_color);
      sumW += w;
      s0 += ip.x * w; s1 += ip.y * w; s2 += ip.z * w;
      m0 += mp.x * w; m1 += mp.y * w;
    }
  }
  sumW = f_max(sumW, 1e-6f);
  s0 /= sumW; s1 /= sumW; s2 /= sumW; m0 /= sumW; m1 /= sumW;
  float var = m1 - m0 * m0;
  var *= 4.0f / h;
  float4 o;
  o.x = s0; o.y = s1; o.z = s2; o.w = var;
  stp(p.out, x, y, o);
}

// ------------------------------------------------- a-trous (exact form) ---
__global__ void __launch_bounds__(256) atrous_exact_kernel(AtrousParams p) {
  int x = blockIdx.x * 16 + (threadIdx.x & 15);
  int y = p.y0 + blockIdx.y * 16 + (threadIdx.x >> 4);
  if (x >= p.W || y >= p.y1) return;
  float4 ic = ldp(p.illum, x, y);
  float lc = lum(ic.x, ic.y, ic.z);
  // computeVarianceCenter reads the centre 9 times (svgf_Atrous.frag:36)
  float var = 0.0f;
  var += ic.w * (1.0f / 16.0f); var += ic.w * (1.0f / 8.0f); var += ic.w * (1.0f / 16.0f);
  var += ic.w * (1.0f / 8.0f);  var += ic.w * (1.0f / 4.0f); var += ic.w * (1.0f / 8.0f);
  var += ic.w * (1.0f / 16.0f); var += ic.w * (1.0f / 8.0f); var += ic.w * (1.0f / 16.0f);
  float4 nd = ldp(p.nd, x, y);
  if (nd.w == 1.0f) {
    stp(p.out, x, y, ic);
    return;
  }
  v3 nc = mk(nd.x, nd.y, nd.z);
  float phiL = p.phi_color * f_sqrt(f_max(0.0f, 1e-10f + var));
  float fwz = p.fwidth.aux ? fabsf(p.fwidth.aux[(size_t)row_of(p.fwidth, y) * p.fwidth.W + x]) : ldp(p.fwidth, x, y).y;
  float phiDepth = f_max(fwz, 1e-8f) * (float)p.step;
  const float kw[3] = {1.0f, 2.0f / 3.0f, 1.0f / 6.0f};
  float sumW = 1.0f;
  float s0 = ic.x, s1 = ic.y, s2 = ic.z, s3 = ic.w;
  for (int yy = -2; yy <= 2; ++yy) {
    int py = y + yy * p.step;
    for (int xx = -2; xx <= 2; ++xx) {
      int px = x + xx * p.step;
      bool inside = px >= 0 && px < p.W && py >= 0 && py < p.H;
      if (!inside || (xx == 0 && yy == 0)) continue;
      float kernel = kw[xx < 0 ? -xx : xx] * kw[yy < 0 ? -yy : yy];
      float4 ip = ldp(p.illum, px, py);
      float4 q = ldp(p.nd, px, py);
      float len = f_sqrt((float)(xx * xx) + (float)(yy * yy));
      float w = edge_weight(nd.w, q.w, phiDepth * len, nc, mk(q.x, q.y, q.z), p.phi_normal, lc,
                            lum(ip.x, ip.y, ip.z), phiL);
      float wi = w * kernel;
      sumW += wi;
      s0 += wi * ip.x; s1 += wi * ip.y; s2 += wi * ip.z;
      s3 += (wi * wi) * ip.w;
    }
  }
  float4 o;
  o.x = s0 / sumW; o.y = s1 / sumW; o.z = s2 / sumW; o.w = s3 / (sumW * sumW);
  stp(p.out, x, y, o);
}

// -------------------------------------------------------------- modulate ---
__global__ void __launch_bounds__(256) modulate_kernel(ModulateParams p) {
  int x = blockIdx.x * 16 + (threadIdx.x & 15);
  int y = p.y0 + blockIdx.y * 16 + (threadIdx.x >> 4);
  if (x >= p.W || y >= p.y1) return;
  float4 c = ldp(p.illum, x, y);
  float4 o;
  if (ldp(p.nd, x, y).w == 1.0f) {
    o.x = c.x; o.y = c.y; o.z = c.z;
  } else {
    float4 a = ldp(p.albedo, x, y), e = ldp(p.emission, x, y);
    o.x = c.x * a.x + e.x; o.y = c.y * a.y + e.y; o.z = c.z * a.z + e.z;
  }
  o.w = 1.0f;
  stp(p.out, x, y, o);
}

// ---------------------------------------------------------------- output ---
__global__ void __launch_bounds__(256) output_kernel(OutputParams p) {
  int x = blockIdx.x * 16 + (threadIdx.x & 15);
  int y = p.y0 + blockIdx.y * 16 + (threadIdx.x >> 4);
  if (x >= p.W || y >= p.y1) return;
  float4 c = ldp(p.in, x, y);
  float l = (0.3f * c.x + 0.6f * c.y) + 0.1f * c.z;
  float den = 1.0f + l / 1.5f;
  float4 o;
  o.x = g_pow((c.x * 1.0f) / den, 1.0f / 2.2f);
  o.y = g_pow((c.y * 1.0f) / den, 1.0f / 2.2f);
  o.z = g_pow((c.z * 1.0f) / den, 1.0f / 2.2f);
  o.w = 1.0f;
  stp(p.out, x, y, o);
}

static dim3 grid16(int W, int rows) { return dim3((W + 15) / 16, (rows + 15) / 16); }

int launch_reproject(const ReprojParams& p, hipStream_t s) {
  if (p.y1 <= p.y0) return 0;
  hipLaunchKernelGGL(reproject_kernel, grid16(p.W, p.y1 - p.y0), dim3(256), 0, s, p);
  return (int)hipGetLastError();
}
int launch_variance(const VarianceParams& p, hipStream_t s) {
  if (p.y1 <= p.y0) return 0;
  hipLaunchKernelGGL(variance_kernel, grid16(p.W, p.y1 - p.y0), dim3(256), 0, s, p);
  return (int)hipGetLastError();
}
int launch_atrous_exact(const AtrousParams& p, hipStream_t s) {
  if (p.y1 <= p.y0) return 0;
  hipLaunchKernelGGL(atrous_exact_kernel, grid16(p.W, p.y1 - p.y0), dim3(256), 0, s, p);
  return (int)hipGetLastError();
}
int launch_modulate(const ModulateParams& p, hipStream_t s) {
  if (p.y1 <= p.y0) return 0;
  hipLaunchKernelGGL(modulate_kernel, grid16(p.W, p.y1 - p.y0), dim3(256), 0, s, p);
  return (int)hipGetLastError();
}
int launch_output(const OutputParams& p, hipStream_t s) {
  if (p.y1 <= p.y0) return 0;
  hipLaunchKernelGGL(output_kernel, grid16(p.W, p.y1 - p.y0), dim3(256), 0, s, p);
  return (int)hipGetLastError();
}

}  // namespace ptk

// kernels_atrous.hip — production edge-stopping a-trous wavelet pass
// (shaders/svgf_Atrous.frag:61-126; driven 5x per frame with step 1<<i,
// main.cpp:499-526). HBM-bound stencil: 52 algorithmic B/px/iteration
// (illum 16 + normal/z 16 + depth-fwidth 4 + out 16).
//
// Differences from the exact form (kernels_svgf.hip::atrous_exact_kernel),
// all within the parity tolerance (tests/test_gpu_parity.py):
//  * pow(max(dot,0),phiN) * exp(-(wl+wz)) is evaluated as ONE exp2 of
//    phiN*log2(dot) - (wl+wz)*log2(e) with the hardware v_log_f32/v_exp_f32;
//  * the per-tap divisions by phiIllum / phiDepth*|offset| become multiplies by
//    per-pixel reciprocals (5 distinct |offset| values);
//  * depth fwidth comes from the compact 4-B side plane when present.
// Built with -ffp-contract=off and explicit FMAs: the checked (border) and
// unchecked (interior) instantiations must give identical bits, or a pixel's
// result would depend on which band or block it falls in.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "glsl_builtins.h"
#include "pt_device.h"

using namespace glsl;

namespace ptk {

__device__ __forceinline__ int arow(const Plane& P, int y) {
  int ly = y - P.row0;
  return ly < 0 ? 0 : (ly >= P.rows ? P.rows - 1 : ly);
}

__global__ void __launch_bounds__(256) atrous_fast_kernel(AtrousParams p) {
  const int x = blockIdx.x * 64 + (threadIdx.x & 63);
  const int y = p.y0 + blockIdx.y * 4 + (threadIdx.x >> 6);
  if (x >= p.W || y >= p.y1) return;
  const size_t W = p.illum.W;
  const float4* __restrict__ I = p.illum.p;
  const float4* __restrict__ ND = p.nd.p;
  float4 ic = I[(size_t)arow(p.illum, y) * W + x];
  float4 nd = ND[(size_t)arow(p.nd, y) * W + x];
  float4* out = p.out.p + (size_t)arow(p.out, y) * W + x;
  if (nd.w == 1.0f) {
    *out = ic;
    return;
  }
  const float LOG2E = 1.4426950408889634f;
  float lc = (0.2125f * ic.x + 0.7154f * ic.y) + 0.0721f * ic.z;
  float phiL = p.phi_color * __builtin_sqrtf(fmaxf(0.0f, 1e-10f + ic.w));  // variance: centre only (:36)
  float fwz = p.fwidth.aux ? fabsf(p.fwidth.aux[(size_t)arow(p.fwidth, y) * p.fwidth.W + x])
                           : p.fwidth.p[(size_t)arow(p.fwidth, y) * p.fwidth.W + x].y;
  float phiD = fmaxf(fwz, 1e-8f) * (float)p.step;
  float kL = LOG2E / phiL;   // exp(-a) = exp2(-a*log2e)
  float kD = LOG2E / phiD;
  // 1/|offset| for |offset|^2 = 1, 2, 4, 5, 8
  const float inv1 = 1.0f, inv2 = 0.70710678f, inv4 = 0.5f, inv5 = 0.44721360f, inv8 = 0.35355339f;
  const float kw[3] = {1.0f, 2.0f / 3.0f, 1.0f / 6.0f};
  float sumW = 1.0f, s0 = ic.x, s1 = ic.y, s2 = ic.z, s3 = ic.w;
#pragma unroll
  for (int yy = -2; yy <= 2; ++yy) {
    const int py = y + yy * p.step;
    if (py < 0 || py >= p.H) continue;
    const size_t ro = (size_t)arow(p.illum, py) * W, rn = (size_t)arow(p.nd, py) * W;
#pragma unroll
    for (int xx = -2; xx <= 2; ++xx) {
      if (xx == 0 && yy == 0) continue;
      const int px = x + xx * p.step;
      if (px < 0 || px >= p.W) continue;
      const int r2 = xx * xx + yy * yy;
      const float invlen = r2 == 1 ? inv1 : r2 == 2 ? inv2 : r2 == 4 ? inv4 : r2 == 5 ? inv5 : inv8;
      const float kern = kw[xx < 0 ? -xx : xx] * kw[yy < 0 ? -yy : yy];
      float4 ip = I[ro + px];
      float4 q = ND[rn + px];
      float lp = (0.2125f * ip.x + 0.7154f * ip.y) + 0.0721f * ip.z;
      float dn = fminf(fmaxf((nd.x * q.x + nd.y * q.y) + nd.z * q.z, 0.0f), 1.0f);
      // fmaxf: 0 * inf (phiIllumination == 0, equal luminance) is NaN, which the shader's max(., 0) zeroes
      float e = p.phi_normal * __builtin_amdgcn_logf(dn) -
                (fmaxf(fabsf(lc - lp) * kL, 0.0f) + fabsf(nd.w - q.w) * (kD * invlen));
      float w = __builtin_amdgcn_exp2f(e) * kern;
      sumW += w;
      s0 += w * ip.x;
      s1 += w * ip.y;
      s2 += w * ip.z;
      s3 += (w * w) * ip.w;
    }
  }
  float inv = 1.0f / sumW;
  float4 o;
  o.x = s0 * inv;
  o.y = s1 * inv;
  o.z = s2 * inv;
  o.w = s3 * (inv * inv);
  *out = o;
}

// ---------------------------------------------------------------------------
// Step-specialised form (production). The simple kernel above is VALU-bound, not
// HBM-bound: per tap it spends ~39 VALU instructions, a third of them 64-bit
// address arithmetic and bounds tests. Here the step is a template constant, so
// for blocks whose 5x5 dilated footprint lies inside the frame and the band
// (all but the border blocks) every tap is a load from a wave-uniform row
// pointer (SGPR base) at a constant column offset (immediate), with no tests;
// the 1/|offset| and kernel weights fold into per-pixel constants and the
// exponent. Border blocks run the checked path with the same arithmetic.
typedef float f2v __attribute__((ext_vector_type(2)));

// Luminance (svgf_Atrous.frag:57-59) of a tap's illumination, and the tap's luminance term |lp - lc| * kL: the
// tiled kernels of steps 1-4 (tile_stage_lum) stage lp per texel in LDS, so a tap's term is ONE FMA,
// |fma(lp, kL, -(lc * kL))|, instead of deriving it in each of up to 24 taps; the other steps keep the prescaled form
// |fma(z, wLb, fma(y, wLg, fma(x, wLr, -(lc * kL))))| (3 FMAs, no staged plane). The step kernel uses each step's form,
// so the tiled kernels stay bit-identical to it.
__device__ __forceinline__ float tap_luminance(float4 ip) {
  return __builtin_fmaf(0.0721f, ip.z, __builtin_fmaf(0.7154f, ip.y, 0.2125f * ip.x));
}
template <int S> constexpr bool tile_stage_lum() { return S <= 4; }

struct LumTerm {
  float lc, kL, cL, wLr, wLg, wLb;
  __device__ __forceinline__ void init(float4 ic, float kL_) {
    lc = tap_luminance(ic);
    kL = kL_;
    cL = -(lc * kL);
    wLr = 0.2125f * kL;
    wLg = 0.7154f * kL;
    wLb = 0.0721f * kL;
  }
  // lp - lc scaled by kL (its absolute value is the tap's term); LUM: lp given
  template <bool LUM>
  __device__ __forceinline__ float scaled(float4 ip, float lp) const {
    if (LUM) return __builtin_fmaf(lp, kL, cL);
    return __builtin_fmaf(ip.z, wLb, __builtin_fmaf(ip.y, wLg, __builtin_fmaf(ip.x, wLr, cL)));
  }
};

struct AtrousCentre {
  float4 ic, nd;
  LumTerm lum;
  float kD1, kD2, kD4, kD5, kD8, phiN;
};

// The 24 taps of one pixel. FLAT: phiIllumination == 0 (variance <= -1e-10 or NaN),
// where the shader's |lc - lp| / phiIllumination is +inf (weight 0) unless
// lp == lc (0/0 = NaN, which max(., 0) turns into 0): handled exactly, apart.
template <int S, bool EDGE, bool FLAT>
__device__ __forceinline__ void atrous_taps(const AtrousParams& p, const AtrousCentre& c, int x, int y, int ly,
                                            float& sumW, f2v& s01, f2v& s23) {
  const int W = p.illum.W;
  const float4* __restrict__ I = p.illum.p;
  const float4* __restrict__ ND = p.nd.p;
#pragma unroll
  for (int yy = -2; yy <= 2; ++yy) {
    const int py = y + yy * S;
    if (EDGE && (py < 0 || py >= p.H)) continue;
    const float4* __restrict__ Ir = I + (size_t)(EDGE ? arow(p.illum, py) : ly + yy * S) * W;
    const float4* __restrict__ Nr = ND + (size_t)(EDGE ? arow(p.nd, py) : ly + yy * S) * W;
#pragma unroll
    for (int xx = -2; xx <= 2; ++xx) {
      if (xx == 0 && yy == 0) continue;
      const int px = x + xx * S;
      if (EDGE && (px < 0 || px >= p.W)) continue;
      const int r2 = xx * xx + yy * yy;
      const float kDl = r2 == 1 ? c.kD1 : r2 == 2 ? c.kD2 : r2 == 4 ? c.kD4 : r2 == 5 ? c.kD5 : c.kD8;
      const int ax = xx < 0 ? -xx : xx, ay = yy < 0 ? -yy : yy;
      const float kern = (ax == 0 ? 1.0f : ax == 1 ? 2.0f / 3.0f : 1.0f / 6.0f) *
                         (ay == 0 ? 1.0f : ay == 1 ? 2.0f / 3.0f : 1.0f / 6.0f);
      const float4 ip = Ir[px];
      const float4 q = Nr[px];
      const float dn = fminf(fmaxf(__builtin_fmaf(c.nd.z, q.z, __builtin_fmaf(c.nd.y, q.y, c.nd.x * q.x)), 0.0f),
                             1.0f);
      constexpr bool LUM = tile_stage_lum<S>();
      float a;
      if (FLAT) {
        a = tap_luminance(ip) == c.lum.lc ? fabsf(c.nd.w - q.w) * kDl : __builtin_inff();
      } else {
        const float lp = LUM ? tap_luminance(ip) : 0.0f;
        a = __builtin_fmaf(fabsf(c.nd.w - q.w), kDl, fabsf(c.lum.scaled<LUM>(ip, lp)));
      }
      const float w = __builtin_amdgcn_exp2f(__builtin_fmaf(c.phiN, __builtin_amdgcn_logf(dn), -a)) * kern;
      sumW += w;
      s01 = __builtin_elementwise_fma(f2v{w, w}, f2v{ip.x, ip.y}, s01);
      s23 = __builtin_elementwise_fma(f2v{w, w * w}, f2v{ip.z, ip.w}, s23);
    }
  }
}

template <int S, bool EDGE>
__device__ __forceinline__ void atrous_pixel(const AtrousParams& p, int x, int y) {
  const int W = p.illum.W;
  const int ly = EDGE ? arow(p.illum, y) : y - p.illum.row0;
  AtrousCentre c;
  c.ic = p.illum.p[(size_t)ly * W + x];
  c.nd = p.nd.p[(size_t)ly * W + x];
  float4* out = p.out.p + (size_t)ly * W + x;
  if (c.nd.w == 1.0f) {
    *out = c.ic;
    return;
  }
  const float LOG2E = 1.4426950408889634f;
  const float phiL = p.phi_color * __builtin_sqrtf(fmaxf(0.0f, 1e-10f + c.ic.w));
  const float fwz = p.fwidth.aux ? fabsf(p.fwidth.aux[(size_t)ly * W + x]) : p.fwidth.p[(size_t)ly * W + x].y;
  c.lum.init(c.ic, LOG2E / phiL);  // |lc - lp| * kL = |lp * kL - lc * kL|
  const float kD = LOG2E / (fmaxf(fwz, 1e-8f) * (float)S);
  // kD / |offset| for |offset|^2 = 1, 2, 4, 5, 8
  c.kD1 = kD;
  c.kD2 = kD * 0.70710678f;
  c.kD4 = kD * 0.5f;
  c.kD5 = kD * 0.44721360f;
  c.kD8 = kD * 0.35355339f;
  c.phiN = p.phi_normal;
  float sumW = 1.0f;
  f2v s01 = {c.ic.x, c.ic.y}, s23 = {c.ic.z, c.ic.w};  // packed accumulators (v_pk_fma_f32)
  if (__builtin_expect(phiL > 0.0f, 1)) atrous_taps<S, EDGE, false>(p, c, x, y, ly, sumW, s01, s23);
  else atrous_taps<S, EDGE, true>(p, c, x, y, ly, sumW, s01, s23);
  const float inv = 1.0f / sumW;
  float4 o;
  o.x = s01.x * inv;
  o.y = s01.y * inv;
  o.z = s23.x * inv;
  o.w = s23.y * (inv * inv);
  *out = o;
}

// Block = 4 waves, each one row of 64 pixels; the row index is wave-uniform so
// the compiler keeps row pointers in SGPRs. Every plane of the pass must hold the
// same rows (always true for frame planes; the launcher checks).
template <int S>
__global__ void __launch_bounds__(256) atrous_step_kernel(AtrousParams p) {
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int x0 = blockIdx.x * 64;
  const int y = p.y0 + blockIdx.y * 4 + wv;
  if (y >= p.y1) return;
  const int x = x0 + (threadIdx.x & 63);
  const int yb = p.y0 + blockIdx.y * 4;
  const int lo = max(0, p.illum.row0), hi = min(p.H, p.illum.row0 + p.illum.rows);
  const bool interior = x0 - 2 * S >= 0 && x0 + 63 + 2 * S < p.W && yb - 2 * S >= lo &&
                        yb + 3 + 2 * S < hi;
  if (interior) {
    atrous_pixel<S, false>(p, x, y);
  } else if (x < p.W) {
    atrous_pixel<S, true>(p, x, y);
  }
}

// ---------------------------------------------------------------------------
// LDS-tiled form (production). The step kernel above is bound by the texture
// address path, not by HBM: 48 wave-wide 16-B loads per pixel keep the TA busy
// ~85% of the launch (rocprofv3 TA_TA_BUSY, profiles/). Here a block of 8 waves
// computes 64 columns x TJ = 8 rows taken from ONE residue class of rows mod S
// (rows ybase + S*j), so the whole dilated 5x5 footprint of the block is a dense
// (TJ+4) x (64+4S) texel tile of each plane: staged once into LDS with
// coalesced loads, then all 24 taps of every pixel read LDS (ds_read_b128 at
// immediate offsets). Blocks whose pixels are all background (zCenter == 1,
// svgf_Atrous.frag:77) copy and exit without staging. Same arithmetic, same tap
// order as atrous_taps: bit-identical to the step kernel.
//
// AUX: the G-buffer's compact depth-fwidth plane carries the zCenter == 1 flag in
// its sign bit (its magnitude is .y, always >= 0 or a NaN with the sign clear), so
// background pixels read 4 + 16 B and write 16 B.
// NX: 64-column strips per tile (waves side by side). The halo costs 4S staged columns per tile, so the widest
// step stages twice its output with NX = 1; S = 16 uses NX = 2 (128 columns, 1024 threads, 74 KB of LDS: measured
// 100 -> 91.5 us on the 4K bench inputs, measured with the harness tools/exp_atrous_real.hip of commit 6ee5990,
// removed in 53232a8: `git show 6ee5990:tools/exp_atrous_real.hip`), the other steps are fastest with NX = 1.
template <int S> constexpr int tile_nx() { return atrous_tile_nx(S); }
template <int S> constexpr int tile_tj() { return atrous_tile_tj(S); }  // tile rows = waves per 64-column strip
// tile_stage_lum: stage every texel's luminance beside it (4 B more LDS per staged texel and 3 VALU per staged texel,
// against 2 VALU per tap: each staged texel serves up to 24 taps). Steps 8 and 16 keep the prescaled per-tap form:
// their tiles are the widest (C = 64 NX + 4S columns), and the extra plane would cost them a resident block per CU
// (S = 8: 36.9 -> 41.5 KB, 4 -> 3 blocks; S = 16: 73.8 -> 83 KB, 2 -> 1).

__device__ __forceinline__ bool aux_flag(float a) { return (__float_as_uint(a) >> 31) != 0; }

// One output pixel of the tiled kernels: its constants and accumulators, and one tap (atrous_taps' arithmetic and tap
// order, so every tiled form is bit-identical to the step kernel). FLAT: phiIllumination == 0 (see atrous_taps).
struct TapPixel {
  float4 nd;
  LumTerm lum;
  float sumW;
  float kDr[5];
  f2v s01, s23;
  bool flat;
  __device__ __forceinline__ void init(float4 ic, float4 nd_, float fwz, float phi_color, int S) {
    const float LOG2E = 1.4426950408889634f;
    nd = nd_;
    const float phiL = phi_color * __builtin_sqrtf(fmaxf(0.0f, 1e-10f + ic.w));
    flat = !(phiL > 0.0f);
    lum.init(ic, LOG2E / phiL);
    const float kD = LOG2E / (fmaxf(fwz, 1e-8f) * (float)S);
    kDr[0] = kD;
    kDr[1] = kD * 0.70710678f;
    kDr[2] = kD * 0.5f;
    kDr[3] = kD * 0.44721360f;
    kDr[4] = kD * 0.35355339f;
    sumW = 1.0f;
    s01 = f2v{ic.x, ic.y};
    s23 = f2v{ic.z, ic.w};
  }
  template <bool FLAT, bool LUM>
  __device__ __forceinline__ void tap(float4 ip, float4 q, float lp, int xx, int yy, float phi_normal) {
    const int r2 = xx * xx + yy * yy;
    const float kDl = r2 == 1 ? kDr[0] : r2 == 2 ? kDr[1] : r2 == 4 ? kDr[2] : r2 == 5 ? kDr[3] : kDr[4];
    const int ax = xx < 0 ? -xx : xx, ay = yy < 0 ? -yy : yy;
    const float kern = (ax == 0 ? 1.0f : ax == 1 ? 2.0f / 3.0f : 1.0f / 6.0f) *
                       (ay == 0 ? 1.0f : ay == 1 ? 2.0f / 3.0f : 1.0f / 6.0f);
    const float dn = fminf(fmaxf(__builtin_fmaf(nd.z, q.z, __builtin_fmaf(nd.y, q.y, nd.x * q.x)), 0.0f), 1.0f);
    float a;
    if (FLAT) {
      a = (LUM ? lp : tap_luminance(ip)) == lum.lc ? fabsf(nd.w - q.w) * kDl : __builtin_inff();
    } else {
      a = __builtin_fmaf(fabsf(nd.w - q.w), kDl, fabsf(lum.scaled<LUM>(ip, lp)));
    }
    const float w = __builtin_amdgcn_exp2f(__builtin_fmaf(phi_normal, __builtin_amdgcn_logf(dn), -a)) * kern;
    sumW += w;
    s01 = __builtin_elementwise_fma(f2v{w, w}, f2v{ip.x, ip.y}, s01);
    s23 = __builtin_elementwise_fma(f2v{w, w * w}, f2v{ip.z, ip.w}, s23);
  }
  // the 24 taps of a window whose top-left texel is Li / Ln (row stride C, column step S); EDGE: skip taps outside
  // the frame for the pixel at (x, y). Ll: the staged luminance of the texels (null: derived per tap)
  template <bool FLAT, bool EDGE, int S, int C, bool LUM>
  __device__ __forceinline__ void window(const float4* Li, const float4* Ln, const float* Ll, int x, int y, int W,
                                         int H, float phi_normal) {
#pragma unroll
    for (int yy = -2; yy <= 2; ++yy) {
      if (EDGE && (y + yy * S < 0 || y + yy * S >= H)) continue;
#pragma unroll
      for (int xx = -2; xx <= 2; ++xx) {
        if (xx == 0 && yy == 0) continue;
        if (EDGE && (x + xx * S < 0 || x + xx * S >= W)) continue;
        const int o = (yy + 2) * C + (xx + 2) * S;
        tap<FLAT, LUM>(Li[o], Ln[o], LUM ? Ll[o] : 0.0f, xx, yy, phi_normal);
      }
    }
  }
  __device__ __forceinline__ float4 result() const {
    const float inv = 1.0f / sumW;
    return float4{s01.x * inv, s01.y * inv, s23.x * inv, s23.y * (inv * inv)};
  }
};

// The fused modulate (svgf_modulate.frag; kernels_svgf.hip::modulate_kernel's arithmetic, also built with
// -ffp-contract=off): c * albedo + emission on surface pixels, c passed through on background pixels (zCenter == 1,
// the a-trous kernel's own background test), alpha 1.
__device__ __forceinline__ void modulate_store(const AtrousParams& p, int x, int y, float4 c, bool bg) {
  float4 o;
  if (bg) {
    o.x = c.x;
    o.y = c.y;
    o.z = c.z;
  } else {
    const float4 a = p.albedo.p[(size_t)(y - p.albedo.row0) * p.albedo.W + x];
    const float4 e = p.emission.p[(size_t)(y - p.emission.row0) * p.emission.W + x];
    o.x = c.x * a.x + e.x;
    o.y = c.y * a.y + e.y;
    o.z = c.z * a.z + e.z;
  }
  o.w = 1.0f;
  p.mod.p[(size_t)(y - p.mod.row0) * p.mod.W + x] = o;
}

template <int S, bool AUX>
__global__ void __launch_bounds__(64 * tile_tj<S>() * tile_nx<S>()) atrous_tile_kernel(AtrousParams p) {
  constexpr int NX = tile_nx<S>();
  constexpr int TJ = tile_tj<S>(), NW = TJ * NX, R = TJ + 4, C = 64 * NX + 4 * S, NT = 64 * NW;
  constexpr bool LUM = tile_stage_lum<S>();
  constexpr int PAD = (R * C) % NT ? 16 : 0;  // dummy slots of the staging's last trip (16: S = 2 keeps 5 blocks/CU)
  __shared__ float4 LI[R * C + PAD];
  __shared__ float4 LN[R * C + PAD];
  __shared__ float LL[LUM ? R * C + PAD : 1];
  const int W = p.illum.W, row0 = p.illum.row0;
  const float4* __restrict__ I = p.illum.p;
  const float4* __restrict__ ND = p.nd.p;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bx = blockIdx.x, g = blockIdx.y / S, b = blockIdx.y - g * S;
  const int ybase = p.y0 + g * S * TJ + b;  // frame row of tile row j = 0
  const int j = wv / NX, xl = (wv - j * NX) * 64 + lane;  // tile row, tile column
  const int x0 = bx * 64 * NX, x = x0 + xl, y = ybase + S * j;
  const bool own = x < p.W && y < p.y1;
  const size_t ci = (size_t)(y - row0) * W + x;
  bool bg = true;
  float fwz = 0.0f;
  // Per-tile flags precomputed from the depth-fwidth plane once per G-buffer (atrous_tile_flags): a background tile
  // copies without reading its pixels' flags or meeting at a barrier; the others read them for their taps.
  const bool pre = AUX && p.tile_any != nullptr;
  bool tile_any = true;
  if (pre) tile_any = p.tile_any[(g * S + b) * gridDim.x + bx] != 0;
  if (!pre && own) {  // (with the flags the pixel's own flag is read beside the staging loads, below)
    if (AUX) {
      const float a = p.fwidth.aux[ci];
      bg = aux_flag(a);
      fwz = fabsf(a);
    } else {
      bg = ND[ci].w == 1.0f;
      fwz = p.fwidth.p[ci].y;
    }
  }
  if (!pre) {
// any surface pixel in the tile? One ballot per wave and ONE barrier (the flags have their own LDS words) instead
// of __syncthreads_or's three (76.1 vs 79.8 us default view, 152.4 vs 158.5 surface view, tools/bench_atrous.py).
    __shared__ int any_surface[NW];
    const bool wave_any = __ballot(!bg) != 0ull;
    if (lane == 0) any_surface[wv] = wave_any;
    __syncthreads();
    tile_any = false;
#pragma unroll
    for (int w = 0; w < NW; ++w) tile_any |= any_surface[w] != 0;
  }
  if (!tile_any) {
    if (own) {
      const float4 v = I[ci];
      p.out.p[ci] = v;
      if (p.mod.p) modulate_store(p, x, y, v, true);
    }
    return;
  }
  // stage: tile row r <-> frame row ybase + S*(r-2), column c <-> x0 - 2S + c; rows outside the frame and
  // columns outside [0, W) are clamped (their taps are skipped below), rows outside the stored band clamp too.
  // All of a thread's staging loads are issued before its first LDS write (NIT = 2 or 3 texels per thread), so a
  // tile waits for one memory latency, not one per loop trip; a thread past the tile's end loads the last texel again
  // (an address inside the planes) into a dummy slot.
  const int lo = max(0, row0), hi = min(p.H, row0 + p.illum.rows) - 1;
  // the pixel's flag and depth fwidth (a pixel outside the frame or band reads its clamped neighbour's, unused)
  float own_aux = 0.0f;
  if (pre) own_aux = p.fwidth.aux[(size_t)(min(y, p.y1 - 1) - row0) * W + min(x, p.W - 1)];
  constexpr int NIT = (R * C + NT - 1) / NT;
  float4 sv[NIT], sn[NIT];
#pragma unroll
  for (int k = 0; k < NIT; ++k) {
    const int e = min(tid + k * NT, R * C - 1);
    const int r = e / C, c = e - r * C;
    int gy = ybase + S * (r - 2), gx = x0 - 2 * S + c;
    gy = gy < lo ? lo : (gy > hi ? hi : gy);
    gx = gx < 0 ? 0 : (gx >= p.W ? p.W - 1 : gx);
    const size_t gi = (size_t)(gy - row0) * W + gx;
    sv[k] = I[gi];
    sn[k] = ND[gi];
  }
#pragma unroll
  for (int k = 0; k < NIT; ++k) {
    // every trip stores (past the tile's end into one of PAD dummy slots): a conditional store would let the compiler
    // sink its loads into the branch, one memory latency per trip again
    const int e = tid + k * NT < R * C ? tid + k * NT : R * C + (lane & (PAD - 1));
    LI[e] = sv[k];
    LN[e] = sn[k];
    if (LUM) LL[e] = tap_luminance(sv[k]);
  }
  if (pre && own) {
    bg = aux_flag(own_aux);
    fwz = fabsf(own_aux);
  }
  __syncthreads();
  if (!own) return;
  const float4* Li = LI + j * C + xl;  // top-left tap of this pixel's window
  const float4* Ln = LN + j * C + xl;
  const float* Ll = LL + (LUM ? j * C + xl : 0);
  const float4 ic = Li[2 * C + 2 * S];
  float4* out = p.out.p + ci;
  if (bg) {
    *out = ic;
    if (p.mod.p) modulate_store(p, x, y, ic, true);
    return;
  }
  const bool edge =
      x0 - 2 * S < 0 || x0 + 64 * NX - 1 + 2 * S >= p.W || ybase - 2 * S < 0 || ybase + S * (TJ + 1) >= p.H;
  TapPixel px;
  px.init(ic, Ln[2 * C + 2 * S], fwz, p.phi_color, S);
  // EDGE = false: the block's dilated footprint lies inside the frame, so the 24 taps are straight-line code the
  // compiler schedules freely (LDS reads of later taps issued ahead of earlier taps' arithmetic). A per-tap `edge`
  // test in that path compiles to an exec-masked branch per tap, each behind its own LDS wait (the r02 kernel).
  if (__builtin_expect(!px.flat, 1)) {
    if (__builtin_expect(!edge, 1)) px.window<false, false, S, C, LUM>(Li, Ln, Ll, x, y, p.W, p.H, p.phi_normal);
    else px.window<false, true, S, C, LUM>(Li, Ln, Ll, x, y, p.W, p.H, p.phi_normal);
  } else {
    px.window<true, true, S, C, LUM>(Li, Ln, Ll, x, y, p.W, p.H, p.phi_normal);  // FLAT: rare
  }
  const float4 r = px.result();
  *out = r;
  if (p.mod.p) modulate_store(p, x, y, r, false);
}

// Tile flags of the five step sizes (atrous_tile_kernel's tiles: S = 1 << si, NX = tile_nx<S>(), TJ = tile_tj<S>() rows of one
// residue class): byte (g * S + b) * NXT + bx of step si is 1 iff an owned pixel of that tile is a surface pixel
// (the depth-fwidth plane's sign bit clear). One wave per 64 columns of a row; a ballot, then one byte store per step.
static int tiles_of(int S, int W, int y0, int y1) {
  const int nx = atrous_tile_nx(S), nxt = (W + 64 * nx - 1) / (64 * nx), tj = atrous_tile_tj(S);
  const int groups = (y1 - y0 + S * tj - 1) / (S * tj);
  return nxt * groups * S;
}
size_t atrous_flag_offset(int si, int W, int y0, int y1) {
  size_t o = 0;
  for (int t = 0; t < si; ++t) o += (size_t)tiles_of(1 << t, W, y0, y1);
  return o;
}
__global__ void __launch_bounds__(64) atrous_flags_kernel(const float* __restrict__ aux, int row0, int W, int y0,
                                                         unsigned char* __restrict__ flags, int o1, int o2, int o3,
                                                         int o4) {
  const int x0 = blockIdx.x * 64, x = x0 + (int)threadIdx.x, y = y0 + (int)blockIdx.y;
  const bool surf = x < W && !aux_flag(aux[(size_t)(y - row0) * W + x]);
  if (__ballot(surf) == 0ull || threadIdx.x != 0) return;
  const int off[5] = {0, o1, o2, o3, o4};
  atrous_mark_tiles(flags, off, W, x0, y - y0);
}
size_t atrous_flag_bytes(int W, int y0, int y1) { return atrous_flag_offset(5, W, y0, y1); }
int atrous_tile_flags(const Plane& fw, int W, int y0, int y1, unsigned char* flags, hipStream_t s) {
  if (y1 <= y0 || !fw.aux) return 0;
  hipError_t e = hipMemsetAsync(flags, 0, atrous_flag_bytes(W, y0, y1), s);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(atrous_flags_kernel, dim3((W + 63) / 64, y1 - y0), dim3(64), 0, s, fw.aux, fw.row0, W, y0, flags,
                     (int)atrous_flag_offset(1, W, y0, y1), (int)atrous_flag_offset(2, W, y0, y1),
                     (int)atrous_flag_offset(3, W, y0, y1), (int)atrous_flag_offset(4, W, y0, y1));
  return (int)hipGetLastError();
}

template <int S>
static void launch_tile_s(const AtrousParams& p, bool aux, hipStream_t s) {
  constexpr int NX = tile_nx<S>(), TJ = tile_tj<S>();
  const int groups = (p.y1 - p.y0 + S * TJ - 1) / (S * TJ);
  dim3 grid((p.W + 64 * NX - 1) / (64 * NX), groups * S);
  if (aux) hipLaunchKernelGGL((atrous_tile_kernel<S, true>), grid, dim3(64 * TJ * NX), 0, s, p);
  else hipLaunchKernelGGL((atrous_tile_kernel<S, false>), grid, dim3(64 * TJ * NX), 0, s, p);
}

static bool same_geometry(const AtrousParams& p) {
  const Plane* planes[3] = {&p.nd, &p.out, &p.fwidth};
  for (const Plane* q : planes)
    if (q->row0 != p.illum.row0 || q->rows != p.illum.rows || q->W != p.illum.W) return false;
  return p.illum.W == p.W;
}

// the fused modulate of a draw whose kernel does not fuse it: modulate_kernel over the same rows, after the a-trous
int launch_modulate_after(const AtrousParams& p, hipStream_t s) {
  if (!p.mod.p || p.y1 <= p.y0) return 0;
  ModulateParams m;
  m.W = p.W;
  m.H = p.H;
  m.y0 = p.y0;
  m.y1 = p.y1;
  m.albedo = p.albedo;
  m.emission = p.emission;
  m.illum = p.out;
  m.nd = p.nd;
  m.out = p.mod;
  return launch_modulate(m, s);
}

int launch_atrous_fast(const AtrousParams& p, hipStream_t s) {
  if (p.y1 <= p.y0) return 0;
  if (!same_geometry(p)) {
    const int rc = launch_atrous_simple(p, s);
    return rc ? rc : launch_modulate_after(p, s);
  }
  const bool aux = p.fwidth.aux != nullptr;
  switch (p.step) {
    case 1: launch_tile_s<1>(p, aux, s); break;
    case 2: launch_tile_s<2>(p, aux, s); break;
    case 4: launch_tile_s<4>(p, aux, s); break;
    case 8: launch_tile_s<8>(p, aux, s); break;
    case 16: launch_tile_s<16>(p, aux, s); break;
    default: {
      const int rc = launch_atrous_step(p, s);
      return rc ? rc : launch_modulate_after(p, s);
    }
  }
  return (int)hipGetLastError();
}

int launch_atrous_step(const AtrousParams& p, hipStream_t s) {
  if (p.y1 <= p.y0) return 0;
  if (!same_geometry(p)) return launch_atrous_simple(p, s);
  dim3 grid((p.W + 63) / 64, (p.y1 - p.y0 + 3) / 4);
  switch (p.step) {
    case 1: hipLaunchKernelGGL(atrous_step_kernel<1>, grid, dim3(256), 0, s, p); break;
    case 2: hipLaunchKernelGGL(atrous_step_kernel<2>, grid, dim3(256), 0, s, p); break;
    case 4: hipLaunchKernelGGL(atrous_step_kernel<4>, grid, dim3(256), 0, s, p); break;
    case 8: hipLaunchKernelGGL(atrous_step_kernel<8>, grid, dim3(256), 0, s, p); break;
    case 16: hipLaunchKernelGGL(atrous_step_kernel<16>, grid, dim3(256), 0, s, p); break;
    default: return launch_atrous_simple(p, s);  // other steps (iterations > 5): generic kernel
  }
  return (int)hipGetLastError();
}

int launch_atrous_simple(const AtrousParams& p, hipStream_t s) {
  if (p.y1 <= p.y0) return 0;
  dim3 grid((p.W + 63) / 64, (p.y1 - p.y0 + 3) / 4);
  hipLaunchKernelGGL(atrous_fast_kernel, grid, dim3(256), 0, s, p);
  return (int)hipGetLastError();
}

}  // namespace ptk

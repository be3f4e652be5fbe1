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
#include <hip/hip_runtime.h>

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
  float fwz = p.fwidth.aux ? p.fwidth.aux[(size_t)arow(p.fwidth, y) * p.fwidth.W + x]
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
      float e = p.phi_normal * __builtin_amdgcn_logf(dn) -
                (fabsf(lc - lp) * kL + fabsf(nd.w - q.w) * (kD * invlen));
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

int launch_atrous_fast(const AtrousParams& p, hipStream_t s) {
  if (p.y1 <= p.y0) return 0;
  dim3 grid((p.W + 63) / 64, (p.y1 - p.y0 + 3) / 4);
  hipLaunchKernelGGL(atrous_fast_kernel, grid, dim3(256), 0, s, p);
  return (int)hipGetLastError();
}

}  // namespace ptk

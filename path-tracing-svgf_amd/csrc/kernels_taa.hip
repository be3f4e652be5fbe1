// kernels_taa.hip — temporal anti-aliasing pass (shaders/taa.frag:15-153),
// the consumer of svgf_modulate's output (main.cpp:537-544). One thread per
// pixel; integer-offset taps are direct texel reads with CLAMP_TO_EDGE (the GL
// sampler returns texels exactly there, glsl_builtins.h), the history fetch at
// (uv - velocity) is a bilinear fetch.
#include <hip/hip_runtime.h>

#include "glsl_builtins.h"
#include "pt_device.h"

using namespace glsl;

namespace ptk {

__device__ __forceinline__ int trow(const Plane& P, int y) {
  int ly = y - P.row0;
  return ly < 0 ? 0 : (ly >= P.rows ? P.rows - 1 : ly);
}
__device__ __forceinline__ float4 tld(const Plane& P, int x, int y) { return P.p[(size_t)trow(P, y) * P.W + x]; }

// RGB2YCoCgR / YCoCgR2RGB (taa.frag:41-62)
__device__ __forceinline__ v3 to_ycocg(v3 c) {
  v3 r;
  r.y = c.x - c.z;
  float temp = c.z + r.y / 2.0f;
  r.z = c.y - temp;
  r.x = temp + r.z / 2.0f;
  return r;
}
__device__ __forceinline__ v3 from_ycocg(v3 c) {
  v3 r;
  float temp = c.x - c.z / 2.0f;
  r.y = c.z + temp;
  r.z = temp - c.y / 2.0f;
  r.x = r.z + c.y;
  return r;
}
__device__ __forceinline__ float taa_lum(v3 c) { return (0.25f * c.x + 0.5f * c.y) + 0.25f * c.z; }
__device__ __forceinline__ v3 tonemap(v3 c) { return divs(c, 1.0f + taa_lum(c)); }
__device__ __forceinline__ v3 untonemap(v3 c) { return divs(c, 1.0f - taa_lum(c)); }

__global__ void __launch_bounds__(256) taa_kernel(TAAParams p) {
  int x = blockIdx.x * 16 + (threadIdx.x & 15);
  int y = p.y0 + blockIdx.y * 16 + (threadIdx.x >> 4);
  if (x >= p.W || y >= p.y1) return;
  float4 o;
  float4 now4 = tld(p.cur, x, y);
  v3 nowColor = mk(now4.x, now4.y, now4.z);
  if (p.frameCounter == 0u || tld(p.nd, x, y).w == 1.0f) {  // :126-135
    o.x = nowColor.x; o.y = nowColor.y; o.z = nowColor.z; o.w = 1.0f;
    p.out.p[(size_t)trow(p.out, y) * p.out.W + x] = o;
    return;
  }
  // getClosestOffset (:19-39): strict '<' keeps the first minimum in (i, j) order
  float closest = 1.0f;
  int cx = x, cy = y;
  for (int i = -1; i <= 1; ++i)
    for (int j = -1; j <= 1; ++j) {
      int tx = clampi(x + i, 0, p.W - 1), ty = clampi(y + j, 0, p.H - 1);
      float dd = tld(p.nd, tx, ty).w;
      if (dd < closest) { closest = dd; cx = tx; cy = ty; }
    }
  float4 vel = tld(p.vel, cx, cy);
  float sx = ((float)(2 * x + 1) / (float)p.W - 1.0f) * 0.5f + 0.5f;
  float sy = ((float)(2 * y + 1) / (float)p.H - 1.0f) * 0.5f + 0.5f;
  float ou = f_clamp(sx - vel.x, 0.0f, 1.0f), ov = f_clamp(sy - vel.y, 0.0f, 1.0f);
  Bilin b = bilin_setup(ou, ov, p.W, p.H);
  float4 c00 = tld(p.prev, b.x0, b.y0), c10 = tld(p.prev, b.x1, b.y0);
  float4 c01 = tld(p.prev, b.x0, b.y1), c11 = tld(p.prev, b.x1, b.y1);
  v3 pre = mk(bilin_mix(b, c00.x, c10.x, c01.x, c11.x), bilin_mix(b, c00.y, c10.y, c01.y, c11.y),
              bilin_mix(b, c00.z, c10.z, c01.z, c11.z));
  v3 now = to_ycocg(tonemap(nowColor));
  pre = to_ycocg(tonemap(pre));
  // clipAABB (:80-121)
  v3 m1 = splat(0.0f), m2 = splat(0.0f);
  for (int i = -1; i <= 1; ++i)
    for (int j = -1; j <= 1; ++j) {
      float4 q = tld(p.cur, clampi(x + i, 0, p.W - 1), clampi(y + j, 0, p.H - 1));
      v3 C = to_ycocg(tonemap(mk(q.x, q.y, q.z)));
      m1 = add(m1, C);
      m2 = add(m2, mul(C, C));
    }
  v3 mu = divs(m1, 9.0f);
  v3 var = sub(divs(m2, 9.0f), mul(mu, mu));
  v3 sigma = mk(f_sqrt(f_abs(var.x)), f_sqrt(f_abs(var.y)), f_sqrt(f_abs(var.z)));
  v3 amin = sub(mu, muls(sigma, 1.0f)), amax = add(mu, muls(sigma, 1.0f));
  v3 pc = muls(add(amax, amin), 0.5f), ec = muls(sub(amax, amin), 0.5f);
  v3 vc = sub(pre, pc);
  v3 vu = divv(vc, ec);
  float ma = f_max(f_abs(vu.x), f_max(f_abs(vu.y), f_abs(vu.z)));
  if (ma > 1.0f) pre = add(pc, divs(vc, ma));
  pre = untonemap(from_ycocg(pre));
  now = untonemap(from_ycocg(now));
  float vlen = f_sqrt(vel.x * vel.x + vel.y * vel.y);
  float bf = f_clamp(0.05f + vlen * 100.0f, 0.0f, 1.0f);
  o.x = bf * now.x + (1.0f - bf) * pre.x;
  o.y = bf * now.y + (1.0f - bf) * pre.y;
  o.z = bf * now.z + (1.0f - bf) * pre.z;
  o.w = 1.0f;
  p.out.p[(size_t)trow(p.out, y) * p.out.W + x] = o;
}

int launch_taa(const TAAParams& p, hipStream_t s) {
  if (p.y1 <= p.y0) return 0;
  dim3 grid((p.W + 15) / 16, (p.y1 - p.y0 + 15) / 16);
  hipLaunchKernelGGL(taa_kernel, grid, dim3(256), 0, s, p);
  return (int)hipGetLastError();
}

}  // namespace ptk

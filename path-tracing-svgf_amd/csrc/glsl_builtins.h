// glsl_builtins.h — deterministic fp32 restatement of the GLSL 4.50 built-in
// functions the reference shaders call (GLSL 4.50 spec §8: sin, cos, atan(y,x),
// asin, log, exp, pow, normalize, cross, dot, mix, clamp, reflect, length,
// distance) plus the two texture samplers the shaders use (texelFetch on an
// RGB32F buffer, texture2D with GL_LINEAR + GL_CLAMP_TO_EDGE).
//
// Why this exists: GLSL leaves the precision of transcendentals to the driver,
// and a 1-ulp difference in sin/atan/log between the GPU and a CPU checker can
// flip a path-tracer branch (SURVEY.md §7 "Hard parts" 1). Every function here
// is built from IEEE-754 + - * / sqrt (correctly rounded on gfx950 under hipcc's
// default -fhip-fp32-correctly-rounded-divide-sqrt, and on x86-64 SSE), so with
// -ffp-contract=off the HIP kernels and the CPU oracle evaluate the identical
// built-in on identical bits. Polynomials follow the published Cephes single-
// precision algorithms (sinf/cosf/atanf/asinf/logf/expf, S. L. Moshier),
// accuracy 1-3 ulp over the argument ranges the shaders use.
//
// This is the GL *built-in library*, shared by product and checker the way a
// driver's built-ins are shared by every shader; the shader algorithms
// themselves are restated separately in csrc/*.hip (product) and oracle/*.cpp
// (checker).
#pragma once

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define GL_HD __host__ __device__ __forceinline__
#else
#include <cmath>
#include <cstdint>
#include <cstring>
#define GL_HD static inline
#endif

#include <stdint.h>

namespace glsl {

// ---------------------------------------------------------------- scalar ---
GL_HD float f_abs(float x) { return fabsf(x); }
GL_HD float f_min(float a, float b) { return fminf(a, b); }  // NaN-ignoring (IEEE minNum)
GL_HD float f_max(float a, float b) { return fmaxf(a, b); }
GL_HD float f_clamp(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
GL_HD float f_mix(float x, float y, float a) { return x * (1.0f - a) + y * a; }  // GLSL §8.3 definition
GL_HD float f_sqrt(float x) { return sqrtf(x); }
GL_HD float f_floor(float x) { return floorf(x); }
GL_HD bool f_isnan(float x) { return x != x; }
// int(float): GLSL leaves NaN / out-of-range undefined (and C makes it UB). Defined here
// as gfx950's v_cvt_i32_f32: NaN -> 0, saturate to the int range, else truncate.
GL_HD int f2i(float x) {
  if (x != x) return 0;
  if (x >= 2147483648.0f) return 2147483647;
  if (x <= -2147483648.0f) return (int)0x80000000;
  return (int)x;
}

GL_HD uint32_t f_bits(float f) {
#if defined(__HIPCC__)
  return __float_as_uint(f);
#else
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
#endif
}
GL_HD float f_from_bits(uint32_t u) {
#if defined(__HIPCC__)
  return __uint_as_float(u);
#else
  float f;
  memcpy(&f, &u, 4);
  return f;
#endif
}

constexpr float kPIO4 = 0.785398163397448309616f;
constexpr float kPIO2 = 1.570796326794896619f;
constexpr float kPI = 3.14159265358979323846f;

// Cephes sinf/cosf shared reduction (x >= 0): octant j and reduced argument.
GL_HD float cephes_sin_poly(float x, float z) {
  return ((-1.9515295891E-4f * z + 8.3321608736E-3f) * z - 1.6666654611E-1f) * z * x + x;
}
GL_HD float cephes_cos_poly(float z) {
  return ((2.443315711809948E-005f * z - 1.388731625493765E-003f) * z + 4.166664568298827E-002f) * z * z -
         0.5f * z + 1.0f;
}

GL_HD float g_sin(float xx) {
  float x = xx;
  int sign = 1;
  if (x < 0.0f) { sign = -1; x = -x; }
  int j = f2i(1.27323954473516f * x);
  float y = (float)j;
  if (j & 1) { j += 1; y += 1.0f; }
  j &= 7;
  if (j > 3) { sign = -sign; j -= 4; }
  x = ((x - y * 0.78515625f) - y * 2.4187564849853515625e-4f) - y * 3.77489497744594108e-8f;
  float z = x * x;
  float r = (j == 1 || j == 2) ? cephes_cos_poly(z) : cephes_sin_poly(x, z);
  return sign < 0 ? -r : r;
}

GL_HD float g_cos(float xx) {
  float x = xx < 0.0f ? -xx : xx;
  int sign = 1;
  int j = f2i(1.27323954473516f * x);
  float y = (float)j;
  if (j & 1) { j += 1; y += 1.0f; }
  j &= 7;
  if (j > 3) { j -= 4; sign = -sign; }
  if (j > 1) sign = -sign;
  x = ((x - y * 0.78515625f) - y * 2.4187564849853515625e-4f) - y * 3.77489497744594108e-8f;
  float z = x * x;
  float r = (j == 1 || j == 2) ? cephes_sin_poly(x, z) : cephes_cos_poly(z);
  return sign < 0 ? -r : r;
}

GL_HD float g_atan(float xx) {
  float x = xx < 0.0f ? -xx : xx;
  float y;
  if (x > 2.414213562373095f) { y = kPIO2; x = -(1.0f / x); }
  else if (x > 0.4142135623730950f) { y = kPIO4; x = (x - 1.0f) / (x + 1.0f); }
  else y = 0.0f;
  float z = x * x;
  y += (((8.05374449538e-2f * z - 1.38776856032E-1f) * z + 1.99777106478E-1f) * z - 3.33329491539E-1f) * z * x + x;
  return xx < 0.0f ? -y : y;
}

// GLSL atan(y, x) (Cephes atan2f quadrant logic).
GL_HD float g_atan2(float y, float x) {
  int code = 0;
  if (x < 0.0f) code = 2;
  if (y < 0.0f) code |= 1;
  if (x == 0.0f) {
    if (code & 1) return -kPIO2;
    if (y == 0.0f) return 0.0f;
    return kPIO2;
  }
  if (y == 0.0f) return (code & 2) ? kPI : 0.0f;
  float w = 0.0f;
  if (code == 2) w = kPI;
  else if (code == 3) w = -kPI;
  return w + g_atan(y / x);
}

GL_HD float g_asin(float xx) {
  float a = xx < 0.0f ? -xx : xx;
  if (a > 1.0f) return f_from_bits(0x7fc00000u);
  float x, z;
  int flag;
  if (a < 1.0e-4f) return xx;
  if (a > 0.5f) { z = 0.5f * (1.0f - a); x = f_sqrt(z); flag = 1; }
  else { x = a; z = x * x; flag = 0; }
  z = ((((4.2163199048E-2f * z + 2.4181311049E-2f) * z + 4.5470025998E-2f) * z + 7.4953002686E-2f) * z +
       1.6666752422E-1f) * z * x + x;
  if (flag) { z = z + z; z = kPIO2 - z; }
  return xx < 0.0f ? -z : z;
}

// Exact frexp for finite positive x (subnormals included).
GL_HD float g_frexp_pos(float x, int* e) {
  uint32_t u = f_bits(x);
  int ex = (int)((u >> 23) & 0xffu);
  int bias = 0;
  if (ex == 0) {  // subnormal: scale by 2^25 exactly
    x = x * 33554432.0f;
    u = f_bits(x);
    ex = (int)((u >> 23) & 0xffu);
    bias = -25;
  }
  *e = ex - 126 + bias;
  return f_from_bits((u & 0x807fffffu) | 0x3f000000u);
}

// Exact ldexp(x, n) for x in [0.5, 4) and n in [-160, 128] (one rounding).
GL_HD float g_ldexp(float x, int n) {
  if (n > 127) { x = x * 1.7014118346046923e38f; n -= 127; if (n > 127) n = 127; }
  if (n < -126) {
    x = x * f_from_bits((uint32_t)(n + 64 + 127) << 23);  // exact: result stays normal
    return x * 5.42101086242752217e-20f;                   // 2^-64, the only rounding
  }
  return x * f_from_bits((uint32_t)(n + 127) << 23);
}

GL_HD float g_log(float xx) {
  if (f_isnan(xx)) return xx;
  if (xx <= 0.0f) return xx == 0.0f ? -__builtin_inff() : f_from_bits(0x7fc00000u);
  if (xx == __builtin_inff()) return xx;
  int e;
  float x = g_frexp_pos(xx, &e);
  if (x < 0.707106781186547524f) { e -= 1; x = x + x - 1.0f; }
  else x = x - 1.0f;
  float z = x * x;
  float y = ((((((((7.0376836292E-2f * x - 1.1514610310E-1f) * x + 1.1676998740E-1f) * x - 1.2420140846E-1f) * x +
                 1.4249322787E-1f) * x - 1.6668057665E-1f) * x + 2.0000714765E-1f) * x - 2.4999993993E-1f) * x +
            3.3333331174E-1f) * x * z;
  float fe = (float)e;
  y += -2.12194440e-4f * fe;
  y += -0.5f * z;
  z = x + y;
  z += 0.693359375f * fe;
  return z;
}

GL_HD float g_exp(float xx) {
  if (f_isnan(xx)) return xx;
  if (xx > 88.72283905206835f) return __builtin_inff();
  if (xx < -103.278929903431851103f) return 0.0f;
  float z = f_floor(1.44269504088896341f * xx + 0.5f);
  float x = xx - z * 0.693359375f;
  x = x - z * -2.12194440e-4f;
  int n = (int)z;
  z = x * x;
  z = (((((1.9875691500E-4f * x + 1.3981999507E-3f) * x + 8.3334519073E-3f) * x + 4.1665795894E-2f) * x +
        1.6666665459E-1f) * x + 5.0000001201E-1f) * z + x + 1.0f;
  return g_ldexp(z, n);
}

// GLSL pow: results undefined for x < 0 or (x == 0 and y <= 0); spec defines it
// through exp2(y * log2(x)). Here: exp(y * log(x)) with the exact zero cases.
GL_HD float g_pow(float x, float y) {
  if (y == 0.0f) return 1.0f;
  if (x == 0.0f) return y > 0.0f ? 0.0f : __builtin_inff();
  if (x == 1.0f) return 1.0f;
  return g_exp(y * g_log(x));
}

// ---------------------------------------------------------------- vec3 ---
struct v3 {
  float x, y, z;
};
GL_HD v3 mk(float x, float y, float z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
GL_HD v3 splat(float s) { return mk(s, s, s); }
GL_HD v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
GL_HD v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
GL_HD v3 mul(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
GL_HD v3 muls(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
GL_HD v3 divv(v3 a, v3 b) { return mk(a.x / b.x, a.y / b.y, a.z / b.z); }
GL_HD v3 divs(v3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
GL_HD v3 neg(v3 a) { return mk(-a.x, -a.y, -a.z); }
GL_HD float dot(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
GL_HD v3 cross(v3 a, v3 b) {
  return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
GL_HD float length(v3 a) { return f_sqrt(dot(a, a)); }
// GLSL normalize(x) = x / length(x); evaluated as x * (1 / length(x)).
GL_HD v3 normalize(v3 a) {
  float inv = 1.0f / f_sqrt(dot(a, a));
  return muls(a, inv);
}
GL_HD float distance(v3 a, v3 b) { return length(sub(a, b)); }
GL_HD v3 mixv(v3 x, v3 y, float a) { return mk(f_mix(x.x, y.x, a), f_mix(x.y, y.y, a), f_mix(x.z, y.z, a)); }
GL_HD v3 mixvv(v3 x, v3 y, v3 a) { return mk(f_mix(x.x, y.x, a.x), f_mix(x.y, y.y, a.y), f_mix(x.z, y.z, a.z)); }
GL_HD v3 vmin(v3 a, v3 b) { return mk(f_min(a.x, b.x), f_min(a.y, b.y), f_min(a.z, b.z)); }
GL_HD v3 vmax(v3 a, v3 b) { return mk(f_max(a.x, b.x), f_max(a.y, b.y), f_max(a.z, b.z)); }
GL_HD v3 vclamp(v3 a, float lo, float hi) { return mk(f_clamp(a.x, lo, hi), f_clamp(a.y, lo, hi), f_clamp(a.z, lo, hi)); }
// GLSL reflect(I, N) = I - 2 * dot(N, I) * N
GL_HD v3 reflect(v3 I, v3 N) {
  float d = 2.0f * dot(N, I);
  return sub(I, muls(N, d));
}

// ------------------------------------------------------------- samplers ---
// GL_LINEAR + GL_CLAMP_TO_EDGE bilinear addressing, texel (0,0) centred at
// uv = (0.5/W, 0.5/H). The texel-space coordinate is snapped to 8 fractional
// bits, as GPU texture units do (the GL spec leaves the sub-texel precision to
// the implementation; SURVEY.md §7 hard part 3). Consequence used throughout the
// build: a fetch at a texel centre (or an integer texel offset from one) returns
// that texel exactly, so those taps are plain loads.
struct Bilin {
  int x0, x1, y0, y1;
  float ax, ay;
};
GL_HD int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
GL_HD Bilin bilin_setup(float u, float v, int W, int H) {
  float tx = u * (float)W - 0.5f;
  float ty = v * (float)H - 0.5f;
  // 8-bit sub-texel fixed point (round to nearest); clamp keeps int conversion defined
  float qx = f_floor(f_clamp(tx, -4.0e6f, 4.0e6f) * 256.0f + 0.5f);
  float qy = f_floor(f_clamp(ty, -4.0e6f, 4.0e6f) * 256.0f + 0.5f);
  int ix = (int)qx, iy = (int)qy;
  int x0 = ix >> 8, y0 = iy >> 8;  // arithmetic shift = floor division by 256
  Bilin b;
  b.ax = (float)(ix & 255) * (1.0f / 256.0f);
  b.ay = (float)(iy & 255) * (1.0f / 256.0f);
  b.x0 = clampi(x0, 0, W - 1);
  b.x1 = clampi(x0 + 1, 0, W - 1);
  b.y0 = clampi(y0, 0, H - 1);
  b.y1 = clampi(y0 + 1, 0, H - 1);
  return b;
}
GL_HD float bilin_mix(const Bilin& b, float c00, float c10, float c01, float c11) {
  float top = c00 * (1.0f - b.ax) + c10 * b.ax;
  float bot = c01 * (1.0f - b.ax) + c11 * b.ax;
  return top * (1.0f - b.ay) + bot * b.ay;
}
// Fetch `nout` channels from a row-major image with `nch` floats per texel.
GL_HD void tex2d_linear(const float* img, int W, int H, int nch, float u, float v, float* out, int nout) {
  Bilin b = bilin_setup(u, v, W, H);
  const float* p00 = img + ((size_t)b.y0 * W + b.x0) * nch;
  const float* p10 = img + ((size_t)b.y0 * W + b.x1) * nch;
  const float* p01 = img + ((size_t)b.y1 * W + b.x0) * nch;
  const float* p11 = img + ((size_t)b.y1 * W + b.x1) * nch;
  for (int c = 0; c < nout; ++c) out[c] = bilin_mix(b, p00[c], p10[c], p01[c], p11[c]);
}

// --------------------------------------------------------------- hashing ---
// wang_hash (path_tracing.frag:438-445)
GL_HD uint32_t wang_hash(uint32_t* seed) {
  uint32_t s = *seed;
  s = (s ^ 61u) ^ (s >> 16);
  s *= 9u;
  s = s ^ (s >> 4);
  s *= 0x27d4eb2du;
  s = s ^ (s >> 15);
  *seed = s;
  return s;
}
// float(uint) / 4294967296.0 (path_tracing.frag:447-449); float(uint) rounds to
// nearest, so the result can be exactly 1.0.
GL_HD float u32_to_unit(uint32_t h) { return (float)h / 4294967296.0f; }

}  // namespace glsl

// Standalone timing experiment: step-specialised a-trous on RGBA planes (production
// kernel, included) vs a pixel-pair kernel on channel-paired planes (packed FP32).
// Synthetic 4K data; interior-only grid for the pair kernel (timing, and a bitwise
// comparison against the production kernel on the interior pixels).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include <cstring>
#include "../path-tracing-svgf_amd/csrc/kernels_atrous.hip"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

namespace ptk {
int launch_atrous_exact(const AtrousParams&, hipStream_t) { return 0; }
}

typedef float f2 __attribute__((ext_vector_type(2)));
struct __attribute__((aligned(16))) Pair { f2 c0, c1, c2, c3; };

__device__ __forceinline__ f2 pk_fma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

template <int S>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, 8))) atrous_pair_kernel(const Pair* __restrict__ I, const Pair* __restrict__ ND,
                                                          const float* __restrict__ aux, Pair* __restrict__ out,
                                                          int W, int H, float phi_color, float phi_normal, int kx0,
                                                          int y0) {
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int Wp = W >> 1;
  const int k = kx0 + blockIdx.x * 64 + (threadIdx.x & 63);
  const int y = y0 + blockIdx.y * 4 + wv;
  const Pair c = I[(size_t)y * Wp + k];
  const Pair n = ND[(size_t)y * Wp + k];
  const float LOG2E = 1.4426950408889634f;
  const f2 lc = (0.2125f * c.c0 + 0.7154f * c.c1) + 0.0721f * c.c2;
  f2 phiL;
  phiL.x = phi_color * __builtin_sqrtf(fmaxf(0.0f, 1e-10f + c.c3.x));
  phiL.y = phi_color * __builtin_sqrtf(fmaxf(0.0f, 1e-10f + c.c3.y));
  const f2 fwz = *(const f2*)(aux + (size_t)y * W + 2 * k);
  f2 kL, kD;
  kL.x = LOG2E / phiL.x;
  kL.y = LOG2E / phiL.y;
  kD.x = LOG2E / (fmaxf(fwz.x, 1e-8f) * (float)S);
  kD.y = LOG2E / (fmaxf(fwz.y, 1e-8f) * (float)S);
  const f2 wLr = 0.2125f * kL, wLg = 0.7154f * kL, wLb = 0.0721f * kL, cL = -(lc * kL);
  const f2 kD1 = kD, kD2 = kD * 0.70710678f, kD4 = kD * 0.5f, kD5 = kD * 0.44721360f, kD8 = kD * 0.35355339f;
  const f2 phiN = {phi_normal, phi_normal};
  f2 sumW = {1.0f, 1.0f}, s0 = c.c0, s1 = c.c1, s2 = c.c2, s3 = c.c3;
  auto tap = [&](const Pair& ip, const Pair& q, f2 kDl, float kern) __attribute__((always_inline)) {
    f2 dn = pk_fma(n.c2, q.c2, pk_fma(n.c1, q.c1, n.c0 * q.c0));
    dn = __builtin_elementwise_min(__builtin_elementwise_max(dn, f2{0.0f, 0.0f}), f2{1.0f, 1.0f});
    const f2 tl = pk_fma(ip.c2, wLb, pk_fma(ip.c1, wLg, pk_fma(ip.c0, wLr, cL)));
    const f2 dz = n.c3 - q.c3;
    f2 a;
    a.x = __builtin_fmaf(fabsf(dz.x), kDl.x, fabsf(tl.x));
    a.y = __builtin_fmaf(fabsf(dz.y), kDl.y, fabsf(tl.y));
    f2 lg;
    lg.x = __builtin_amdgcn_logf(dn.x);
    lg.y = __builtin_amdgcn_logf(dn.y);
    const f2 e = pk_fma(phiN, lg, -a);
    f2 w;
    w.x = __builtin_amdgcn_exp2f(e.x);
    w.y = __builtin_amdgcn_exp2f(e.y);
    w = w * kern;
    sumW += w;
    s0 = pk_fma(w, ip.c0, s0);
    s1 = pk_fma(w, ip.c1, s1);
    s2 = pk_fma(w, ip.c2, s2);
    s3 = pk_fma(w * w, ip.c3, s3);
  };
#if ROWLOOP
  // rows as runtime loops (one row of loads in flight per wave), in the production kernel's tap order
  auto outer_row = [&](int yy) __attribute__((always_inline)) {
    const int ay = yy < 0 ? -yy : yy;
    const float ky = ay == 1 ? 2.0f / 3.0f : 1.0f / 6.0f;
    const f2 kDa = ay == 1 ? kD2 : kD5;   // |xx| = 1
    const f2 kDb = ay == 1 ? kD5 : kD8;   // |xx| = 2
    const f2 kD0 = ay == 1 ? kD1 : kD4;   // xx = 0
    const Pair* __restrict__ Ir = I + (size_t)(y + yy * S) * Wp + k;
    const Pair* __restrict__ Nr = ND + (size_t)(y + yy * S) * Wp + k;
#pragma unroll
    for (int xx = -2; xx <= 2; ++xx) {
      const int ax = xx < 0 ? -xx : xx;
      const float kx = ax == 0 ? 1.0f : ax == 1 ? 2.0f / 3.0f : 1.0f / 6.0f;
      tap(Ir[xx * (S / 2)], Nr[xx * (S / 2)], ax == 0 ? kD0 : ax == 1 ? kDa : kDb, kx * ky);
    }
  };
#pragma unroll 1
  for (int yy = -2; yy < 0; ++yy) outer_row(yy);
  {
    const Pair* __restrict__ Ir = I + (size_t)y * Wp + k;
    const Pair* __restrict__ Nr = ND + (size_t)y * Wp + k;
    tap(Ir[-S], Nr[-S], kD4, 1.0f / 6.0f);
    tap(Ir[-S / 2], Nr[-S / 2], kD1, 2.0f / 3.0f);
    tap(Ir[S / 2], Nr[S / 2], kD1, 2.0f / 3.0f);
    tap(Ir[S], Nr[S], kD4, 1.0f / 6.0f);
  }
#pragma unroll 1
  for (int yy = 1; yy <= 2; ++yy) outer_row(yy);
#else
#pragma unroll
  for (int yy = -2; yy <= 2; ++yy) {
    const Pair* __restrict__ Ir = I + (size_t)(y + yy * S) * Wp + k;
    const Pair* __restrict__ Nr = ND + (size_t)(y + yy * S) * Wp + k;
#pragma unroll
    for (int xx = -2; xx <= 2; ++xx) {
      if (xx == 0 && yy == 0) continue;
      const int r2 = xx * xx + yy * yy;
      const f2 kDl = r2 == 1 ? kD1 : r2 == 2 ? kD2 : r2 == 4 ? kD4 : r2 == 5 ? kD5 : kD8;
      const int ax = xx < 0 ? -xx : xx, ay = yy < 0 ? -yy : yy;
      const float kern = (ax == 0 ? 1.0f : ax == 1 ? 2.0f / 3.0f : 1.0f / 6.0f) *
                         (ay == 0 ? 1.0f : ay == 1 ? 2.0f / 3.0f : 1.0f / 6.0f);
      tap(Ir[xx * (S / 2)], Nr[xx * (S / 2)], kDl, kern);
    }
  }
#endif
  f2 inv;
  inv.x = 1.0f / sumW.x;
  inv.y = 1.0f / sumW.y;
  Pair o;
  o.c0 = s0 * inv;
  o.c1 = s1 * inv;
  o.c2 = s2 * inv;
  o.c3 = s3 * (inv * inv);
  out[(size_t)y * Wp + k] = o;
}


// Probes on the RGBA layout (interior only): MODE 0 full math, 1 loads only (sum), 2 full math with every
// tap at the centre address (L1-resident: VALU-only time); zmul = 0 collapses offsets at run time.
template <int S, int MODE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(7, 8))) probe_kernel(const float4* __restrict__ I, const float4* __restrict__ ND,
                                                    const float* __restrict__ aux, float4* __restrict__ out, int W,
                                                    int H, float phi_color, float phi_normal, int zmul, int x0, int y0) {
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int x = x0 + blockIdx.x * 64 + (threadIdx.x & 63);
  const int y = y0 + blockIdx.y * 4 + wv;
  const float4 ic = I[(size_t)y * W + x];
  const float4 nd = ND[(size_t)y * W + x];
  const float LOG2E = 1.4426950408889634f;
  const float lc = (0.2125f * ic.x + 0.7154f * ic.y) + 0.0721f * ic.z;
  const float phiL = phi_color * __builtin_sqrtf(fmaxf(0.0f, 1e-10f + ic.w));
  const float kL = LOG2E / phiL;
  const float wLr = 0.2125f * kL, wLg = 0.7154f * kL, wLb = 0.0721f * kL, cL = -(lc * kL);
  const float kD = LOG2E / (fmaxf(aux[(size_t)y * W + x], 1e-8f) * (float)S);
  const float kD1 = kD, kD2 = kD * 0.70710678f, kD4 = kD * 0.5f, kD5 = kD * 0.44721360f, kD8 = kD * 0.35355339f;
  float sumW = 1.0f;
  f2 s01 = {ic.x, ic.y}, s23 = {ic.z, ic.w};
  const int dS = MODE == 2 ? S * zmul : S;
#pragma unroll
  for (int yy = -2; yy <= 2; ++yy) {
    const float4* __restrict__ Ir = I + (size_t)(y + yy * dS) * W + x;
    const float4* __restrict__ Nr = ND + (size_t)(y + yy * dS) * W + x;
#pragma unroll
    for (int xx = -2; xx <= 2; ++xx) {
      if (xx == 0 && yy == 0) continue;
      const float4 ip = Ir[xx * dS];
      const float4 q = Nr[xx * dS];
      if (MODE == 1) {
        s01 += f2{ip.x, ip.y} + f2{q.x, q.y};
        s23 += f2{ip.z, ip.w} + f2{q.z, q.w};
        continue;
      }
      const int r2 = xx * xx + yy * yy;
      const float kDl = r2 == 1 ? kD1 : r2 == 2 ? kD2 : r2 == 4 ? kD4 : r2 == 5 ? kD5 : kD8;
      const int ax = xx < 0 ? -xx : xx, ay = yy < 0 ? -yy : yy;
      const float kern = (ax == 0 ? 1.0f : ax == 1 ? 2.0f / 3.0f : 1.0f / 6.0f) *
                         (ay == 0 ? 1.0f : ay == 1 ? 2.0f / 3.0f : 1.0f / 6.0f);
      const float dn = fminf(fmaxf(__builtin_fmaf(nd.z, q.z, __builtin_fmaf(nd.y, q.y, nd.x * q.x)), 0.0f), 1.0f);
      const float tl = __builtin_fmaf(ip.z, wLb, __builtin_fmaf(ip.y, wLg, __builtin_fmaf(ip.x, wLr, cL)));
      const float a = __builtin_fmaf(fabsf(nd.w - q.w), kDl, fabsf(tl));
      const float w = __builtin_amdgcn_exp2f(__builtin_fmaf(phi_normal, __builtin_amdgcn_logf(dn), -a)) * kern;
      sumW += w;
      s01 = __builtin_elementwise_fma(f2{w, w}, f2{ip.x, ip.y}, s01);
      s23 = __builtin_elementwise_fma(f2{w, w * w}, f2{ip.z, ip.w}, s23);
    }
  }
  const float inv = 1.0f / sumW;
  out[(size_t)y * W + x] = float4{s01.x * inv, s01.y * inv, s23.x * inv, s23.y * (inv * inv)};
}

static float frand(uint32_t& s) {
  s = s * 1664525u + 1013904223u;
  return (s >> 8) * (1.0f / 16777216.0f);
}

int main(int argc, char** argv) {
  const int W = 3840, H = 2160, N = W * H;
  std::vector<float4> illum(N), nd(N);
  std::vector<float> fw(N);
  uint32_t s = 1;
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      int i = y * W + x;
      float sx = sinf(x * 0.01f), sy = cosf(y * 0.013f);
      illum[i] = {0.5f + 0.3f * sx + 0.05f * frand(s), 0.4f + 0.2f * sy + 0.05f * frand(s), 0.3f + 0.05f * frand(s),
                  0.01f + 0.02f * frand(s)};
      float nx = 0.2f * sx + 0.05f * frand(s), ny = 0.2f * sy, nz = 1.0f;
      float l = 1.0f / sqrtf(nx * nx + ny * ny + nz * nz);
      nd[i] = {nx * l, ny * l, nz * l, 2.0f + 0.5f * sx * sy};
      fw[i] = 0.001f + 0.002f * frand(s);
    }
  // paired copies
  std::vector<float> pil(N * 4), pnd(N * 4);
  for (int y = 0; y < H; ++y)
    for (int k = 0; k < W / 2; ++k)
      for (int h = 0; h < 2; ++h) {
        const float4 a = illum[y * W + 2 * k + h], b = nd[y * W + 2 * k + h];
        float* pa = &pil[((size_t)y * (W / 2) + k) * 8];
        float* pb = &pnd[((size_t)y * (W / 2) + k) * 8];
        pa[0 + h] = a.x; pa[2 + h] = a.y; pa[4 + h] = a.z; pa[6 + h] = a.w;
        pb[0 + h] = b.x; pb[2 + h] = b.y; pb[4 + h] = b.z; pb[6 + h] = b.w;
      }
  float4 *dI, *dN, *dO;
  float* dA;
  Pair *pI, *pN, *pO;
  CK(hipMalloc(&dI, N * 16)); CK(hipMalloc(&dN, N * 16)); CK(hipMalloc(&dO, N * 16)); CK(hipMalloc(&dA, N * 4));
  CK(hipMalloc(&pI, N * 16)); CK(hipMalloc(&pN, N * 16)); CK(hipMalloc(&pO, N * 16));
  CK(hipMemcpy(dI, illum.data(), N * 16, hipMemcpyHostToDevice));
  CK(hipMemcpy(dN, nd.data(), N * 16, hipMemcpyHostToDevice));
  CK(hipMemcpy(dA, fw.data(), N * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(pI, pil.data(), N * 16, hipMemcpyHostToDevice));
  CK(hipMemcpy(pN, pnd.data(), N * 16, hipMemcpyHostToDevice));
  ptk::AtrousParams p{};
  p.W = W; p.H = H; p.y0 = 0; p.y1 = H;
  p.illum = {dI, nullptr, W, 0, H};
  p.nd = {dN, nullptr, W, 0, H};
  p.fwidth = {nullptr, dA, W, 0, H};
  p.out = {dO, nullptr, W, 0, H};
  p.phi_color = 4.0f; p.phi_normal = 128.0f;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int steps[5] = {1, 2, 4, 8, 16};
  for (int si = 1; si < 5; ++si) {
    const int S = steps[si];
    p.step = S;
    // interior region for the pair kernel: pairs whose 5x5 footprint is inside
    const int m = 2 * S;                     // margin in pixels
    const int kx0 = (m + 1) / 2, kx1 = (W - m) / 2;  // pair range
    const int nbx = (kx1 - kx0) / 64, nby = (H - 2 * m) / 4;
    dim3 grid(nbx, nby);
    auto runpair = [&]() {
      switch (S) {
        case 2: hipLaunchKernelGGL(atrous_pair_kernel<2>, grid, dim3(256), 0, 0, pI, pN, dA, pO, W, H, 4.0f, 128.0f, kx0, m); break;
        case 4: hipLaunchKernelGGL(atrous_pair_kernel<4>, grid, dim3(256), 0, 0, pI, pN, dA, pO, W, H, 4.0f, 128.0f, kx0, m); break;
        case 8: hipLaunchKernelGGL(atrous_pair_kernel<8>, grid, dim3(256), 0, 0, pI, pN, dA, pO, W, H, 4.0f, 128.0f, kx0, m); break;
        case 16: hipLaunchKernelGGL(atrous_pair_kernel<16>, grid, dim3(256), 0, 0, pI, pN, dA, pO, W, H, 4.0f, 128.0f, kx0, m); break;
      }
    };
    float tb = 0, tp = 0;
    const int R = 50;
    for (int r = 0; r < 300; ++r) { ptk::launch_atrous_fast(p, 0); runpair(); }  // clocks up
    CK(hipDeviceSynchronize());
    for (int r = 0; r < R + 2; ++r) {
      float ms;
      CK(hipEventRecord(e0)); ptk::launch_atrous_fast(p, 0); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1)); if (r >= 2) tb += ms;
      CK(hipEventRecord(e0)); runpair(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1)); if (r >= 2) tp += ms;
    }
    {
      const int px0 = 2 * S, nbx2 = (W - 4 * S) / 64, nby2 = (H - 4 * S) / 4;
      dim3 g2(nbx2, nby2);
      float tm[3] = {0, 0, 0};
      for (int r = 0; r < R; ++r)
        for (int md = 0; md < 3; ++md) {
          float ms;
          CK(hipEventRecord(e0));
#define PROBE(SS) if (S == SS) { if (md == 0) hipLaunchKernelGGL((probe_kernel<SS, 0>), g2, dim3(256), 0, 0, dI, dN, dA, dO, W, H, 4.0f, 128.0f, 0, px0, px0); \
            if (md == 1) hipLaunchKernelGGL((probe_kernel<SS, 1>), g2, dim3(256), 0, 0, dI, dN, dA, dO, W, H, 4.0f, 128.0f, 0, px0, px0); \
            if (md == 2) hipLaunchKernelGGL((probe_kernel<SS, 2>), g2, dim3(256), 0, 0, dI, dN, dA, dO, W, H, 4.0f, 128.0f, 0, px0, px0); }
          PROBE(2) PROBE(4) PROBE(8) PROBE(16)
          CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
          CK(hipEventElapsedTime(&ms, e0, e1)); tm[md] += ms;
        }
      const double sc = (double)N / ((double)nbx2 * 64 * nby2 * 4);
      printf("   probe S=%2d (full-frame equiv): full %.1f us, loads-only %.1f us, math-only %.1f us\n", S,
             tm[0] / R * 1e3 * sc, tm[1] / R * 1e3 * sc, tm[2] / R * 1e3 * sc);
    }
    CK(hipGetLastError());
    // compare interior pixels bitwise
    std::vector<float4> ob(N);
    std::vector<float> op(N * 4);
    CK(hipMemcpy(ob.data(), dO, N * 16, hipMemcpyDeviceToHost));
    CK(hipMemcpy(op.data(), pO, N * 16, hipMemcpyDeviceToHost));
    long bad = 0, tot = 0;
    for (int y = m; y < m + nby * 4; ++y)
      for (int k = kx0; k < kx0 + nbx * 64; ++k)
        for (int h = 0; h < 2; ++h) {
          const float4 a = ob[y * W + 2 * k + h];
          const float* q = &op[((size_t)y * (W / 2) + k) * 8];
          float b[4] = {q[0 + h], q[2 + h], q[4 + h], q[6 + h]};
          float av[4] = {a.x, a.y, a.z, a.w};
          for (int c = 0; c < 4; ++c) bad += memcmp(&av[c], &b[c], 4) != 0;
          tot += 4;
        }
    const double px_pair = (double)nbx * 64 * 2 * nby * 4;
    printf("S=%2d base %.1f us (%.0f GB/s @52B/px full frame)  pair %.1f us over %.0f%% of px -> %.1f us full-frame equiv (%.0f GB/s)  mismatches %ld/%ld\n",
           S, tb / R * 1e3, 52.0 * N / (tb / R * 1e-3) / 1e9, tp / R * 1e3, 100.0 * px_pair / N,
           tp / R * 1e3 * N / px_pair, 52.0 * px_pair / (tp / R * 1e-3) / 1e9, bad, tot);
  }
  return 0;
}

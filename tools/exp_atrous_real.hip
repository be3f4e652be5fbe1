// Standalone a-trous experiments on the real 4K bench-frame inputs (tools/dump_atrous_inputs.py).
// Variants of the production step kernel (kernels_atrous.hip), interior + edge, full frame:
//   V_PROD   production launcher (included)
//   V_AUXBG  background detected from the sign of the compact depth-fwidth plane (nd not read for background)
//   V_LOADS  probe: loads only (no weight math)
//   V_MATH   probe: every tap reads the centre address (L1-resident): VALU-only time
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include <cstring>
#include <string>
#include "../path-tracing-svgf_amd/csrc/kernels_atrous.hip"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

namespace ptk {
int launch_atrous_exact(const AtrousParams&, hipStream_t) { return 0; }
}
using ptk::f2v;

enum { V_AUXBG = 1, V_LOADS = 2, V_MATH = 3, V_COPY = 4, V_COPY1 = 5, V_FGONLY = 6 };

template <int S, int V>
__global__ void __launch_bounds__(256) exp_kernel(const float4* __restrict__ I, const float4* __restrict__ ND,
                                                  const float* __restrict__ aux, float4* __restrict__ out, int W,
                                                  int H, float phi_color, float phi_normal, int zmul) {
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int x0 = blockIdx.x * 64;
  const int y = blockIdx.y * 4 + wv;
  const int x = x0 + (threadIdx.x & 63);
  if (y >= H || x >= W) return;
  const bool interior = x0 - 2 * S >= 0 && x0 + 63 + 2 * S < W && (int)(blockIdx.y * 4) - 2 * S >= 0 &&
                        (int)(blockIdx.y * 4) + 3 + 2 * S < H;
  const size_t ci = (size_t)y * W + x;
  float4 ic, nd;
  float fwz;
  if (V == V_COPY) {
    ic = I[ci];
    nd = ND[ci];
    out[ci] = float4{ic.x, ic.y, ic.z, nd.w};
    return;
  }
  if (V == V_COPY1) {
    out[ci] = I[ci];
    return;
  }
  if (V == V_AUXBG) {
    fwz = aux[ci];
    ic = I[ci];
    if (fwz < 0.0f) {  // background (sign bit set by the G-buffer)
      out[ci] = ic;
      return;
    }
    nd = ND[ci];
  } else {
    ic = I[ci];
    nd = ND[ci];
    if (nd.w == 1.0f) {
      if (V != V_FGONLY) out[ci] = ic;
      return;
    }
    fwz = fabsf(aux[ci]);
  }
  const float LOG2E = 1.4426950408889634f;
  const float lc = (0.2125f * ic.x + 0.7154f * ic.y) + 0.0721f * ic.z;
  const float phiL = phi_color * __builtin_sqrtf(fmaxf(0.0f, 1e-10f + ic.w));
  const float kL = LOG2E / phiL;
  const float wLr = 0.2125f * kL, wLg = 0.7154f * kL, wLb = 0.0721f * kL, cL = -(lc * kL);
  const float kD = LOG2E / (fmaxf(fwz, 1e-8f) * (float)S);
  const float kD1 = kD, kD2 = kD * 0.70710678f, kD4 = kD * 0.5f, kD5 = kD * 0.44721360f, kD8 = kD * 0.35355339f;
  float sumW = 1.0f;
  f2v s01 = {ic.x, ic.y}, s23 = {ic.z, ic.w};
  const int dS = V == V_MATH ? S * zmul : S;
#pragma unroll
  for (int yy = -2; yy <= 2; ++yy) {
    const int py = y + yy * dS;
    if (!interior && (py < 0 || py >= H)) continue;
    const float4* __restrict__ Ir = I + (size_t)py * W;
    const float4* __restrict__ Nr = ND + (size_t)py * W;
#pragma unroll
    for (int xx = -2; xx <= 2; ++xx) {
      if (xx == 0 && yy == 0) continue;
      const int px = x + xx * dS;
      if (!interior && (px < 0 || px >= W)) continue;
      const float4 ip = Ir[px];
      const float4 q = Nr[px];
      if (V == V_LOADS) {
        s01 += f2v{ip.x, ip.y} + f2v{q.x, q.y};
        s23 += f2v{ip.z, ip.w} + f2v{q.z, q.w};
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
      s01 = __builtin_elementwise_fma(f2v{w, w}, f2v{ip.x, ip.y}, s01);
      s23 = __builtin_elementwise_fma(f2v{w, w * w}, f2v{ip.z, ip.w}, s23);
    }
  }
  const float inv = 1.0f / sumW;
  out[ci] = float4{s01.x * inv, s01.y * inv, s23.x * inv, s23.y * (inv * inv)};
}

template <int V>
static void launch_exp(int S, dim3 g, const float4* I, const float4* N, const float* A, float4* O, int W, int H) {
  switch (S) {
    case 1: hipLaunchKernelGGL((exp_kernel<1, V>), g, dim3(256), 0, 0, I, N, A, O, W, H, 4.0f, 128.0f, 0); break;
    case 2: hipLaunchKernelGGL((exp_kernel<2, V>), g, dim3(256), 0, 0, I, N, A, O, W, H, 4.0f, 128.0f, 0); break;
    case 4: hipLaunchKernelGGL((exp_kernel<4, V>), g, dim3(256), 0, 0, I, N, A, O, W, H, 4.0f, 128.0f, 0); break;
    case 8: hipLaunchKernelGGL((exp_kernel<8, V>), g, dim3(256), 0, 0, I, N, A, O, W, H, 4.0f, 128.0f, 0); break;
    case 16: hipLaunchKernelGGL((exp_kernel<16, V>), g, dim3(256), 0, 0, I, N, A, O, W, H, 4.0f, 128.0f, 0); break;
  }
}


// ---------------------------------------------------------------------------------------------
// LDS-tiled a-trous. A block computes 64 columns x TJ rows taken from ONE residue class of rows
// mod S (rows ybase + S*j), so its whole 5x5 dilated footprint is a dense (TJ+4) x (64+4S) texel
// tile: staged once into LDS (2 planes), the 24 taps then read LDS, not the texture path.
// Background (sign bit of the compact depth-fwidth plane) tiles copy and exit.
__device__ __forceinline__ bool bgflag(float a) { return (__float_as_uint(a) >> 31) != 0; }

// Block = TJ*NX waves, one pixel per thread; tile = 64*NX columns x TJ rows of one residue class mod S.
template <int S, int TJ, int NX>
__global__ void __launch_bounds__(64 * TJ * NX) atrous_tile_kernel(const float4* __restrict__ I,
                                                              const float4* __restrict__ ND,
                                                              const float* __restrict__ aux, float4* __restrict__ out,
                                                              int W, int H, int Y0, int Y1, float phi_color,
                                                              float phi_normal) {
  constexpr int R = TJ + 4, C = 64 * NX + 4 * S, NT = 64 * TJ * NX;
  __shared__ float4 LI[R * C];
  __shared__ float4 LN[R * C];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int j = wv / NX, xl = (wv % NX) * 64 + lane;
  const int g = blockIdx.y / S, b = blockIdx.y - g * S;
  const int ybase = Y0 + g * S * TJ + b;
  const int x0 = blockIdx.x * 64 * NX, x = x0 + xl, y = ybase + S * j;
  const bool own = x < W && y < Y1;
  const size_t ci = (size_t)y * W + x;
  bool bg = true;
  float fwz = 0.0f;
  if (own) {
    const float a = aux[ci];
    bg = bgflag(a);
    fwz = fabsf(a);
  }
  if (!__syncthreads_or(!bg)) {
    if (own) out[ci] = I[ci];
    return;
  }
  for (int e = tid; e < R * C; e += NT) {
    const int r = e / C, c = e - r * C;
    int gy = ybase + S * (r - 2), gx = x0 - 2 * S + c;
    gy = gy < 0 ? 0 : (gy >= H ? H - 1 : gy);
    gx = gx < 0 ? 0 : (gx >= W ? W - 1 : gx);
    const size_t gi = (size_t)gy * W + gx;
    LI[e] = I[gi];
    LN[e] = ND[gi];
  }
  __syncthreads();
  if (!own) return;
  const float4* Li = LI + j * C + xl;
  const float4* Ln = LN + j * C + xl;
  const float4 ic = Li[2 * C + 2 * S];
  if (bg) {
    out[ci] = ic;
    return;
  }
  const float4 nd = Ln[2 * C + 2 * S];
  const bool edge = x0 - 2 * S < 0 || x0 + 64 * NX - 1 + 2 * S >= W || ybase - 2 * S < 0 || ybase + S * (TJ + 1) >= H;
  const float LOG2E = 1.4426950408889634f;
  const float lc = (0.2125f * ic.x + 0.7154f * ic.y) + 0.0721f * ic.z;
  const float phiL = phi_color * __builtin_sqrtf(fmaxf(0.0f, 1e-10f + ic.w));
  const float kL = LOG2E / phiL;
  const float kD = LOG2E / (fmaxf(fwz, 1e-8f) * (float)S);
  const float kDr[5] = {kD, kD * 0.70710678f, kD * 0.5f, kD * 0.44721360f, kD * 0.35355339f};
  float sumW = 1.0f;
  f2v s01 = {ic.x, ic.y}, s23 = {ic.z, ic.w};
  const float wLr = 0.2125f * kL, wLg = 0.7154f * kL, wLb = 0.0721f * kL, cL = -(lc * kL);
#pragma unroll
  for (int yy = -2; yy <= 2; ++yy) {
    if (edge && (y + yy * S < 0 || y + yy * S >= H)) continue;
#pragma unroll
    for (int xx = -2; xx <= 2; ++xx) {
      if (xx == 0 && yy == 0) continue;
      if (edge && (x + xx * S < 0 || x + xx * S >= W)) continue;
      const int r2 = xx * xx + yy * yy;
      const float kDl = r2 == 1 ? kDr[0] : r2 == 2 ? kDr[1] : r2 == 4 ? kDr[2] : r2 == 5 ? kDr[3] : kDr[4];
      const int ax = xx < 0 ? -xx : xx, ay = yy < 0 ? -yy : yy;
      const float kern = (ax == 0 ? 1.0f : ax == 1 ? 2.0f / 3.0f : 1.0f / 6.0f) *
                         (ay == 0 ? 1.0f : ay == 1 ? 2.0f / 3.0f : 1.0f / 6.0f);
      const int o = (yy + 2) * C + (xx + 2) * S;
      const float4 ip = Li[o];
      const float4 q = Ln[o];
      const float dn = fminf(fmaxf(__builtin_fmaf(nd.z, q.z, __builtin_fmaf(nd.y, q.y, nd.x * q.x)), 0.0f), 1.0f);
      const float tl = __builtin_fmaf(ip.z, wLb, __builtin_fmaf(ip.y, wLg, __builtin_fmaf(ip.x, wLr, cL)));
      const float a = __builtin_fmaf(fabsf(nd.w - q.w), kDl, fabsf(tl));
      const float w = __builtin_amdgcn_exp2f(__builtin_fmaf(phi_normal, __builtin_amdgcn_logf(dn), -a)) * kern;
      sumW += w;
      s01 = __builtin_elementwise_fma(f2v{w, w}, f2v{ip.x, ip.y}, s01);
      s23 = __builtin_elementwise_fma(f2v{w, w * w}, f2v{ip.z, ip.w}, s23);
    }
  }
  const float inv = 1.0f / sumW;
  out[ci] = float4{s01.x * inv, s01.y * inv, s23.x * inv, s23.y * (inv * inv)};
}

template <int S, int TJ, int NX>
static void lt(const float4* I, const float4* N, const float* A, float4* O, int W, int H) {
  dim3 grid((W + 64 * NX - 1) / (64 * NX), ((H + S * TJ - 1) / (S * TJ)) * S);
  hipLaunchKernelGGL((atrous_tile_kernel<S, TJ, NX>), grid, dim3(64 * TJ * NX), 0, 0, I, N, A, O, W, H, 0, H, 4.0f,
                     128.0f);
}
static int g_cfg = 0;
static const char* cfg_names[6] = {"TJ8 NX1", "TJ4 NX2", "TJ8 NX2", "TJ4 NX4", "TJ2 NX4", "TJ16 NX1"};
template <int S>
static void lts(const float4* I, const float4* N, const float* A, float4* O, int W, int H) {
  if (g_cfg == 0) lt<S, 8, 1>(I, N, A, O, W, H);
  if (g_cfg == 1) lt<S, 4, 2>(I, N, A, O, W, H);
  if (g_cfg == 2) lt<S, 8, 2>(I, N, A, O, W, H);
  if (g_cfg == 3) lt<S, 4, 4>(I, N, A, O, W, H);
  if (g_cfg == 4) lt<S, 2, 4>(I, N, A, O, W, H);
  if (g_cfg == 5) lt<S, 16, 1>(I, N, A, O, W, H);
}
static void launch_tile(int S, const float4* I, const float4* N, const float* A, float4* O, int W, int H) {
  switch (S) {
    case 1: lts<1>(I, N, A, O, W, H); break;
    case 2: lts<2>(I, N, A, O, W, H); break;
    case 4: lts<4>(I, N, A, O, W, H); break;
    case 8: lts<8>(I, N, A, O, W, H); break;
    case 16: lts<16>(I, N, A, O, W, H); break;
  }
}

static bool load(const std::string& f, void* dst, size_t bytes) {
  FILE* fp = fopen(f.c_str(), "rb");
  if (!fp) return false;
  size_t n = fread(dst, 1, bytes, fp);
  fclose(fp);
  return n == bytes;
}

int main(int argc, char** argv) {
  const int W = 3840, H = 2160, N = W * H;
  const std::string base = argc > 1 ? argv[1] : "/tmp/atrous_in";
  std::vector<float4> illum(N), nd(N);
  std::vector<float> aux(N);
  if (!load(base + "_illum.f32", illum.data(), N * 16ull) || !load(base + "_nd.f32", nd.data(), N * 16ull) ||
      !load(base + "_aux.f32", aux.data(), N * 4ull)) {
    printf("cannot read %s_*.f32\n", base.c_str());
    return 1;
  }
  std::vector<float> auxpos(N);
  for (int i = 0; i < N; ++i) auxpos[i] = fabsf(aux[i]);
  float4 *dI, *dN, *dO, *dO2;
  float *dA, *dAp;
  CK(hipMalloc(&dI, N * 16ull)); CK(hipMalloc(&dN, N * 16ull)); CK(hipMalloc(&dO, N * 16ull));
  CK(hipMalloc(&dO2, N * 16ull)); CK(hipMalloc(&dA, N * 4ull)); CK(hipMalloc(&dAp, N * 4ull));
  CK(hipMemcpy(dI, illum.data(), N * 16ull, hipMemcpyHostToDevice));
  CK(hipMemcpy(dN, nd.data(), N * 16ull, hipMemcpyHostToDevice));
  CK(hipMemcpy(dA, aux.data(), N * 4ull, hipMemcpyHostToDevice));
  CK(hipMemcpy(dAp, auxpos.data(), N * 4ull, hipMemcpyHostToDevice));
  ptk::AtrousParams p{};
  p.W = W; p.H = H; p.y0 = 0; p.y1 = H;
  p.illum = {dI, nullptr, W, 0, H};
  p.nd = {dN, nullptr, W, 0, H};
  p.fwidth = {nullptr, dA, W, 0, H};
  p.out = {dO, nullptr, W, 0, H};
  p.phi_color = 4.0f; p.phi_normal = 128.0f;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  dim3 g((W + 63) / 64, (H + 3) / 4);
  const char* names[7] = {"prod", "tile", "loads", "math", "copy2", "copy1", "fgonly"};
  for (int r = 0; r < 200; ++r) { p.step = 4; ptk::launch_atrous_fast(p, 0); }  // clocks up
  CK(hipDeviceSynchronize());
  if (argc > 3) {  // profiling mode: variant argv[2], step argv[3], 20 launches
    const int v = atoi(argv[2]), S = atoi(argv[3]);
    p.step = S;
    for (int r = 0; r < 20; ++r) {
      if (v == 0) ptk::launch_atrous_fast(p, 0);
      if (v == 6) launch_exp<V_FGONLY>(S, g, dI, dN, dAp, dO2, W, H);
      if (v == 1) launch_tile(S, dI, dN, dA, dO2, W, H);
      if (v == 3) launch_exp<V_MATH>(S, g, dI, dN, dAp, dO2, W, H);
      if (v == 2) launch_exp<V_LOADS>(S, g, dI, dN, dAp, dO2, W, H);
    }
    CK(hipDeviceSynchronize());
    return 0;
  }
  for (int S : {1, 2, 4, 8, 16}) {  // tile statistics (TJ = 8, 64 columns)
    long tiles = 0, fgt = 0, fgpx = 0, wavesfg = 0;
    for (int y0 = 0; y0 < H; y0 += 8 * S)
      for (int b = 0; b < S; ++b)
        for (int x0 = 0; x0 < W; x0 += 64) {
          bool any = false;
          long n = 0;
          int wf = 0;
          for (int j = 0; j < 8; ++j) {
            const int y = y0 + b + S * j;
            if (y >= H) continue;
            bool wany = false;
            for (int x = x0; x < x0 + 64 && x < W; ++x)
              if (!(__builtin_bit_cast(uint32_t, aux[(size_t)y * W + x]) >> 31)) { any = true; wany = true; ++n; }
            wf += wany;
          }
          ++tiles;
          if (any) { ++fgt; fgpx += n; wavesfg += wf; }
        }
    printf("S=%2d tiles %ld fg tiles %.1f%%  fg px %.1f%% of frame  fg waves in fg tiles %.1f%%\n", S, tiles,
           100.0 * fgt / tiles, 100.0 * fgpx / N, 100.0 * wavesfg / (8.0 * fgt));
  }
  const int R = 30;
  const int ncfg = getenv("NCFG") ? atoi(getenv("NCFG")) : 1;
  for (int cfg = 0; cfg < ncfg; ++cfg) {
  g_cfg = cfg;
  printf("tile cfg %s\n", cfg_names[cfg]);
  for (int S : {1, 2, 4, 8, 16}) {
    p.step = S;
    double t[7] = {0, 0, 0, 0, 0, 0, 0};
    for (int r = 0; r < R; ++r)
      for (int v = 0; v < 7; ++v) {
        float ms;
        CK(hipEventRecord(e0));
        if (v == 0) ptk::launch_atrous_fast(p, 0);
        if (v == 1) launch_tile(S, dI, dN, dA, dO2, W, H);
        if (v == 2) launch_exp<V_LOADS>(S, g, dI, dN, dAp, dO2, W, H);
        if (v == 3) launch_exp<V_MATH>(S, g, dI, dN, dAp, dO2, W, H);
        if (v == 4) launch_exp<V_COPY>(S, g, dI, dN, dAp, dO2, W, H);
        if (v == 5) launch_exp<V_COPY1>(S, g, dI, dN, dAp, dO2, W, H);
        if (v == 6) launch_exp<V_FGONLY>(S, g, dI, dN, dAp, dO2, W, H);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        t[v] += ms;
      }
    CK(hipGetLastError());
    // bitwise check of the result-preserving variant against production
    ptk::launch_atrous_fast(p, 0);
    launch_tile(S, dI, dN, dA, dO2, W, H);
    CK(hipDeviceSynchronize());
    std::vector<float4> a(N), b(N);
    CK(hipMemcpy(a.data(), dO, N * 16ull, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), dO2, N * 16ull, hipMemcpyDeviceToHost));
    const long bad = memcmp(a.data(), b.data(), N * 16ull) ? 1 : 0;
    printf("S=%2d", S);
    for (int v = 0; v < 7; ++v) printf("  %s %.1f", names[v], t[v] / R * 1e3);
    printf("  tile==prod: %s\n", bad ? "NO" : "yes");
  }
  }
  return 0;
}

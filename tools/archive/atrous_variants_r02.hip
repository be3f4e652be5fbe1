// ARCHIVED a-trous variants (round 2), measured SLOWER than the production atrous_tile_kernel and removed from
// the product library in round 3 (VERDICT r02 "prune the product library"). Kept as the record behind DESIGN.md's
// "measured and not kept" notes; NOT compiled (they need kernels_atrous.hip's helpers and the AtrousParams of
// round 2, which also carried `xcd_run`).
//  * atrous_slide_kernel (atrous_variant=4): an LDS ring sliding down a residue class; 72 -> 88-116 us default view,
//    145 -> 157-173 us surface view (profiles/r02/atrous_ab_slide.log).
//  * atrous_pair_kernel (atrous_variant=3): packed pixel pairs on a channel-planar LDS tile; 76 -> 108.7 us default,
//    152 -> 178 us surface view.
//  * xcd_run (tile kernel, runs of C consecutive tiles per XCD): 72 -> 78-79 us (profiles/r02/atrous_ab_xcd_run.log).
//  * PT_ATROUS_BATCH=1 (every staging load before the first LDS write): 76 -> 102 us, 152 -> 219 us.

// ---------------------------------------------------------------------------
// Sliding form. The tiled kernel stages (TJ + 4) rows of each plane for TJ output rows: the 4 halo rows (1.5x
// staged rows) are fetched again by the tile above and the tile below, and on 4K frames those re-reads come from
// the fabric, not L2 (PMC FETCH ~ staged bytes). Here a block walks DOWN its residue class: chunk k outputs class
// rows 8k .. 8k+7 and needs class rows 8k-2 .. 8k+9; the 12 staged rows live in an LDS ring (class row i in slot
// (i + 2) mod 12), so a chunk following a staged chunk loads only its 8 new rows. Chunks whose pixels are all
// background copy from HBM and stage nothing (the ring keeps what it holds). Same taps, same arithmetic, same
// order as atrous_taps: bit-identical to the step and tiled kernels.
// XCD: with `xcd`, linear block L runs tile (L % 8) * (N / 8) + L / 8, so each XCD (blocks L = 8i + x land on XCD
// x) walks a contiguous run of column tiles and the horizontal halos neighbouring tiles share stay in its L2.
template <int S, int NX, bool AUX>
__global__ void __launch_bounds__(64 * kTileWaves * NX) atrous_slide_kernel(AtrousParams p, int chunks, int xcd) {
  constexpr int TJ = kTileRows, NW = kTileWaves * NX, R = TJ + 4, C = 64 * NX + 4 * S, NT = 64 * NW;
  __shared__ float4 LI[R * C];
  __shared__ float4 LN[R * C];
  __shared__ int any_surface[2][NW];
  const int W = p.illum.W, row0 = p.illum.row0;
  const float4* __restrict__ I = p.illum.p;
  const float4* __restrict__ ND = p.nd.p;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  int bx = blockIdx.x, by = blockIdx.y;
  if (xcd) {
    const int N = gridDim.x * gridDim.y, L = by * gridDim.x + bx, per = N >> 3;
    const int t = L < (per << 3) ? (L & 7) * per + (L >> 3) : L;
    by = t / gridDim.x;
    bx = t - by * gridDim.x;
  }
  const int seg = by / S, b = by - seg * S;
  const int j = wv / NX, xl = (wv - j * NX) * 64 + lane;  // tile row, tile column
  const int x0 = bx * 64 * NX, x = x0 + xl;
  const int lo = max(0, row0), hi = min(p.H, row0 + p.illum.rows) - 1;
  const bool xedge = x0 - 2 * S < 0 || x0 + 64 * NX - 1 + 2 * S >= p.W;
  int rlo = 0, rhi = 0;  // ring holds u = class row + 2 in [rlo, rhi)
  const int k0 = seg * chunks;
  for (int k = k0; k < k0 + chunks; ++k) {
    const int ybase = p.y0 + b + S * TJ * k;  // frame row of chunk row 0 (block-uniform)
    if (ybase >= p.y1) break;
    const int y = ybase + S * j;
    const bool own = x < p.W && y < p.y1;
    const size_t ci = (size_t)(y - row0) * W + x;
    bool bg = true;
    float fwz = 0.0f;
    if (own) {
      if (AUX) {
        const float a = p.fwidth.aux[ci];
        bg = aux_flag(a);
        fwz = fabsf(a);
      } else {
        bg = ND[ci].w == 1.0f;
        fwz = p.fwidth.p[ci].y;
      }
    }
    const bool wave_any = __ballot(!bg) != 0ull;
    if (lane == 0) any_surface[k & 1][wv] = wave_any;
    __syncthreads();  // also: every thread is done with the previous chunk's ring reads
    bool tile_any = false;
#pragma unroll
    for (int w = 0; w < NW; ++w) tile_any |= any_surface[k & 1][w] != 0;
    if (!tile_any) {
      if (own) p.out.p[ci] = I[ci];
      continue;
    }
    const int ua = TJ * k, ub = ua + R;  // rows this chunk reads
    const int us = (rhi > ua && rlo <= ua) ? rhi : ua;
    for (int e = tid; e < (ub - us) * C; e += NT) {
      const int rr = e / C, c = e - rr * C, u = us + rr;
      int gy = p.y0 + b + S * (u - 2), gx = x0 - 2 * S + c;
      gy = gy < lo ? lo : (gy > hi ? hi : gy);
      gx = gx < 0 ? 0 : (gx >= p.W ? p.W - 1 : gx);
      const size_t gi = (size_t)(gy - row0) * W + gx;
      const int li = (u % R) * C + c;
      LI[li] = I[gi];
      LN[li] = ND[gi];
    }
    rlo = ua;
    rhi = ub;
    __syncthreads();
    if (!own) continue;
    const int sb = (ua + j) % R;  // slot of this pixel's tap row yy = -2
    int so[5];
#pragma unroll
    for (int t = 0; t < 5; ++t) so[t] = (sb + t >= R ? sb + t - R : sb + t) * C + xl;
    const float4 ic = LI[so[2] + 2 * S];
    float4* out = p.out.p + ci;
    if (bg) {
      *out = ic;
      continue;
    }
    const float4 nd = LN[so[2] + 2 * S];
    const bool edge = xedge || ybase - 2 * S < 0 || ybase + S * (TJ + 1) >= p.H;
    const float LOG2E = 1.4426950408889634f;
    const float lc = (0.2125f * ic.x + 0.7154f * ic.y) + 0.0721f * ic.z;
    const float phiL = p.phi_color * __builtin_sqrtf(fmaxf(0.0f, 1e-10f + ic.w));
    const float kL = LOG2E / phiL;
    const float kD = LOG2E / (fmaxf(fwz, 1e-8f) * (float)S);
    const float kDr[5] = {kD, kD * 0.70710678f, kD * 0.5f, kD * 0.44721360f, kD * 0.35355339f};
    float sumW = 1.0f;
    f2v s01 = {ic.x, ic.y}, s23 = {ic.z, ic.w};
    auto taps = [&](auto flat_tag) __attribute__((always_inline)) {
      constexpr bool FLAT = decltype(flat_tag)::value;
      const float wLr = 0.2125f * kL, wLg = 0.7154f * kL, wLb = 0.0721f * kL, cL = -(lc * kL);
#pragma unroll
      for (int yy = -2; yy <= 2; ++yy) {
        if (edge && (y + yy * S < 0 || y + yy * S >= p.H)) continue;
#pragma unroll
        for (int xx = -2; xx <= 2; ++xx) {
          if (xx == 0 && yy == 0) continue;
          if (edge && (x + xx * S < 0 || x + xx * S >= p.W)) continue;
          const int r2 = xx * xx + yy * yy;
          const float kDl = r2 == 1 ? kDr[0] : r2 == 2 ? kDr[1] : r2 == 4 ? kDr[2] : r2 == 5 ? kDr[3] : kDr[4];
          const int ax = xx < 0 ? -xx : xx, ay = yy < 0 ? -yy : yy;
          const float kern = (ax == 0 ? 1.0f : ax == 1 ? 2.0f / 3.0f : 1.0f / 6.0f) *
                             (ay == 0 ? 1.0f : ay == 1 ? 2.0f / 3.0f : 1.0f / 6.0f);
          const int o = so[yy + 2] + (xx + 2) * S;
          const float4 ip = LI[o];
          const float4 q = LN[o];
          const float dn =
              fminf(fmaxf(__builtin_fmaf(nd.z, q.z, __builtin_fmaf(nd.y, q.y, nd.x * q.x)), 0.0f), 1.0f);
          float a;
          if (FLAT) {
            const float lp = (0.2125f * ip.x + 0.7154f * ip.y) + 0.0721f * ip.z;
            a = lp == lc ? fabsf(nd.w - q.w) * kDl : __builtin_inff();
          } else {
            const float tl = __builtin_fmaf(ip.z, wLb, __builtin_fmaf(ip.y, wLg, __builtin_fmaf(ip.x, wLr, cL)));
            a = __builtin_fmaf(fabsf(nd.w - q.w), kDl, fabsf(tl));
          }
          const float w = __builtin_amdgcn_exp2f(__builtin_fmaf(p.phi_normal, __builtin_amdgcn_logf(dn), -a)) * kern;
          sumW += w;
          s01 = __builtin_elementwise_fma(f2v{w, w}, f2v{ip.x, ip.y}, s01);
          s23 = __builtin_elementwise_fma(f2v{w, w * w}, f2v{ip.z, ip.w}, s23);
        }
      }
    };
    if (__builtin_expect(phiL > 0.0f, 1)) taps(std::false_type{});
    else taps(std::true_type{});
    const float inv = 1.0f / sumW;
    *out = float4{s01.x * inv, s01.y * inv, s23.x * inv, s23.y * (inv * inv)};
  }
}

template <int S, int NX>
static void launch_slide_snx(const AtrousParams& p, bool aux, int chunks, int xcd, hipStream_t s) {
  const int class_rows = (p.y1 - p.y0 + S - 1) / S;        // rows of the largest residue class
  const int nchunk = (class_rows + kTileRows - 1) / kTileRows;
  const int segs = (nchunk + chunks - 1) / chunks;
  dim3 grid((p.W + 64 * NX - 1) / (64 * NX), segs * S);
  if (aux) hipLaunchKernelGGL((atrous_slide_kernel<S, NX, true>), grid, dim3(64 * kTileWaves * NX), 0, s, p, chunks, xcd);
  else hipLaunchKernelGGL((atrous_slide_kernel<S, NX, false>), grid, dim3(64 * kTileWaves * NX), 0, s, p, chunks, xcd);
}

template <int S>
static void launch_slide_s(const AtrousParams& p, bool aux, int chunks, int nx, int xcd, hipStream_t s) {
  if ((nx ? nx : tile_nx<S>()) == 2) launch_slide_snx<S, 2>(p, aux, chunks, xcd, s);
  else launch_slide_snx<S, 1>(p, aux, chunks, xcd, s);
}

int launch_atrous_slide(const AtrousParams& p, int chunks, int nx, int xcd, hipStream_t s) {
  if (p.y1 <= p.y0) return 0;
  if (!same_geometry(p)) return launch_atrous_simple(p, s);
  const bool aux = p.fwidth.aux != nullptr;
  chunks = chunks < 1 ? 1 : chunks;
  switch (p.step) {
    case 1: launch_slide_s<1>(p, aux, chunks, nx, xcd, s); break;
    case 2: launch_slide_s<2>(p, aux, chunks, nx, xcd, s); break;
    case 4: launch_slide_s<4>(p, aux, chunks, nx, xcd, s); break;
    case 8: launch_slide_s<8>(p, aux, chunks, nx, xcd, s); break;
    case 16: launch_slide_s<16>(p, aux, chunks, nx, xcd, s); break;
    default: return launch_atrous_step(p, s);
  }
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Pixel-pair form: packed FP32 on a channel-planar LDS tile. On surface-heavy
// frames the tiled kernel above is compute/latency-bound, not HBM-bound (4K
// surface view: 147 us per launch, VALU pipe 45 % busy, LDS array 36 %, waves
// waiting 52 %; rocprofv3 profiles/r02s): ~20 VALU per tap. Here a thread owns
// two horizontally adjacent pixels and stages the footprint one channel per LDS
// plane (illum r g b var, normal x y z, linearZ), so a tap of the pair reads each
// channel of both texels with one 8-byte LDS read into a register pair, and the
// tap arithmetic runs on v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 for both
// pixels at once. Per pixel the operations (and their order) are those of
// atrous_taps, element by element, so the bits are the step kernel's
// (tests/test_gpu_atrous.py). Pairs that are not two interior surface pixels of
// positive phiIllumination (border tiles, background, FLAT, the frame's last
// column) run the same taps pixel by pixel.
// Tile: TJ = 8 rows of one residue class mod S x 128 columns; 8 waves, one tile
// row each, 64 lanes x 2 pixels.
constexpr int kPairCols = 128;
#ifdef PT_PAIR_WPE
#define PT_PAIR_ATTR __attribute__((amdgpu_waves_per_eu(PT_PAIR_WPE)))
#else
#define PT_PAIR_ATTR
#endif

template <int S, bool AUX>
__global__ void __launch_bounds__(512) PT_PAIR_ATTR atrous_pair_kernel(AtrousParams p) {
  constexpr int TJ = kTileRows, R = TJ + 4, C = kPairCols + 4 * S, PL = R * C, NT = 512;
  __shared__ float L[8 * PL];
  const int W = p.illum.W, row0 = p.illum.row0;
  const float4* __restrict__ I = p.illum.p;
  const float4* __restrict__ ND = p.nd.p;
  const int tid = threadIdx.x, lane = tid & 63;
  const int j = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = blockIdx.y / S, b = blockIdx.y - g * S;
  const int ybase = p.y0 + g * S * TJ + b;
  const int x0 = blockIdx.x * kPairCols, xl = 2 * lane, y = ybase + S * j;
  const int xa = x0 + xl;
  const bool rowok = y < p.y1;
  const bool ownA = rowok && xa < p.W, ownB = rowok && xa + 1 < p.W;
  const size_t ci = (size_t)(y - row0) * W + xa;
  bool bgA = true, bgB = true;
  float fwA = 0.0f, fwB = 0.0f;
  if (ownA) {
    if (AUX) {
      const float a = p.fwidth.aux[ci];
      bgA = aux_flag(a);
      fwA = fabsf(a);
    } else {
      bgA = ND[ci].w == 1.0f;
      fwA = p.fwidth.p[ci].y;
    }
  }
  if (ownB) {
    if (AUX) {
      const float a = p.fwidth.aux[ci + 1];
      bgB = aux_flag(a);
      fwB = fabsf(a);
    } else {
      bgB = ND[ci + 1].w == 1.0f;
      fwB = p.fwidth.p[ci + 1].y;
    }
  }
  __shared__ int any_surface[8];
  const bool wave_any = __ballot(!bgA || !bgB) != 0ull;
  if (lane == 0) any_surface[j] = wave_any;
  __syncthreads();
  bool tile_any = false;
#pragma unroll
  for (int w = 0; w < 8; ++w) tile_any |= any_surface[w] != 0;
  if (!tile_any) {
    if (ownA) p.out.p[ci] = I[ci];
    if (ownB) p.out.p[ci + 1] = I[ci + 1];
    return;
  }
  // stage two adjacent texels per item: tile row r <-> frame row ybase + S*(r-2), column c <-> x0 - 2S + c,
  // clamped into the frame and the stored band as the tiled kernel does
#if PT_ATROUS_BATCH
  constexpr int ITERS = (PL / 2 + NT - 1) / NT;
  const int lo = max(0, row0), hi = min(p.H, row0 + p.illum.rows) - 1;
  float4 i0[ITERS], i1[ITERS], n0[ITERS], n1[ITERS];
#pragma unroll
  for (int it = 0; it < ITERS; ++it) {
    const int e = tid + it * NT;
    if (e < PL / 2) {
      const int r = e / (C / 2), c = 2 * (e - r * (C / 2));
      int gy = ybase + S * (r - 2);
      gy = gy < lo ? lo : (gy > hi ? hi : gy);
      int gx0 = x0 - 2 * S + c, gx1 = gx0 + 1;
      gx0 = gx0 < 0 ? 0 : (gx0 >= p.W ? p.W - 1 : gx0);
      gx1 = gx1 < 0 ? 0 : (gx1 >= p.W ? p.W - 1 : gx1);
      const size_t rb = (size_t)(gy - row0) * W;
      i0[it] = I[rb + gx0];
      i1[it] = I[rb + gx1];
      n0[it] = ND[rb + gx0];
      n1[it] = ND[rb + gx1];
    }
  }
#pragma unroll
  for (int it = 0; it < ITERS; ++it) {
    const int e = tid + it * NT;
    if (e < PL / 2) {
      const int r = e / (C / 2), c = 2 * (e - r * (C / 2));
      f2v* q = (f2v*)(L + r * C + c);
      q[0 * PL / 2] = f2v{i0[it].x, i1[it].x};
      q[1 * PL / 2] = f2v{i0[it].y, i1[it].y};
      q[2 * PL / 2] = f2v{i0[it].z, i1[it].z};
      q[3 * PL / 2] = f2v{i0[it].w, i1[it].w};
      q[4 * PL / 2] = f2v{n0[it].x, n1[it].x};
      q[5 * PL / 2] = f2v{n0[it].y, n1[it].y};
      q[6 * PL / 2] = f2v{n0[it].z, n1[it].z};
      q[7 * PL / 2] = f2v{n0[it].w, n1[it].w};
    }
  }
#else
  const int lo = max(0, row0), hi = min(p.H, row0 + p.illum.rows) - 1;
  for (int e = tid; e < PL / 2; e += NT) {
    const int r = e / (C / 2), c = 2 * (e - r * (C / 2));
    int gy = ybase + S * (r - 2);
    gy = gy < lo ? lo : (gy > hi ? hi : gy);
    int gx0 = x0 - 2 * S + c, gx1 = gx0 + 1;
    gx0 = gx0 < 0 ? 0 : (gx0 >= p.W ? p.W - 1 : gx0);
    gx1 = gx1 < 0 ? 0 : (gx1 >= p.W ? p.W - 1 : gx1);
    const size_t rb = (size_t)(gy - row0) * W;
    const float4 i0 = I[rb + gx0], i1 = I[rb + gx1], n0 = ND[rb + gx0], n1 = ND[rb + gx1];
    f2v* q = (f2v*)(L + r * C + c);
    q[0 * PL / 2] = f2v{i0.x, i1.x};
    q[1 * PL / 2] = f2v{i0.y, i1.y};
    q[2 * PL / 2] = f2v{i0.z, i1.z};
    q[3 * PL / 2] = f2v{i0.w, i1.w};
    q[4 * PL / 2] = f2v{n0.x, n1.x};
    q[5 * PL / 2] = f2v{n0.y, n1.y};
    q[6 * PL / 2] = f2v{n0.z, n1.z};
    q[7 * PL / 2] = f2v{n0.w, n1.w};
  }
#endif
  __syncthreads();
  if (!ownA) return;
  const float* Lt = L + j * C + xl;  // top-left tap of pixel A's window; pixel B's is Lt + 1
  const bool edge =
      x0 - 2 * S < 0 || x0 + kPairCols - 1 + 2 * S >= p.W || ybase - 2 * S < 0 || ybase + S * (TJ + 1) >= p.H;
  const float LOG2E = 1.4426950408889634f;
  constexpr int CTR = 2 * C + 2 * S;  // centre tap offset
  auto ld = [&](const float* q, int ch) __attribute__((always_inline)) { return q[ch * PL]; };
  // one pixel, the tiled kernel's arithmetic (FLAT: phiIllumination == 0), reading the planar tile
  auto scalar = [&](int k, int x, bool bg, float fwz) __attribute__((always_inline)) {
    const float* Lp = Lt + k;
    const float4 ic = float4{ld(Lp + CTR, 0), ld(Lp + CTR, 1), ld(Lp + CTR, 2), ld(Lp + CTR, 3)};
    float4* out = p.out.p + ci + k;
    if (bg) {
      *out = ic;
      return;
    }
    const float4 nd = float4{ld(Lp + CTR, 4), ld(Lp + CTR, 5), ld(Lp + CTR, 6), ld(Lp + CTR, 7)};
    const float lc = (0.2125f * ic.x + 0.7154f * ic.y) + 0.0721f * ic.z;
    const float phiL = p.phi_color * __builtin_sqrtf(fmaxf(0.0f, 1e-10f + ic.w));
    const float kL = LOG2E / phiL;
    const float kD = LOG2E / (fmaxf(fwz, 1e-8f) * (float)S);
    const float kDr[5] = {kD, kD * 0.70710678f, kD * 0.5f, kD * 0.44721360f, kD * 0.35355339f};
    float sumW = 1.0f;
    f2v s01 = {ic.x, ic.y}, s23 = {ic.z, ic.w};
    auto taps = [&](auto flat_tag) __attribute__((always_inline)) {
      constexpr bool FLAT = decltype(flat_tag)::value;
      const float wLr = 0.2125f * kL, wLg = 0.7154f * kL, wLb = 0.0721f * kL, cL = -(lc * kL);
#pragma unroll
      for (int yy = -2; yy <= 2; ++yy) {
        if (edge && (y + yy * S < 0 || y + yy * S >= p.H)) continue;
#pragma unroll
        for (int xx = -2; xx <= 2; ++xx) {
          if (xx == 0 && yy == 0) continue;
          if (edge && (x + xx * S < 0 || x + xx * S >= p.W)) continue;
          const int r2 = xx * xx + yy * yy;
          const float kDl = r2 == 1 ? kDr[0] : r2 == 2 ? kDr[1] : r2 == 4 ? kDr[2] : r2 == 5 ? kDr[3] : kDr[4];
          const int ax = xx < 0 ? -xx : xx, ay = yy < 0 ? -yy : yy;
          const float kern = (ax == 0 ? 1.0f : ax == 1 ? 2.0f / 3.0f : 1.0f / 6.0f) *
                             (ay == 0 ? 1.0f : ay == 1 ? 2.0f / 3.0f : 1.0f / 6.0f);
          const float* q = Lp + (yy + 2) * C + (xx + 2) * S;
          const float4 ip = float4{ld(q, 0), ld(q, 1), ld(q, 2), ld(q, 3)};
          const float qx = ld(q, 4), qy = ld(q, 5), qz = ld(q, 6), qw = ld(q, 7);
          const float dn = fminf(fmaxf(__builtin_fmaf(nd.z, qz, __builtin_fmaf(nd.y, qy, nd.x * qx)), 0.0f), 1.0f);
          float a;
          if (FLAT) {
            const float lp = (0.2125f * ip.x + 0.7154f * ip.y) + 0.0721f * ip.z;
            a = lp == lc ? fabsf(nd.w - qw) * kDl : __builtin_inff();
          } else {
            const float tl = __builtin_fmaf(ip.z, wLb, __builtin_fmaf(ip.y, wLg, __builtin_fmaf(ip.x, wLr, cL)));
            a = __builtin_fmaf(fabsf(nd.w - qw), kDl, fabsf(tl));
          }
          const float w = __builtin_amdgcn_exp2f(__builtin_fmaf(p.phi_normal, __builtin_amdgcn_logf(dn), -a)) * kern;
          sumW += w;
          s01 = __builtin_elementwise_fma(f2v{w, w}, f2v{ip.x, ip.y}, s01);
          s23 = __builtin_elementwise_fma(f2v{w, w * w}, f2v{ip.z, ip.w}, s23);
        }
      }
    };
    if (__builtin_expect(phiL > 0.0f, 1)) taps(std::false_type{});
    else taps(std::true_type{});
    const float inv = 1.0f / sumW;
    *out = float4{s01.x * inv, s01.y * inv, s23.x * inv, s23.y * (inv * inv)};
  };
  // the pair on packed FP32, when both pixels take the interior non-FLAT path
  const f2v icR = *(const f2v*)(Lt + CTR), icG = *(const f2v*)(Lt + PL + CTR);
  const f2v icB = *(const f2v*)(Lt + 2 * PL + CTR), icV = *(const f2v*)(Lt + 3 * PL + CTR);
  const float phiLA = p.phi_color * __builtin_sqrtf(fmaxf(0.0f, 1e-10f + icV.x));
  const float phiLB = p.phi_color * __builtin_sqrtf(fmaxf(0.0f, 1e-10f + icV.y));
  if (edge || !ownB || bgA || bgB || !(phiLA > 0.0f) || !(phiLB > 0.0f)) {
#pragma nounroll
    for (int k = 0; k < (ownB ? 2 : 1); ++k) scalar(k, xa + k, k ? bgB : bgA, k ? fwB : fwA);
    return;
  }
  const f2v ndX = *(const f2v*)(Lt + 4 * PL + CTR), ndY = *(const f2v*)(Lt + 5 * PL + CTR);
  const f2v ndZ = *(const f2v*)(Lt + 6 * PL + CTR), ndW = *(const f2v*)(Lt + 7 * PL + CTR);
  const f2v lc = (0.2125f * icR + 0.7154f * icG) + 0.0721f * icB;
  const f2v kL = f2v{LOG2E / phiLA, LOG2E / phiLB};
  const f2v kD = f2v{LOG2E / (fmaxf(fwA, 1e-8f) * (float)S), LOG2E / (fmaxf(fwB, 1e-8f) * (float)S)};
  const f2v kDr[5] = {kD, kD * 0.70710678f, kD * 0.5f, kD * 0.44721360f, kD * 0.35355339f};
  const f2v wLr = 0.2125f * kL, wLg = 0.7154f * kL, wLb = 0.0721f * kL, cL = -(lc * kL);
  const f2v phiN = f2v{p.phi_normal, p.phi_normal};
  f2v sumW = f2v{1.0f, 1.0f}, sR = icR, sG = icG, sB = icB, sV = icV;
#pragma unroll
  for (int yy = -2; yy <= 2; ++yy) {
#pragma unroll
    for (int xx = -2; xx <= 2; ++xx) {
      if (xx == 0 && yy == 0) continue;
      const int r2 = xx * xx + yy * yy;
      const f2v kDl = r2 == 1 ? kDr[0] : r2 == 2 ? kDr[1] : r2 == 4 ? kDr[2] : r2 == 5 ? kDr[3] : kDr[4];
      const int ax = xx < 0 ? -xx : xx, ay = yy < 0 ? -yy : yy;
      const float kern = (ax == 0 ? 1.0f : ax == 1 ? 2.0f / 3.0f : 1.0f / 6.0f) *
                         (ay == 0 ? 1.0f : ay == 1 ? 2.0f / 3.0f : 1.0f / 6.0f);
      const float* q = Lt + (yy + 2) * C + (xx + 2) * S;
      f2v ch[8];
      if constexpr ((S & 1) != 0) {  // odd S: odd-column taps are 4-byte aligned (two dword reads)
#pragma unroll
        for (int k = 0; k < 8; ++k) ch[k] = f2v{q[k * PL], q[k * PL + 1]};
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) ch[k] = *(const f2v*)(q + k * PL);
      }
      f2v dn = __builtin_elementwise_fma(ndZ, ch[6], __builtin_elementwise_fma(ndY, ch[5], ndX * ch[4]));
      dn = __builtin_elementwise_min(__builtin_elementwise_max(dn, f2v{0.0f, 0.0f}), f2v{1.0f, 1.0f});
      const f2v tl = __builtin_elementwise_fma(
          ch[2], wLb, __builtin_elementwise_fma(ch[1], wLg, __builtin_elementwise_fma(ch[0], wLr, cL)));
      const f2v dz = ndW - ch[7];
      const f2v a = f2v{__builtin_fmaf(fabsf(dz.x), kDl.x, fabsf(tl.x)), __builtin_fmaf(fabsf(dz.y), kDl.y, fabsf(tl.y))};
      const f2v lg = f2v{__builtin_amdgcn_logf(dn.x), __builtin_amdgcn_logf(dn.y)};
      const f2v e = __builtin_elementwise_fma(phiN, lg, -a);
      const f2v w = f2v{__builtin_amdgcn_exp2f(e.x), __builtin_amdgcn_exp2f(e.y)} * kern;
      sumW += w;
      sR = __builtin_elementwise_fma(w, ch[0], sR);
      sG = __builtin_elementwise_fma(w, ch[1], sG);
      sB = __builtin_elementwise_fma(w, ch[2], sB);
      sV = __builtin_elementwise_fma(w * w, ch[3], sV);
    }
  }
  const f2v inv = f2v{1.0f / sumW.x, 1.0f / sumW.y};
  p.out.p[ci] = float4{sR.x * inv.x, sG.x * inv.x, sB.x * inv.x, sV.x * (inv.x * inv.x)};
  p.out.p[ci + 1] = float4{sR.y * inv.y, sG.y * inv.y, sB.y * inv.y, sV.y * (inv.y * inv.y)};
}

template <int S>
static void launch_pair_s(const AtrousParams& p, bool aux, hipStream_t s) {
  const int groups = (p.y1 - p.y0 + S * kTileRows - 1) / (S * kTileRows);
  dim3 grid((p.W + kPairCols - 1) / kPairCols, groups * S);
  if (aux) hipLaunchKernelGGL((atrous_pair_kernel<S, true>), grid, dim3(512), 0, s, p);
  else hipLaunchKernelGGL((atrous_pair_kernel<S, false>), grid, dim3(512), 0, s, p);
}

int launch_atrous_pair(const AtrousParams& p, hipStream_t s) {
  if (p.y1 <= p.y0) return 0;
  if (!same_geometry(p)) return launch_atrous_simple(p, s);
  const bool aux = p.fwidth.aux != nullptr;
  switch (p.step) {
    case 1: launch_pair_s<1>(p, aux, s); break;
    case 2: launch_pair_s<2>(p, aux, s); break;
    case 4: launch_pair_s<4>(p, aux, s); break;
    case 8: launch_pair_s<8>(p, aux, s); break;
    case 16: launch_pair_s<16>(p, aux, s); break;
    default: return launch_atrous_step(p, s);
  }
  return (int)hipGetLastError();
}


// ---------------------------------------------------------------------------------------------------------------
// Round 3: atrous_rows2_kernel (atrous_variant = 3), two tile rows per thread sharing their windows' LDS reads
// (30 texel reads for 48 taps). Bit-identical to the step kernel (tests/test_gpu_atrous.py at the time), but slower:
// 4K default view 74.4 vs 69.2 us, surface view 150.0 vs 144.5 us (79 VGPRs: 6 waves/SIMD against 8; the kernel is
// VALU/latency-bound there, not LDS-bound). Uses kernels_atrous.hip's TapPixel.
// Two pixels per thread (atrous_variant = 3): the thread owns tile rows 2k and 2k + 1 of one column, whose 5 x 5
// windows share 4 of their 5 rows, so each of the 6 x 5 staged texels under the pair is read from LDS once and
// applied to both pixels (30 texel reads for 48 taps instead of 48): 37.5 % fewer LDS reads, the same VALU work.
// Per pixel the taps are applied in the same order with the same arithmetic (TapPixel): bit-identical to the step
// kernel. Border tiles and FLAT pixels take the per-pixel windows of atrous_tile_kernel. Same tile geometry and
// staging as atrous_tile_kernel (half the threads), so the same per-tile surface flags.
template <int S, bool AUX>
__global__ void __launch_bounds__(32 * tile_tj<S>() * tile_nx<S>()) atrous_rows2_kernel(AtrousParams p) {
  constexpr int NX = tile_nx<S>();
  constexpr int TJ = tile_tj<S>(), NW = TJ / 2 * NX, R = TJ + 4, C = 64 * NX + 4 * S, NT = 64 * NW;
  static_assert(TJ % 2 == 0, "row pairs");
  __shared__ float4 LI[R * C];
  __shared__ float4 LN[R * C];
  const int W = p.illum.W, row0 = p.illum.row0;
  const float4* __restrict__ I = p.illum.p;
  const float4* __restrict__ ND = p.nd.p;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bx = blockIdx.x, g = blockIdx.y / S, b = blockIdx.y - g * S;
  const int ybase = p.y0 + g * S * TJ + b;
  const int jp = wv / NX, xl = (wv - jp * NX) * 64 + lane;
  const int j0 = 2 * jp;  // tile rows j0, j0 + 1
  const int x0 = bx * 64 * NX, x = x0 + xl, yA = ybase + S * j0, yB = yA + S;
  const bool ownA = x < p.W && yA < p.y1, ownB = x < p.W && yB < p.y1;
  const size_t ciA = (size_t)(yA - row0) * W + x, ciB = ciA + (size_t)S * W;
  bool bgA = true, bgB = true;
  float fwA = 0.0f, fwB = 0.0f;
  const bool pre = AUX && p.tile_any != nullptr;
  bool tile_any = true;
  if (pre) tile_any = p.tile_any[(g * S + b) * gridDim.x + bx] != 0;
  if (tile_any) {
    if (ownA) {
      if (AUX) {
        const float a = p.fwidth.aux[ciA];
        bgA = aux_flag(a);
        fwA = fabsf(a);
      } else {
        bgA = ND[ciA].w == 1.0f;
        fwA = p.fwidth.p[ciA].y;
      }
    }
    if (ownB) {
      if (AUX) {
        const float a = p.fwidth.aux[ciB];
        bgB = aux_flag(a);
        fwB = fabsf(a);
      } else {
        bgB = ND[ciB].w == 1.0f;
        fwB = p.fwidth.p[ciB].y;
      }
    }
  }
  if (!pre) {
    __shared__ int any_surface[NW];
    const bool wave_any = __ballot(!bgA || !bgB) != 0ull;
    if (lane == 0) any_surface[wv] = wave_any;
    __syncthreads();
    tile_any = false;
#pragma unroll
    for (int w = 0; w < NW; ++w) tile_any |= any_surface[w] != 0;
  }
  if (!tile_any) {
    if (ownA) p.out.p[ciA] = I[ciA];
    if (ownB) p.out.p[ciB] = I[ciB];
    return;
  }
  const int lo = max(0, row0), hi = min(p.H, row0 + p.illum.rows) - 1;
  for (int e = tid; e < R * C; e += NT) {
    const int r = e / C, c = e - r * C;
    int gy = ybase + S * (r - 2), gx = x0 - 2 * S + c;
    gy = gy < lo ? lo : (gy > hi ? hi : gy);
    gx = gx < 0 ? 0 : (gx >= p.W ? p.W - 1 : gx);
    const size_t gi = (size_t)(gy - row0) * W + gx;
    LI[e] = I[gi];
    LN[e] = ND[gi];
  }
  __syncthreads();
  if (!ownA) return;  // (ownB implies ownA)
  const float4* Li = LI + j0 * C + xl;  // top-left tap of pixel A's window; pixel B's is one row lower
  const float4* Ln = LN + j0 * C + xl;
  const float4 icA = Li[2 * C + 2 * S], icB = Li[3 * C + 2 * S];
  const bool cA = !bgA, cB = ownB && !bgB;  // pixels that compute taps
  if (!cA && !cB) {
    p.out.p[ciA] = icA;
    if (ownB) p.out.p[ciB] = icB;
    return;
  }
  const bool edge =
      x0 - 2 * S < 0 || x0 + 64 * NX - 1 + 2 * S >= p.W || ybase - 2 * S < 0 || ybase + S * (TJ + 1) >= p.H;
  TapPixel A, B;
  A.init(icA, Ln[2 * C + 2 * S], fwA, p.phi_color, S);
  B.init(icB, Ln[3 * C + 2 * S], fwB, p.phi_color, S);
  if (__builtin_expect(!edge && !(cA && A.flat) && !(cB && B.flat), 1)) {
    // the pair's 6 window rows: row r serves A as yy = r - 2 (r <= 4) and B as yy = r - 3 (r >= 1)
#pragma unroll
    for (int r = 0; r < 6; ++r) {
#pragma unroll
      for (int xx = -2; xx <= 2; ++xx) {
        const int o = r * C + (xx + 2) * S;
        const float4 ip = Li[o], q = Ln[o];
        if (r <= 4 && !(r == 2 && xx == 0)) A.tap<false>(ip, q, xx, r - 2, p.phi_normal);
        if (r >= 1 && !(r == 3 && xx == 0)) B.tap<false>(ip, q, xx, r - 3, p.phi_normal);
      }
    }
  } else {
    if (cA) {
      if (A.flat) A.window<true, true, S, C>(Li, Ln, x, yA, p.W, p.H, p.phi_normal);
      else A.window<false, true, S, C>(Li, Ln, x, yA, p.W, p.H, p.phi_normal);
    }
    if (cB) {
      if (B.flat) B.window<true, true, S, C>(Li + C, Ln + C, x, yB, p.W, p.H, p.phi_normal);
      else B.window<false, true, S, C>(Li + C, Ln + C, x, yB, p.W, p.H, p.phi_normal);
    }
  }
  p.out.p[ciA] = cA ? A.result() : icA;
  if (ownB) p.out.p[ciB] = cB ? B.result() : icB;
}

template <int S>
static void launch_rows2_s(const AtrousParams& p, bool aux, hipStream_t s) {
  constexpr int NX = tile_nx<S>(), TJ = tile_tj<S>();
  const int groups = (p.y1 - p.y0 + S * TJ - 1) / (S * TJ);
  dim3 grid((p.W + 64 * NX - 1) / (64 * NX), groups * S);
  if (aux) hipLaunchKernelGGL((atrous_rows2_kernel<S, true>), grid, dim3(32 * TJ * NX), 0, s, p);
  else hipLaunchKernelGGL((atrous_rows2_kernel<S, false>), grid, dim3(32 * TJ * NX), 0, s, p);
}

int launch_atrous_rows2(const AtrousParams& p, hipStream_t s) {
  if (p.y1 <= p.y0) return 0;
  if (!same_geometry(p)) return launch_atrous_simple(p, s);
  const bool aux = p.fwidth.aux != nullptr;
  switch (p.step) {
    case 1: launch_rows2_s<1>(p, aux, s); break;
    case 2: launch_rows2_s<2>(p, aux, s); break;
    case 4: launch_rows2_s<4>(p, aux, s); break;
    case 8: launch_rows2_s<8>(p, aux, s); break;
    case 16: launch_rows2_s<16>(p, aux, s); break;
    default: return launch_atrous_step(p, s);
  }
  return (int)hipGetLastError();
}


// kernels_bvh.hip — GPU LBVH builder for dynamic scenes.
//
// The reference builds its BVH once, on the host, with a recursive SAH sweep (buildBVHwithSAH, Utils/BVH.h:42-173,
// called at main.cpp:88-96 with leaf size 8) and uploads it as BVHNode_encoded texels (main.cpp:122-151). A scene
// whose triangles move every frame cannot afford that (a recursive sort per node). This builder produces the SAME
// buffer formats on the device — triangles in leaf order (Triangle_encoded, 15 RGB32F texels each) and
// BVHNode_encoded nodes with the dummy node 0 and the root at node 1 — so every consumer of the reference's buffers
// (the path tracer, the host decode in capi.hip, the CPU oracle) takes them unchanged. It is a different tree than
// the SAH builder's (no GPU builder can reproduce a host sort-and-sweep bit for bit); rendering over it is checked
// against the oracle walking the same buffers (tests/test_gpu_bvh.py).
//
// Algorithm: Karras, "Maximizing Parallelism in the Construction of BVHs, Octrees, and k-d Trees" (HPG 2012):
//   1. centroid c = (p1 + p2 + p3) / 3 (cmpx's centre, BVH.h:25-29) and the centroid bounds (wave max/min, one
//      ordered-int atomic per wave);
//   2. 30-bit Morton code of the centroid quantised to 1024 cells per axis, key = code << b | index (b bits of
//      index: keys are unique, so the radix tree is fully determined and the build deterministic);
//   3. rocPRIM radix sort of the keys (30 + b bits);
//   4. one thread per internal node finds its key range and split (the highest differing key bit);
//   5. bottom-up refit: each primitive walks towards the root; the second child to arrive (one acq_rel atomic per
//      node) computes the box as the union of its children — min/max are exact, so a node box equals the
//      reference's per-triangle min/max loop (BVH.h:52-67) over the same triangles;
//   6. nodes whose range holds <= leaf_n triangles become leaves (their subtrees are dropped); a scan over
//      "reachable" flags (internal nodes first, in Karras order, then single-triangle leaves) numbers the output
//      nodes from 1 (the root), and the emit kernel writes BVHNode_encoded texels and the triangles in key order.
// HBM traffic is a few passes over 16-64 B per triangle: for the 30.6 k-triangle bench scene the build is bound
// by launch latency and the sort's passes, not bytes.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cstdint>

#include "glsl_builtins.h"
#include "pt_device.h"

namespace ptk {

namespace {

constexpr int kTriFloats = 45;   // Triangle_encoded (Utils/Triangle.h:12-24)
constexpr int kNodeFloats = 12;  // BVHNode_encoded (Utils/BVH.h:18-22)

__device__ __forceinline__ unsigned ordered(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unordered(unsigned u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}
// glm::min / glm::max (a < b ? ... as the reference evaluates them)
__device__ __forceinline__ float gmin(float a, float b) { return b < a ? b : a; }
__device__ __forceinline__ float gmax(float a, float b) { return a < b ? b : a; }

// p1 at t[0..2], p2 at t[o2..], p3 at t[o3..] (Triangle_encoded: 3, 6; the raster vertex list: 6, 12)
__device__ __forceinline__ float3 centroid(const float* t, int o2, int o3) {
  return float3{((t[0] + t[o2]) + t[o3]) / 3.0f, ((t[1] + t[o2 + 1]) + t[o3 + 1]) / 3.0f,
                ((t[2] + t[o2 + 2]) + t[o3 + 2]) / 3.0f};
}

// 1. centroids and their bounds. bounds[0..2] = ordered min, bounds[3..5] = ordered max (pre-set by the host).
__global__ void __launch_bounds__(256) lbvh_centroids(const float* __restrict__ tri, int n, TriLayout lay,
                                                       float4* __restrict__ cen, unsigned* __restrict__ bounds) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  unsigned lo[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, hi[3] = {0u, 0u, 0u};
  if (i < n) {
    const float3 c = centroid(tri + (size_t)i * lay.stride, lay.o2, lay.o3);
    cen[i] = float4{c.x, c.y, c.z, 0.0f};
    const float cc[3] = {c.x, c.y, c.z};
#pragma unroll
    for (int a = 0; a < 3; ++a)  // NaN centroids (NaN vertices) stay out of the bounds
      if (cc[a] == cc[a]) lo[a] = hi[a] = ordered(cc[a]);
  }
#pragma unroll
  for (int a = 0; a < 3; ++a) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      lo[a] = min(lo[a], (unsigned)__shfl_xor((int)lo[a], o));
      hi[a] = max(hi[a], (unsigned)__shfl_xor((int)hi[a], o));
    }
  }
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      atomicMin(&bounds[a], lo[a]);
      atomicMax(&bounds[3 + a], hi[a]);
    }
  }
}

__device__ __forceinline__ uint64_t spread10(uint32_t v) {  // 10 bits -> every third bit of 30
  uint64_t x = v & 0x3ffu;
  x = (x | (x << 16)) & 0x030000FFull;
  x = (x | (x << 8)) & 0x0300F00Full;
  x = (x | (x << 4)) & 0x030C30C3ull;
  x = (x | (x << 2)) & 0x09249249ull;
  return x;
}

__device__ __forceinline__ uint32_t cell(float c, float lo, float hi) {
  const float ext = hi - lo;
  const float q = ext > 0.0f ? (c - lo) / ext : 0.0f;
  const float v = floorf(q * 1024.0f);
  return !(v == v) || v < 0.0f ? 0u : (v > 1023.0f ? 1023u : (uint32_t)v);  // NaN -> cell 0
}

// 2. keys: Morton code (x in the highest of each bit triple) above b index bits
__global__ void __launch_bounds__(256) lbvh_keys(const float4* __restrict__ cen, int n, const unsigned* bounds,
                                                  int ibits, uint64_t* __restrict__ keys) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float4 c = cen[i];
  const float lx = unordered(bounds[0]), ly = unordered(bounds[1]), lz = unordered(bounds[2]);
  const float hx = unordered(bounds[3]), hy = unordered(bounds[4]), hz = unordered(bounds[5]);
  const uint64_t m = (spread10(cell(c.x, lx, hx)) << 2) | (spread10(cell(c.y, ly, hy)) << 1) |
                     spread10(cell(c.z, lz, hz));
  keys[i] = (m << ibits) | (uint64_t)i;
}

__device__ __forceinline__ int delta(const uint64_t* __restrict__ k, int n, int i, int j) {
  if (j < 0 || j >= n) return -1;
  return __clzll(k[i] ^ k[j]);
}

// 4. internal node i of n-1: its range [first, last] and children. child refs: >= 0 internal node, < 0 primitive
// (~sorted position). parent[] indexes internal nodes 0..n-2, then primitives at n-1+p.
__global__ void __launch_bounds__(256) lbvh_karras(const uint64_t* __restrict__ k, int n, int2* __restrict__ child,
                                                    int2* __restrict__ range, int* __restrict__ parent) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n - 1) return;
  const int d = delta(k, n, i, i + 1) - delta(k, n, i, i - 1) >= 0 ? 1 : -1;
  const int dmin = delta(k, n, i, i - d);
  int lmax = 2;
  while (delta(k, n, i, i + lmax * d) > dmin) lmax <<= 1;
  int l = 0;
  for (int t = lmax >> 1; t >= 1; t >>= 1)
    if (delta(k, n, i, i + (l + t) * d) > dmin) l += t;
  const int j = i + l * d;
  const int dnode = delta(k, n, i, j);
  int s = 0;
  for (int div = 2;; div <<= 1) {
    const int t = (l + div - 1) / div;
    if (delta(k, n, i, i + (s + t) * d) > dnode) s += t;
    if (t == 1) break;
  }
  const int gamma = i + s * d + min(d, 0);
  const int first = min(i, j), last = max(i, j);
  const int left = first == gamma ? ~gamma : gamma;
  const int right = last == gamma + 1 ? ~(gamma + 1) : gamma + 1;
  child[i] = int2{left, right};
  range[i] = int2{first, last};
  parent[left >= 0 ? left : n - 1 + ~left] = i;
  parent[right >= 0 ? right : n - 1 + ~right] = i;
  if (i == 0) parent[0] = -1;
}

// 5. bottom-up boxes. box[e] (e: internal 0..n-2, primitive n-1+p) = lo.xyz, hi.xyz as 2 float4.
__global__ void __launch_bounds__(256) lbvh_refit(const float* __restrict__ tri, TriLayout lay,
                                                   const uint64_t* __restrict__ k, int n, int ibits,
                                                   const int2* __restrict__ child, const int* __restrict__ parent,
                                                   float4* box, int* flags, int* __restrict__ order) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= n) return;
  const uint64_t mask = (ibits >= 64) ? ~0ull : ((1ull << ibits) - 1ull);
  const int orig = (int)(k[p] & mask);
  if (order) order[p] = orig;
  const float* t = tri + (size_t)orig * lay.stride;
  float lo[3], hi[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {  // BVH.h:54-66: min(p1, min(p2, p3)) per axis
    lo[a] = gmin(t[a], gmin(t[lay.o2 + a], t[lay.o3 + a]));
    hi[a] = gmax(t[a], gmax(t[lay.o2 + a], t[lay.o3 + a]));
  }
  int e = n - 1 + p;
  box[2 * e] = float4{lo[0], lo[1], lo[2], 0.0f};
  box[2 * e + 1] = float4{hi[0], hi[1], hi[2], 0.0f};
  int node = parent[e];
  while (node >= 0) {
    // the first child to arrive stops; the second sees both boxes (acq_rel orders the box stores and loads)
    if (__hip_atomic_fetch_add(&flags[node], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
    const int2 c = child[node];
    const int a = c.x >= 0 ? c.x : n - 1 + ~c.x, b = c.y >= 0 ? c.y : n - 1 + ~c.y;
    const float4 al = box[2 * a], ah = box[2 * a + 1], bl = box[2 * b], bh = box[2 * b + 1];
    box[2 * node] = float4{gmin(al.x, bl.x), gmin(al.y, bl.y), gmin(al.z, bl.z), 0.0f};
    box[2 * node + 1] = float4{gmax(ah.x, bh.x), gmax(ah.y, bh.y), gmax(ah.z, bh.z), 0.0f};
    node = parent[node];
  }
}

// 6a. reachable output nodes: internal node i unless its parent's range fits a leaf; primitive p only when its
// parent is an interior output node (a range > leaf_n). n == 1: the single primitive is the root leaf.
__global__ void __launch_bounds__(256) lbvh_mark(int n, int leaf_n, const int2* __restrict__ range,
                                                  const int* __restrict__ parent, int* __restrict__ keep) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= 2 * n - 1) return;
  const int par = parent[e];
  int k;
  if (par < 0) k = 1;  // the root (internal 0, or the lone primitive when n == 1)
  else {
    const int2 r = range[par];
    k = r.y - r.x + 1 > leaf_n;
  }
  keep[e] = k;
}

// 6b. BVHNode_encoded texels (childs, leafInfo, AA, BB) and the dummy node 0 (main.cpp:88-94).
__global__ void __launch_bounds__(256) lbvh_emit(int n, int leaf_n, const int2* __restrict__ child,
                                                  const int2* __restrict__ range, const int* __restrict__ keep,
                                                  const int* __restrict__ id, const float4* __restrict__ box,
                                                  float* __restrict__ out) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e == 0) {
    const float dummy[kNodeFloats] = {255, 128, 0, 30, 0, 0, 1, 1, 0, 0, 1, 0};
    for (int q = 0; q < kNodeFloats; ++q) out[q] = dummy[q];
  }
  if (e >= 2 * n - 1 || !keep[e]) return;
  float* o = out + (size_t)(1 + id[e]) * kNodeFloats;
  int first, count;
  bool leaf;
  if (e < n - 1) {
    const int2 r = range[e];
    first = r.x;
    count = r.y - r.x + 1;
    leaf = count <= leaf_n;
  } else {
    first = e - (n - 1);
    count = 1;
    leaf = true;
  }
  if (leaf) {
    o[0] = 0.0f; o[1] = 0.0f; o[2] = 0.0f;
    o[3] = (float)count; o[4] = (float)first; o[5] = 0.0f;
  } else {
    const int2 c = child[e];
    const int a = c.x >= 0 ? c.x : n - 1 + ~c.x, b = c.y >= 0 ? c.y : n - 1 + ~c.y;
    o[0] = (float)(1 + id[a]); o[1] = (float)(1 + id[b]); o[2] = 0.0f;
    o[3] = 0.0f; o[4] = 0.0f; o[5] = 0.0f;
  }
  const float4 lo = box[2 * e], hi = box[2 * e + 1];
  o[6] = lo.x; o[7] = lo.y; o[8] = lo.z;
  o[9] = hi.x; o[10] = hi.y; o[11] = hi.z;
}

// 6c. triangles in key (leaf) order
__global__ void __launch_bounds__(256) lbvh_reorder(const float* __restrict__ tri, const uint64_t* __restrict__ k,
                                                     int n, int ibits, float* __restrict__ out) {
  const size_t f = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (f >= (size_t)n * kTriFloats) return;
  const int p = (int)(f / kTriFloats), q = (int)(f - (size_t)p * kTriFloats);
  const uint64_t mask = (1ull << ibits) - 1ull;
  out[f] = tri[(size_t)(k[p] & mask) * kTriFloats + q];
}

// Triangle_encoded texels -> the path tracer's tri_geom / tri_shade records (capi.hip get_scene's host decode,
// same built-ins, so the same bits): the device decode of GPU-built scenes, whose triangles never leave the device.
__global__ void __launch_bounds__(256) decode_tris_kernel(const float* __restrict__ te, int n, float4* __restrict__ geom,
                                                           float4* __restrict__ shade) {
  using namespace glsl;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float* f = te + (size_t)i * kTriFloats;
  const v3 p1 = mk(f[0], f[1], f[2]), p2 = mk(f[3], f[4], f[5]), p3 = mk(f[6], f[7], f[8]);
  const v3 N = normalize(cross(sub(p2, p1), sub(p3, p1)));  // hitTriangle (path_tracing.frag:227)
  geom[4 * i + 0] = float4{p1.x, p1.y, p1.z, dot(N, p1)};
  geom[4 * i + 1] = float4{p2.x, p2.y, p2.z, 0.0f};
  geom[4 * i + 2] = float4{p3.x, p3.y, p3.z, 0.0f};
  geom[4 * i + 3] = float4{N.x, N.y, N.z, 0.0f};
  float4* s = shade + 9 * (size_t)i;
  s[0] = float4{f[9], f[10], f[11], f[12]};
  s[1] = float4{f[13], f[14], f[15], f[16]};
  s[2] = float4{f[17], f[18], f[19], f[20]};
  s[3] = float4{f[21], f[22], f[23], f[24]};
  s[4] = float4{f[25], f[26], f[27], f[28]};
  s[5] = float4{f[29], f[30], f[31], f[32]};
  s[6] = float4{f[33], f[34], f[35], f[42]};
  s[7] = float4{f[36], f[37], f[38], f[39]};
  s[8] = float4{f[40], f[41], 0.0f, 0.0f};
}


// ---------------------------------------------------------------------------------------------------------------
// PLOC top (quality > 0): the LBVH's leaves (ranges of <= leaf_n Morton-ordered triangles, their boxes exact) are
// kept, and the tree above them is rebuilt by Parallel Locally-Ordered Clustering (Meister & Bittner, 2018): every
// cluster in Morton order finds, within r positions, the neighbour whose merged box has the smallest surface area
// (ties: the nearer-indexed pair, a total order on pairs, so the globally best pair is always mutual and every
// iteration merges at least once); mutual pairs merge into a new node at the lower position, the array is
// compacted, until one cluster is left. Clusters: >= 0 PLOC node (creation order), < 0 leaf ~L (Morton rank).
__device__ __forceinline__ float half_area(float4 lo, float4 hi) {
  const float dx = hi.x - lo.x, dy = hi.y - lo.y, dz = hi.z - lo.z;
  return (dx * dy + dy * dz) + dz * dx;
}

// leaves in Morton order: start[first] = 1 for every reachable LBVH leaf
__global__ void __launch_bounds__(256) ploc_leafstart(int n, int leaf_n, const int2* __restrict__ range,
                                                       const int* __restrict__ keep, int* __restrict__ start) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= 2 * n - 1 || !keep[e]) return;
  if (e < n - 1) {
    const int2 r = range[e];
    if (r.y - r.x + 1 <= leaf_n) start[r.x] = 1;
  } else {
    start[e - (n - 1)] = 1;
  }
}

__global__ void __launch_bounds__(256) ploc_init(int n, int leaf_n, const int2* __restrict__ range,
                                                  const int* __restrict__ keep, const int* __restrict__ rank,
                                                  const int* __restrict__ start, const float4* __restrict__ box,
                                                  int2* __restrict__ leaf, float4* __restrict__ leafbox,
                                                  int* __restrict__ C, float4* __restrict__ cbox, int* __restrict__ cnt) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e == 0) {
    cnt[0] = rank[n - 1] + start[n - 1];  // clusters (= leaves, M)
    cnt[1] = 0;                           // PLOC nodes created
    cnt[4] = cnt[0];
  }
  if (e >= 2 * n - 1 || !keep[e]) return;
  int first, count;
  if (e < n - 1) {
    const int2 r = range[e];
    count = r.y - r.x + 1;
    if (count > leaf_n) return;
    first = r.x;
  } else {
    first = e - (n - 1);
    count = 1;
  }
  const int L = rank[first];
  leaf[L] = int2{first, count};
  C[L] = ~L;
  cbox[2 * L] = leafbox[2 * L] = box[2 * e];
  cbox[2 * L + 1] = leafbox[2 * L + 1] = box[2 * e + 1];
}

__global__ void __launch_bounds__(256) ploc_nn(const int* __restrict__ cnt, const float4* __restrict__ cbox, int r,
                                                int* __restrict__ nn) {
  const int n = cnt[0];
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float4 lo = cbox[2 * i], hi = cbox[2 * i + 1];
  float best = __builtin_inff();
  int bj = -1, bs = 1;
  const int j0 = max(0, i - r), j1 = min(n - 1, i + r);
  // Pairs are ranked by (area, j != (i ^ 1), min(i, j), max(i, j)): a total order on pairs, so the globally best pair
  // is mutual and every iteration merges; on runs of equal areas (coincident points, NaN boxes) the sibling pairs
  // (2k, 2k + 1) rank first and are all mutual, so such a run halves per iteration instead of losing one cluster.
  for (int j = j0; j <= j1; ++j) {  // ascending j: for equal (area, sibling flag) the smaller pair comes first
    if (j == i) continue;
    // the union in position order (lower position first), as ploc_compact merges: with NaN coordinates glm's
    // min/max depend on the operand order, and the area must be the same seen from either end of the pair
    const float4 l2 = cbox[2 * j], h2 = cbox[2 * j + 1];
    const float4 la = j < i ? l2 : lo, lb = j < i ? lo : l2, ha = j < i ? h2 : hi, hb = j < i ? hi : h2;
    float a = half_area(float4{gmin(la.x, lb.x), gmin(la.y, lb.y), gmin(la.z, lb.z), 0.0f},
                        float4{gmax(ha.x, hb.x), gmax(ha.y, hb.y), gmax(ha.z, hb.z), 0.0f});
    a = a == a ? a : __builtin_inff();  // NaN boxes rank last: the pair order stays total, so PLOC ends
    const int sj = j != (i ^ 1);
    if (bj < 0 || a < best || (a == best && sj < bs)) {
      best = a;
      bj = j;
      bs = sj;
    }
  }
  nn[i] = bj < 0 ? i : bj;
}

// f[i] = (merges here << 32) | survives, for i < N (zero past the live clusters)
__global__ void __launch_bounds__(256) ploc_flags(const int* __restrict__ cnt, const int* __restrict__ nn, int N,
                                                   uint64_t* __restrict__ f) {
  const int n = cnt[0];
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= N) return;
  if (i >= n) {
    f[i] = 0;
    return;
  }
  const int j = nn[i];
  const bool mutual = j != i && nn[j] == i;
  f[i] = ((uint64_t)(mutual && i < j) << 32) | (uint64_t)!(mutual && i > j);
}

__global__ void __launch_bounds__(256) ploc_compact(const int* __restrict__ cin, int* __restrict__ cout,
                                                     const int* __restrict__ C, const float4* __restrict__ cbox,
                                                     const int* __restrict__ nn, const uint64_t* __restrict__ f,
                                                     const uint64_t* __restrict__ pf, int* __restrict__ C2,
                                                     float4* __restrict__ cbox2, int2* __restrict__ nchild,
                                                     float4* __restrict__ nbox) {
  const int n = cin[0], created = cin[1];
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint64_t fi = f[i], pi = pf[i];
  if (i == n - 1) {
    const uint64_t tot = pi + fi;
    cout[0] = (int)(tot & 0xffffffffu);
    cout[1] = created + (int)(tot >> 32);
  }
  if (!(fi & 1u)) return;
  const int p = (int)(pi & 0xffffffffu);
  if (fi >> 32) {
    const int j = nn[i], k = created + (int)(pi >> 32);
    const float4 al = cbox[2 * i], ah = cbox[2 * i + 1], bl = cbox[2 * j], bh = cbox[2 * j + 1];
    const float4 lo = float4{gmin(al.x, bl.x), gmin(al.y, bl.y), gmin(al.z, bl.z), 0.0f};
    const float4 hi = float4{gmax(ah.x, bh.x), gmax(ah.y, bh.y), gmax(ah.z, bh.z), 0.0f};
    nchild[k] = int2{C[i], C[j]};
    nbox[2 * k] = lo;
    nbox[2 * k + 1] = hi;
    C2[p] = k;
    cbox2[2 * p] = lo;
    cbox2[2 * p + 1] = hi;
  } else {
    C2[p] = C[i];
    cbox2[2 * p] = cbox[2 * i];
    cbox2[2 * p + 1] = cbox[2 * i + 1];
  }
}

// BVHNode_encoded: PLOC node k -> node 1 + (M - 2 - k) (the root, created last, is node 1); leaf L -> node M + L
__global__ void __launch_bounds__(256) ploc_emit(const int* __restrict__ cnt, int N, const int2* __restrict__ nchild,
                                                  const float4* __restrict__ nbox, const int2* __restrict__ leaf,
                                                  const float4* __restrict__ cbox_leaf, float* __restrict__ out) {
  const int M = cnt[4];
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e == 0) {
    const float dummy[kNodeFloats] = {255, 128, 0, 30, 0, 0, 1, 1, 0, 0, 1, 0};
    for (int q = 0; q < kNodeFloats; ++q) out[q] = dummy[q];
  }
  auto id = [&](int ref) { return ref >= 0 ? 1 + (M - 2 - ref) : M + ~ref; };
  if (e < M - 1) {
    float* o = out + (size_t)id(e) * kNodeFloats;
    const int2 c = nchild[e];
    const float4 lo = nbox[2 * e], hi = nbox[2 * e + 1];
    o[0] = (float)id(c.x); o[1] = (float)id(c.y); o[2] = 0.0f;
    o[3] = 0.0f; o[4] = 0.0f; o[5] = 0.0f;
    o[6] = lo.x; o[7] = lo.y; o[8] = lo.z;
    o[9] = hi.x; o[10] = hi.y; o[11] = hi.z;
  }
  if (e < M) {
    float* o = out + (size_t)(M + e) * kNodeFloats;
    const int2 l = leaf[e];
    const float4 lo = cbox_leaf[2 * e], hi = cbox_leaf[2 * e + 1];
    o[0] = 0.0f; o[1] = 0.0f; o[2] = 0.0f;
    o[3] = (float)l.y; o[4] = (float)l.x; o[5] = 0.0f;
    o[6] = lo.x; o[7] = lo.y; o[8] = lo.z;
    o[9] = hi.x; o[10] = hi.y; o[11] = hi.z;
  }
}

// Raster vertex list (pos3 + nrm3 per vertex, obj_loader.h:143-160) -> the G-buffer's records in leaf order, as
// pt_raster_pass_bind writes them on the host: (p1, original index bits), e1, e2, cross(e1, e2); the three normals.
__global__ void __launch_bounds__(256) decode_raster_kernel(const float* __restrict__ verts,
                                                             const int* __restrict__ order, int n,
                                                             float4* __restrict__ geom, float4* __restrict__ nrm) {
  using namespace glsl;
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= n) return;
  const int oi = order[k];
  const float* f = verts + (size_t)oi * 18;
  const v3 p1 = mk(f[0], f[1], f[2]), p2 = mk(f[6], f[7], f[8]), p3 = mk(f[12], f[13], f[14]);
  const v3 e1 = sub(p2, p1), e2 = sub(p3, p1), ng = cross(e1, e2);
  geom[4 * k + 0] = float4{p1.x, p1.y, p1.z, __int_as_float(oi)};
  geom[4 * k + 1] = float4{e1.x, e1.y, e1.z, 0.0f};
  geom[4 * k + 2] = float4{e2.x, e2.y, e2.z, 0.0f};
  geom[4 * k + 3] = float4{ng.x, ng.y, ng.z, 0.0f};
  nrm[3 * k + 0] = float4{f[3], f[4], f[5], 0.0f};
  nrm[3 * k + 1] = float4{f[9], f[10], f[11], 0.0f};
  nrm[3 * k + 2] = float4{f[15], f[16], f[17], 0.0f};
}

}  // namespace

int decode_raster(const float* verts, const int* order, int n, float4* geom, float4* nrm, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(decode_raster_kernel, dim3((n + 255) / 256), dim3(256), 0, s, verts, order, n, geom, nrm);
  return (int)hipGetLastError();
}

int decode_tris(const float* te, int n, float4* geom, float4* shade, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(decode_tris_kernel, dim3((n + 255) / 256), dim3(256), 0, s, te, n, geom, shade);
  return (int)hipGetLastError();
}

size_t LbvhWork::need(int n) {
  size_t b = 0;
  auto add = [&](size_t bytes) { b += (bytes + 255) & ~(size_t)255; };
  add(2 * sizeof(uint64_t) * n);            // keys in / out
  add(sizeof(float4) * n);                  // centroids
  add(sizeof(int2) * n);                    // child
  add(sizeof(int2) * n);                    // range
  add(sizeof(int) * 2 * n);                 // parent
  add(sizeof(float4) * 2 * 2 * n);          // boxes
  add(sizeof(int) * n);                     // flags
  add(sizeof(int) * 2 * n * 2);             // keep, id
  add(64);                                  // bounds + count
  // PLOC top: start, rank, nn, cluster ids x2 | leaf ranges | cluster boxes x2, leaf boxes, node boxes | flags,
  // scanned flags | node children | counters
  add(sizeof(int) * n * 5);
  add(sizeof(int2) * n);
  add(sizeof(float4) * 2 * n * 4);
  add(sizeof(uint64_t) * n * 2);
  add(sizeof(int2) * n);
  add(64);
  return b;
}

int lbvh_build(LbvhWork& w, const float* tri, TriLayout lay, int n, int leaf_n, int ploc_r, float* tri_out,
               float* node_out, int* order, int* nnodes, hipStream_t s) {
  if (n < 1) return (int)hipErrorInvalidValue;
  int ibits = 1;
  while ((1ll << ibits) < n) ++ibits;
  const size_t need = LbvhWork::need(n);
  // rocPRIM scratch: sort of 30 + ibits key bits, scan of 2n - 1 flags
  size_t sort_bytes = 0, scan_bytes = 0;
  hipError_t e = rocprim::radix_sort_keys(nullptr, sort_bytes, (uint64_t*)nullptr, (uint64_t*)nullptr, (size_t)n, 0,
                                          30 + ibits, s);
  if (e != hipSuccess) return (int)e;
  e = rocprim::exclusive_scan(nullptr, scan_bytes, (int*)nullptr, (int*)nullptr, 0, (size_t)(2 * n - 1),
                              rocprim::plus<int>(), s);
  if (e != hipSuccess) return (int)e;
  size_t scan64_bytes = 0;
  e = rocprim::exclusive_scan(nullptr, scan64_bytes, (uint64_t*)nullptr, (uint64_t*)nullptr, (uint64_t)0, (size_t)n,
                              rocprim::plus<uint64_t>(), s);
  if (e != hipSuccess) return (int)e;
  const size_t temp = std::max(sort_bytes, std::max(scan_bytes, scan64_bytes));
  if (w.bytes < need + temp) {
    if (w.base) (void)hipFree(w.base);
    w.base = nullptr;
    w.bytes = 0;
    if ((e = hipMalloc(&w.base, need + temp)) != hipSuccess) return (int)e;
    w.bytes = need + temp;
  }
  char* p = (char*)w.base;
  auto take = [&](size_t bytes) { char* q = p; p += (bytes + 255) & ~(size_t)255; return (void*)q; };
  uint64_t* kin = (uint64_t*)take(sizeof(uint64_t) * n);
  uint64_t* kout = (uint64_t*)take(sizeof(uint64_t) * n);
  float4* cen = (float4*)take(sizeof(float4) * n);
  int2* child = (int2*)take(sizeof(int2) * n);
  int2* range = (int2*)take(sizeof(int2) * n);
  int* parent = (int*)take(sizeof(int) * 2 * n);
  float4* box = (float4*)take(sizeof(float4) * 2 * 2 * n);
  int* flags = (int*)take(sizeof(int) * n);
  int* keep = (int*)take(sizeof(int) * 2 * n);
  int* id = (int*)take(sizeof(int) * 2 * n);
  unsigned* bounds = (unsigned*)take(64);
  int* start = (int*)take(sizeof(int) * n * 5);
  int *rank = start + n, *nn = start + 2 * n, *C0 = start + 3 * n, *C1 = start + 4 * n;
  int2* leaf = (int2*)take(sizeof(int2) * n);
  float4* cb0 = (float4*)take(sizeof(float4) * 2 * n * 4);
  float4 *cb1 = cb0 + 2 * n, *leafbox = cb0 + 4 * n, *nbox = cb0 + 6 * n;
  uint64_t* f = (uint64_t*)take(sizeof(uint64_t) * n * 2);
  uint64_t* pf = f + n;
  int2* nchild = (int2*)take(sizeof(int2) * n);
  int* cnt = (int*)take(64);
  void* scratch = (void*)(p);
  // bounds: ordered min words start at 0xffffffff, max words at 0 (no host buffer involved)
  if ((e = hipMemsetAsync(bounds, 0xff, 3 * sizeof(unsigned), s)) != hipSuccess) return (int)e;
  if ((e = hipMemsetAsync(bounds + 3, 0, 3 * sizeof(unsigned), s)) != hipSuccess) return (int)e;
  if ((e = hipMemsetAsync(flags, 0, sizeof(int) * n, s)) != hipSuccess) return (int)e;
  const int gb = (n + 255) / 256, ge = (2 * n - 1 + 255) / 256;
  hipLaunchKernelGGL(lbvh_centroids, dim3(gb), dim3(256), 0, s, tri, n, lay, cen, bounds);
  hipLaunchKernelGGL(lbvh_keys, dim3(gb), dim3(256), 0, s, cen, n, bounds, ibits, kin);
  size_t sb = sort_bytes;
  if ((e = rocprim::radix_sort_keys(scratch, sb, kin, kout, (size_t)n, 0, 30 + ibits, s)) != hipSuccess) return (int)e;
  if (n > 1) hipLaunchKernelGGL(lbvh_karras, dim3((n - 1 + 255) / 256), dim3(256), 0, s, kout, n, child, range, parent);
  else if ((e = hipMemsetAsync(parent, 0xff, sizeof(int), s)) != hipSuccess) return (int)e;
  hipLaunchKernelGGL(lbvh_refit, dim3(gb), dim3(256), 0, s, tri, lay, kout, n, ibits, child, parent, box, flags, order);
  hipLaunchKernelGGL(lbvh_mark, dim3(ge), dim3(256), 0, s, n, leaf_n, range, parent, keep);
  size_t cb = scan_bytes;
  if ((e = rocprim::exclusive_scan(scratch, cb, keep, id, 0, (size_t)(2 * n - 1), rocprim::plus<int>(), s)) !=
      hipSuccess)
    return (int)e;
  if (ploc_r <= 0 || n == 1) {
    hipLaunchKernelGGL(lbvh_emit, dim3(ge), dim3(256), 0, s, n, leaf_n, child, range, keep, id, box, node_out);
  } else {
    if ((e = hipMemsetAsync(start, 0, sizeof(int) * n, s)) != hipSuccess) return (int)e;
    hipLaunchKernelGGL(ploc_leafstart, dim3(ge), dim3(256), 0, s, n, leaf_n, range, keep, start);
    size_t rb = scan_bytes;
    if ((e = rocprim::exclusive_scan(scratch, rb, start, rank, 0, (size_t)n, rocprim::plus<int>(), s)) != hipSuccess)
      return (int)e;
    hipLaunchKernelGGL(ploc_init, dim3(ge), dim3(256), 0, s, n, leaf_n, range, keep, rank, start, box, leaf, leafbox, C0,
                       cb0, cnt);
    // iterations in batches; a converged array (one cluster) makes further iterations no-ops
    int host_cnt[5] = {0, 0, 0, 0, 0};
    bool converged = false;
    for (int it = 0; it < 4096 && !converged;) {
      for (int b = 0; b < 8; ++b, ++it) {
        int* cin = cnt + 2 * (it & 1);
        int* cout = cnt + 2 * ((it + 1) & 1);
        int* Ci = (it & 1) ? C1 : C0;
        int* Co = (it & 1) ? C0 : C1;
        float4* bi = (it & 1) ? cb1 : cb0;
        float4* bo = (it & 1) ? cb0 : cb1;
        hipLaunchKernelGGL(ploc_nn, dim3(gb), dim3(256), 0, s, cin, bi, ploc_r, nn);
        hipLaunchKernelGGL(ploc_flags, dim3(gb), dim3(256), 0, s, cin, nn, n, f);
        size_t fb = scan64_bytes;
        if ((e = rocprim::exclusive_scan(scratch, fb, f, pf, (uint64_t)0, (size_t)n, rocprim::plus<uint64_t>(), s)) !=
            hipSuccess)
          return (int)e;
        hipLaunchKernelGGL(ploc_compact, dim3(gb), dim3(256), 0, s, cin, cout, Ci, bi, nn, f, pf, Co, bo, nchild, nbox);
      }
      if ((e = hipMemcpyAsync(host_cnt, cnt, sizeof(host_cnt), hipMemcpyDeviceToHost, s)) != hipSuccess) return (int)e;
      if ((e = hipStreamSynchronize(s)) != hipSuccess) return (int)e;
      converged = host_cnt[2 * (it & 1)] <= 1;
    }
    if (converged) {
      hipLaunchKernelGGL(ploc_emit, dim3(gb), dim3(256), 0, s, cnt, n, nchild, nbox, leaf, leafbox, node_out);
      if (tri_out)
        hipLaunchKernelGGL(lbvh_reorder, dim3((unsigned)(((size_t)n * kTriFloats + 255) / 256)), dim3(256), 0, s, tri,
                           kout, n, ibits, tri_out);
      if ((e = hipStreamSynchronize(s)) != hipSuccess) return (int)e;
      *nnodes = 2 * host_cnt[4];  // dummy + (M - 1) PLOC nodes + M leaves
      return (int)hipGetLastError();
    }
    // past the iteration cap (every iteration merges at least one pair, and runs of equal areas halve, so only a
    // pathological input gets here): the plain LBVH top over the same leaves, whose buffers PLOC left untouched
    hipLaunchKernelGGL(lbvh_emit, dim3(ge), dim3(256), 0, s, n, leaf_n, child, range, keep, id, box, node_out);
  }
  if (tri_out)
    hipLaunchKernelGGL(lbvh_reorder, dim3((unsigned)(((size_t)n * kTriFloats + 255) / 256)), dim3(256), 0, s, tri,
                       kout, n, ibits, tri_out);
  // output node count = 1 (dummy) + id[last] + keep[last]
  int tail[2];
  if ((e = hipMemcpyAsync(&tail[0], id + 2 * n - 2, sizeof(int), hipMemcpyDeviceToHost, s)) != hipSuccess) return (int)e;
  if ((e = hipMemcpyAsync(&tail[1], keep + 2 * n - 2, sizeof(int), hipMemcpyDeviceToHost, s)) != hipSuccess)
    return (int)e;
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return (int)e;
  *nnodes = 1 + tail[0] + tail[1];
  return (int)hipGetLastError();
}

}  // namespace ptk

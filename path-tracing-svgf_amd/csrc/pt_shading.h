// pt_shading.h — device-side restatement of shaders/path_tracing.frag shared by
// the megakernel (kernels_pt.hip) and the wavefront kernels (kernels_wavefront.hip):
// scene decode, hitAABB/hitTriangle, BVH traversal (closest / any-hit), the
// Disney BRDF, its pdf and sampling, and the HDR environment lookups.
// Header-only, included by .hip translation units built with -ffp-contract=off.
#pragma once
#include <hip/hip_runtime.h>

#include "glsl_builtins.h"
#include "pt_device.h"

namespace ptk {
using namespace glsl;


#define PT_PI 3.1415926f
#define PT_INF 114514.0f

__device__ __forceinline__ int prow(const Plane& P, int y) {
  int ly = y - P.row0;
  return ly < 0 ? 0 : (ly >= P.rows ? P.rows - 1 : ly);
}
__device__ __forceinline__ float4 pld(const Plane& P, int x, int y) { return P.p[(size_t)prow(P, y) * P.W + x]; }
// Streaming (non-temporal) access to per-pixel state and output planes: each element is touched once per
// launch, so it should not evict the scene (BVH nodes, triangles: ~7 MB) from the 4 MB per-XCD L2 that every
// traversal step reads. Values are unchanged; only the cache policy differs.
#ifndef PT_NT
#define PT_NT 1
#endif
typedef float ptk_f4v __attribute__((ext_vector_type(4)));
typedef int ptk_i2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float4 ldnt(const float4* p) {
#if PT_NT
  const ptk_f4v v = __builtin_nontemporal_load((const ptk_f4v*)p);
  return make_float4(v.x, v.y, v.z, v.w);
#else
  return *p;
#endif
}
__device__ __forceinline__ void stnt(float4* p, float4 a) {
#if PT_NT
  const ptk_f4v v = {a.x, a.y, a.z, a.w};
  __builtin_nontemporal_store(v, (ptk_f4v*)p);
#else
  *p = a;
#endif
}
__device__ __forceinline__ int2 ldnt(const int2* p) {
#if PT_NT
  const ptk_i2v v = __builtin_nontemporal_load((const ptk_i2v*)p);
  return make_int2(v.x, v.y);
#else
  return *p;
#endif
}
__device__ __forceinline__ void stnt(int2* p, int2 a) {
#if PT_NT
  const ptk_i2v v = {a.x, a.y};
  __builtin_nontemporal_store(v, (ptk_i2v*)p);
#else
  *p = a;
#endif
}
template <class T>
__device__ __forceinline__ T ldnt(const T* p) {
#if PT_NT
  return __builtin_nontemporal_load(p);
#else
  return *p;
#endif
}
template <class T>
__device__ __forceinline__ void stnt(T* p, T a) {
#if PT_NT
  __builtin_nontemporal_store(a, p);
#else
  *p = a;
#endif
}
__device__ __forceinline__ void pst(const Plane& P, int x, int y, float4 v) { stnt(P.p + (size_t)prow(P, y) * P.W + x, v); }
__device__ __forceinline__ float4 f4(float x, float y, float z, float w) {
  float4 r;
  r.x = x; r.y = y; r.z = z; r.w = w;
  return r;
}
__device__ __forceinline__ v3 xyz(float4 a) { return mk(a.x, a.y, a.z); }

// ------------------------------------------------------------- materials ---
struct Mat {
  v3 emissive, baseColor;
  float subsurface, metallic, specular, specularTint, roughness, sheen, sheenTint, clearcoat, clearcoatGloss;
};

// hitAABB (:275-288) — returns the reference's distance and the entry t0.
__device__ __forceinline__ float slab(v3 o, v3 inv, float ax, float ay, float az, float bx, float by, float bz,
                                      float* t0o) {
  float fx = (bx - o.x) * inv.x, fy = (by - o.y) * inv.y, fz = (bz - o.z) * inv.z;
  float nx = (ax - o.x) * inv.x, ny = (ay - o.y) * inv.y, nz = (az - o.z) * inv.z;
  float t1 = fminf(fmaxf(fx, nx), fminf(fmaxf(fy, ny), fmaxf(fz, nz)));
  float t0 = fmaxf(fminf(fx, nx), fmaxf(fminf(fy, ny), fminf(fz, nz)));
  *t0o = t0;
  return (t1 >= t0) ? ((t0 > 0.0f) ? t0 : t1) : -1.0f;
}

// hitTriangle (:215-272) hit test; N and dot(N,p1) precomputed on the host with
// the same built-ins. Flipping N for back hits negates both dot products and
// the denominator exactly, so t and the inside test are taken unflipped.
struct TriGeom {
  float4 a, b, c, n;  // (p1, N.p1) (p2, -) (p3, -) (N, -)
};
__device__ __forceinline__ TriGeom tri_load(const float4* __restrict__ g, int i) {
  return TriGeom{g[4 * i], g[4 * i + 1], g[4 * i + 2], g[4 * i + 3]};
}
__device__ __forceinline__ bool tri_test(const TriGeom& tg, v3 S, v3 d, float* t_out) {
  v3 p1 = xyz(tg.a), p2 = xyz(tg.b), p3 = xyz(tg.c), N = xyz(tg.n);
  float dn = dot(N, d);
  if (f_abs(dn) < 0.00001f) return false;
  float t = (tg.a.w - dot(S, N)) / dn;
  if (!(t >= 0.0005f)) return false;
  v3 P = add(S, muls(d, t));
  float e1 = dot(cross(sub(p2, p1), sub(P, p1)), N);
  float e2 = dot(cross(sub(p3, p2), sub(P, p2)), N);
  float e3 = dot(cross(sub(p1, p3), sub(P, p3)), N);
  bool r1 = e1 > 0.0f && e2 > 0.0f && e3 > 0.0f;
  bool r2 = e1 < 0.0f && e2 < 0.0f && e3 < 0.0f;
  *t_out = t;
  return r1 || r2;
}
__device__ __forceinline__ bool tri_hit(const float4* __restrict__ g, int i, v3 S, v3 d, float* t_out) {
  return tri_test(tri_load(g, i), S, d, t_out);
}

// A leaf's triangles in index order (hitArray's strict '<' order, :298-369). on_hit(i, t) returns true to stop the
// scan (any-hit rays). The loop keeps the shape of a chunked fetch (kLeafChunk triangles' geometry loaded before they
// are tested): with a chunk of 1 it compiles to faster code than the plain loop (same box, 4K: 207.5 vs 190.4 fps),
// and chunks of 2 / 4 / 8 measured slower (8.4 -> 10.2 / 13.1 / 23.7 ms: registers).
constexpr int kLeafChunk = 1;
template <class F>
__device__ __forceinline__ bool leaf_scan(const float4* __restrict__ g, int first, int cnt, v3 S, v3 d,
                                          F&& on_hit) {
  const int end = first + cnt;
  for (int i0 = first; i0 < end; i0 += kLeafChunk) {
    TriGeom tg[kLeafChunk];
#pragma unroll
    for (int k = 0; k < kLeafChunk; ++k)
      if (i0 + k < end) tg[k] = tri_load(g, i0 + k);
#pragma unroll
    for (int k = 0; k < kLeafChunk; ++k) {
      if (i0 + k >= end) break;
      float t;
      if (tri_test(tg[k], S, d, &t) && on_hit(i0 + k, t)) return true;
    }
  }
  return false;
}

__device__ __forceinline__ int ref_leaf_first(int ref) { return (-(ref + 1)) >> 4; }
__device__ __forceinline__ int ref_leaf_count(int ref) { return (-(ref + 1)) & 15; }

// Traversal stacks. LdsStack: a column of the block's LDS array (slots STRIDE ints apart); the host guarantees the
// walked tree fits it. SpillStack: the first KS entries in LDS, deeper ones in this ray's column of global memory
// (entry KS + j at g[j * gs]) — for reference trees deeper than the LDS stack, which the reference walks with its
// stack[256] (path_tracing.frag:378). Only kernels launched for such trees use it.
template <int STRIDE>
struct LdsStack {
  static constexpr bool spilled = false;
  int* __restrict__ p;
  __device__ __forceinline__ void put(int sp, int v) const { p[sp * STRIDE] = v; }
  __device__ __forceinline__ int get(int sp) const { return p[sp * STRIDE]; }
};
template <int STRIDE, int KS>
struct SpillStack {
  int* __restrict__ p;
  int* __restrict__ g;
  size_t gs;
  bool spilled = false;  // some entry went past the LDS stack (traversal counter kStatSpills)
  __device__ __forceinline__ void put(int sp, int v) {
    if (sp < KS) {
      p[sp * STRIDE] = v;
    } else {
      g[(size_t)(sp - KS) * gs] = v;
      spilled = true;
    }
  }
  __device__ __forceinline__ int get(int sp) const { return sp < KS ? p[sp * STRIDE] : g[(size_t)(sp - KS) * gs]; }
};

// mode 0: closest hit (hitBVH :372-424); mode 1: any hit (HDR shadow);
// mode 2: any hit nearer than `maxd` by length(P - S) (point-light shadow).
//
// While-while loop with one postponed leaf per lane (Aila & Laine 2009): lanes
// keep descending interior nodes until every lane of the wave holds a leaf, then
// all intersect together, which keeps wave64 lanes converged. Leaves are still
// intersected in the order the depth-first walk reaches them, so the strict '<'
// tie rule of hitArray/hitBVH picks the same triangle.
// `stk` is this lane's stack (LdsStack / SpillStack above).
constexpr int kNone = kNoneRef;

// `steps` (optional) receives the node + triangle visits (load-balancing probe).
template <int MODE, class Stk>
__device__ int traverse(const SceneDev& sc, Stk& stk, v3 S, v3 d, float maxd, int prune,
                        float* t_best_out, uint32_t* steps = nullptr, float t_init = PT_INF, bool* tie = nullptr) {
  v3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  float tbest = t_init;  // MODE 0 with t_init < inf: only hits nearer than t_init are sought (caller falls back)
  int best = -1;
  bool tied = false;  // another triangle met the current best t exactly (the visit order would decide)
  int sp = 0;
  int node = sc.root_ref;
  int leaf = kNone;
  uint32_t nvis = 0;
  if (node < 0) { leaf = node; node = kNone; }
  while (node != kNone || leaf != kNone) {
    while (node >= 0) {  // interior nodes (kNone and leaf refs are negative)
      nvis += PT_NODE_VISIT;
      const float4* nd = sc.bvh + 4 * node;
      float4 q0 = nd[0], q1 = nd[1], q2 = nd[2], q3 = nd[3];
      float t0l, t0r;
      float dl = slab(S, inv, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, &t0l);
      float dr = slab(S, inv, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, &t0r);
      bool hl = dl > 0.0f, hr = dr > 0.0f;
      if (MODE == 0 && prune) {
        float lim = tbest * 1.0002f + 2.0e-4f;
        hl = hl && !(t0l > lim);
        hr = hr && !(t0r > lim);
      } else if (MODE == 2) {
        float lim = maxd * 1.0002f + 2.0e-4f;
        hl = hl && !(t0l > lim);
        hr = hr && !(t0r > lim);
      }
      int cl = __float_as_int(q3.x), cr = __float_as_int(q3.y);
      if (hl && hr) {
        bool lnear = dl < dr;
        stk.put(sp++, lnear ? cr : cl);
        node = lnear ? cl : cr;
      } else if (hl) {
        node = cl;
      } else if (hr) {
        node = cr;
      } else {
        node = sp > 0 ? stk.get(--sp) : kNone;
      }
      if (node < 0 && node != kNone && leaf == kNone) {  // postpone this leaf, keep walking
        leaf = node;
        node = sp > 0 ? stk.get(--sp) : kNone;
      }
      if (!__any(leaf == kNone)) break;  // every lane holds a leaf: intersect together
    }
    while (leaf != kNone) {
      int first = ref_leaf_first(leaf), cnt = ref_leaf_count(leaf);
      nvis += (uint32_t)cnt;
      int anyi = -1;
      float anyt = 0.0f;
      const bool stop = leaf_scan(sc.tri_geom, first, cnt, S, d, [&](int i, float t) {
        if (MODE == 0) {
          if (t < tbest) { tbest = t; best = i; tied = false; }
          else if (t == tbest && best >= 0) tied = true;  // (a hit exactly at the bound t_init is no tie)
          return false;
        }
        if (!(t < PT_INF)) return false;
        if (MODE == 2 && !(length(sub(add(S, muls(d, t)), S)) < maxd)) return false;
        anyi = i;
        anyt = t;
        return true;
      });
      if (MODE != 0 && stop) {
        *t_best_out = anyt;
        if (steps) *steps = nvis;
        return anyi;
      }
      leaf = kNone;
      if (node < 0 && node != kNone) {  // the walk stopped on a second leaf: it is next in order
        leaf = node;
        node = sp > 0 ? stk.get(--sp) : kNone;
      }
    }
  }
  *t_best_out = tbest;
  if (steps) *steps = nvis;
  if (tie) *tie = tied;
  return best;
}

// Closest hit (hitBVH :372-424) for the wavefront kernels. With `sah` (PTParams::closest_tree) the walk runs on
// the SAH tree over the reference's leaves (bvh_any): the candidate set is the reference walk's (the same leaves,
// tested on the same leaf boxes, which lie inside every reference ancestor box, so a leaf box the ray passes is
// one hitBVH reaches), so the minimum t and, when one triangle alone attains it, the triangle are the reference's.
// When two triangles attain the same t exactly, the reference keeps the one its depth-first order meets first:
// that ray is walked again on the reference tree in the reference's order. Same bits either way.
template <class Stk>
__device__ __forceinline__ int closest_hit(const SceneDev& sc, bool sah, Stk& stk, v3 S, v3 d, int prune,
                                           float* t, uint32_t* steps, float t_init = PT_INF, bool* rewalk = nullptr) {
  if (!sah) return traverse<0>(sc, stk, S, d, 0.0f, prune, t, steps, t_init);
  bool tie = false;
  int tri = traverse<0>(anyhit_scene(sc), stk, S, d, 0.0f, 1, t, steps, t_init, &tie);
  if (rewalk) *rewalk = tie;
  if (tie) {
    uint32_t more = 0;
    tri = traverse<0>(sc, stk, S, d, 0.0f, 1, t, &more, t_init);
    if (steps) *steps += more;
  }
  return tri;
}

// Any-hit traversal of the 4-wide BVH (shadow rays): HDR rays take any hit,
// point-light rays any hit nearer than `maxd` by length(P - S) — the same
// triangle tests as traverse<1|2>, whose verdict does not depend on the order
// leaves are visited.
// Per node: the four child boxes are slab-tested (same hitAABB arithmetic); the
// walk continues into one hit child and pushes the others; leaves are postponed
// one per lane (while-while) so the wave intersects together.
// `point` is a runtime flag so HDR and point-light rays share one instruction
// stream in a wave (they differ only in the pruning bound and the hit predicate).
// Any-hit walk of the binary tree for both shadow kinds: traverse<1> (HDR, any
// hit) and traverse<2> (point light: boxes entered beyond the light pruned, hit
// nearer than `maxd`) merged behind a runtime flag, so a wave runs one loop.
// budget > 0: a ray whose walk exceeds `budget` node + triangle visits stops and reports *deferred (its
// verdict is then decided by the wave-cooperative walk, shadow_coop_walk below).
template <class Stk>
__device__ bool anyhit2(const SceneDev& sc, Stk& stk, v3 S, v3 d, bool point, float maxd,
                        uint32_t* steps, uint32_t budget = 0, bool* deferred = nullptr) {
  v3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  const float lim = point ? maxd * 1.0002f + 2.0e-4f : __builtin_inff();
  int sp = 0;
  int node = sc.root_ref;
  int leaf = kNone;
  uint32_t nvis = 0;
  if (node < 0) { leaf = node; node = kNone; }
  while (node != kNone || leaf != kNone) {
    if (budget && nvis > budget) {
      *deferred = true;
      if (steps) *steps = nvis;
      return false;
    }
    while (node >= 0) {
      nvis += PT_NODE_VISIT;
      const float4* nd = sc.bvh + 4 * node;
      float4 q0 = nd[0], q1 = nd[1], q2 = nd[2], q3 = nd[3];
      float t0l, t0r;
      float dl = slab(S, inv, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, &t0l);
      float dr = slab(S, inv, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, &t0r);
      const bool hl = dl > 0.0f && !(t0l > lim), hr = dr > 0.0f && !(t0r > lim);
      int cl = __float_as_int(q3.x), cr = __float_as_int(q3.y);
      if (hl && hr) {
        bool lnear = dl < dr;
        stk.put(sp++, lnear ? cr : cl);
        node = lnear ? cl : cr;
      } else if (hl) {
        node = cl;
      } else if (hr) {
        node = cr;
      } else {
        node = sp > 0 ? stk.get(--sp) : kNone;
      }
      if (node < 0 && node != kNone && leaf == kNone) {
        leaf = node;
        node = sp > 0 ? stk.get(--sp) : kNone;
      }
      if (!__any(leaf == kNone)) break;
    }
    while (leaf != kNone) {
      int first = ref_leaf_first(leaf), cnt = ref_leaf_count(leaf);
      nvis += (uint32_t)cnt;
      if (leaf_scan(sc.tri_geom, first, cnt, S, d, [&](int, float t) {
            return t < PT_INF && (!point || length(sub(add(S, muls(d, t)), S)) < maxd);
          })) {
        if (steps) *steps = nvis;
        return true;
      }
      leaf = kNone;
      if (node < 0 && node != kNone) {
        leaf = node;
        node = sp > 0 ? stk.get(--sp) : kNone;
      }
    }
  }
  if (steps) *steps = nvis;
  return false;
}

// Wave-cooperative any-hit walk of ONE shadow ray (the stragglers of anyhit2's budget): the 64 lanes pop the
// top 64 entries of a shared LDS stack, each tests its node's two child boxes (hitAABB, the same pruning bound)
// or its leaf's triangles, and the surviving children are pushed back (far before near, so the walk stays close
// to depth-first and the stack small). A launch's tail is set by its longest chain of dependent fetches; this
// expands up to 64 nodes per fetch instead of one. The verdict is order-free (any hit), so it equals the
// serial walk's. `st` is this wave's LDS stack of `cap` entries; on overflow the wave falls back to the serial
// walk on lane 0 (rare, correct, slow). Call with the whole wave (wave-uniform ray).
__device__ bool shadow_coop_walk(const SceneDev& sc, int* __restrict__ st, int cap, v3 S, v3 d, bool point, float maxd) {
  const int lane = threadIdx.x & 63;
  const v3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  const float lim = point ? maxd * 1.0002f + 2.0e-4f : __builtin_inff();
  int count = 1;
  if (lane == 0) st[0] = sc.root_ref;
  __builtin_amdgcn_wave_barrier();
  bool overflow = false;
  while (count > 0) {
    const int k = count < 64 ? count : 64;
    const int ref = lane < k ? st[count - 1 - lane] : kNone;
    count -= k;
    __builtin_amdgcn_wave_barrier();
    bool hit = false;
    int push0 = kNone, push1 = kNone;  // far, near
    if (ref >= 0) {
      const float4* nd = sc.bvh + 4 * ref;
      float4 q0 = nd[0], q1 = nd[1], q2 = nd[2], q3 = nd[3];
      float t0l, t0r;
      float dl = slab(S, inv, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, &t0l);
      float dr = slab(S, inv, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, &t0r);
      const bool hl = dl > 0.0f && !(t0l > lim), hr = dr > 0.0f && !(t0r > lim);
      const int cl = __float_as_int(q3.x), cr = __float_as_int(q3.y);
      if (hl && hr) {
        const bool lnear = dl < dr;
        push0 = lnear ? cr : cl;
        push1 = lnear ? cl : cr;
      } else if (hl) {
        push1 = cl;
      } else if (hr) {
        push1 = cr;
      }
    } else if (ref != kNone) {
      hit = leaf_scan(sc.tri_geom, ref_leaf_first(ref), ref_leaf_count(ref), S, d, [&](int, float t) {
        return t < PT_INF && (!point || length(sub(add(S, muls(d, t)), S)) < maxd);
      });
    }
    if (__any(hit)) return true;
    const unsigned long long m0 = __ballot(push0 != kNone), m1 = __ballot(push1 != kNone);
    const int n0 = __popcll(m0), n1 = __popcll(m1);
    if (count + n0 + n1 > cap) {
      overflow = true;
      break;
    }
    const unsigned long long lt = (1ull << lane) - 1ull;
    if (push0 != kNone) st[count + __popcll(m0 & lt)] = push0;           // all far children first,
    if (push1 != kNone) st[count + n0 + __popcll(m1 & lt)] = push1;      // then the near ones on top
    count += n0 + n1;
    __builtin_amdgcn_wave_barrier();
  }
  if (!overflow) return false;
  // overflow: lane 0 walks the whole ray serially on the (now free) LDS region
  bool occ = false;
  LdsStack<1> ls{st};
  if (lane == 0) occ = anyhit2(sc, ls, S, d, point, maxd, nullptr);
  return __any(occ);
}

// Wave-cooperative closest hit of ONE ray (the stragglers of the bounce walk's visit budget), the same answer as
// closest_hit(sah = true): the 64 lanes pop the top 64 entries of a shared LDS stack of the SAH tree over the
// reference leaves, test node children with the walk's pruning bound (from the wave's best t so far) or scan a
// leaf's triangles keeping a lane-local best and how many triangles met it exactly; the candidates are the
// serial walk's, so the minimum t is too, and when one triangle alone attains it, the triangle. When two do, lane 0
// walks the ray on the reference tree in the reference's order (traverse<0>), as closest_hit does; also when the
// shared stack would overflow (closest_hit itself). Returns the triangle; *t_out the t. Call with the whole wave.
__device__ int closest_coop_walk(const SceneDev& sc, int* __restrict__ st, int cap, v3 S, v3 d, float* t_out,
                                 bool* rewalked) {
  const int lane = threadIdx.x & 63;
  const SceneDev sa = anyhit_scene(sc);
  const v3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  float lb = PT_INF, tw = PT_INF;  // lane's best, wave's best so far
  int li = -1, lc = 0;             // lane's best triangle, triangles that met lb exactly
  int count = 1;
  if (lane == 0) st[0] = sa.root_ref;
  __builtin_amdgcn_wave_barrier();
  bool overflow = false;
  while (count > 0) {
    const int k = count < 64 ? count : 64;
    const int ref = lane < k ? st[count - 1 - lane] : kNone;
    count -= k;
    __builtin_amdgcn_wave_barrier();
    const float lim = tw * 1.0002f + 2.0e-4f;
    int push0 = kNone, push1 = kNone;  // far, near
    if (ref >= 0) {
      const float4* nd = sa.bvh + 4 * ref;
      const float4 q0 = nd[0], q1 = nd[1], q2 = nd[2], q3 = nd[3];
      float t0l, t0r;
      const float dl = slab(S, inv, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, &t0l);
      const float dr = slab(S, inv, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, &t0r);
      const bool hl = dl > 0.0f && !(t0l > lim), hr = dr > 0.0f && !(t0r > lim);
      const int cl = __float_as_int(q3.x), cr = __float_as_int(q3.y);
      if (hl && hr) {
        const bool lnear = dl < dr;
        push0 = lnear ? cr : cl;
        push1 = lnear ? cl : cr;
      } else if (hl) {
        push1 = cl;
      } else if (hr) {
        push1 = cr;
      }
    } else if (ref != kNone) {
      leaf_scan(sc.tri_geom, ref_leaf_first(ref), ref_leaf_count(ref), S, d, [&](int i, float t) {
        if (t < lb) { lb = t; li = i; lc = 1; }
        else if (t == lb) ++lc;
        return false;
      });
    }
    float m = lb;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fminf(m, __shfl_xor(m, o));
    tw = m;
    const unsigned long long m0 = __ballot(push0 != kNone), m1 = __ballot(push1 != kNone);
    const int n0 = __popcll(m0), n1 = __popcll(m1);
    if (count + n0 + n1 > cap) {
      overflow = true;
      break;
    }
    const unsigned long long lt = (1ull << lane) - 1ull;
    if (push0 != kNone) st[count + __popcll(m0 & lt)] = push0;           // all far children first,
    if (push1 != kNone) st[count + n0 + __popcll(m1 & lt)] = push1;      // then the near ones on top
    count += n0 + n1;
    __builtin_amdgcn_wave_barrier();
  }
  int n_at = (!overflow && lb == tw && tw < PT_INF) ? lc : 0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) n_at += __shfl_xor(n_at, o);
  if (!overflow && n_at < 2) {  // one triangle attains the minimum (or none: a miss)
    const unsigned long long own = __ballot(tw < PT_INF && lb == tw);
    const int tri = own ? __shfl(li, __ffsll((long long)own) - 1) : -1;
    *t_out = tw;
    *rewalked = false;
    return tri;
  }
  // a tie (or overflow): lane 0 walks, on the (now free) LDS region
  __builtin_amdgcn_wave_barrier();
  int tri = -1;
  float t = PT_INF;
  LdsStack<1> ls{st};
  if (lane == 0) {
    if (overflow) {
      bool rw = false;
      tri = closest_hit(sc, true, ls, S, d, 1, &t, nullptr, PT_INF, &rw);
    } else {
      tri = traverse<0>(sc, ls, S, d, 0.0f, 1, &t, nullptr, PT_INF);
    }
  }
  *t_out = __shfl(t, 0);
  *rewalked = !overflow;
  return __shfl(tri, 0);
}

// One node of a 4-wide walk (pack_wide's layout) for the lane-refill kernels: the four child boxes are slab-tested
// (hitAABB, :275-288), a child counts as hit when hitAABB's distance is > 0 and its entry t0 is not beyond `lim` (the
// pruning bound of the binary walks), the walk descends into the nearest hit child (hitAABB's distance, ties to the
// lower slot) and pushes the others farthest first, so the next pop is the next nearest (SORT; without it, for
// any-hit rays whose verdict does not depend on the order, the first hit slot is taken and the others pushed). With
// no hit child it pops.
// Returns false, leaving the stack as it was, when the pushes would overflow the KS-entry stack: the caller hands the
// ray to the cooperative walk.
__device__ __forceinline__ bool finite3(v3 a) {
  return __builtin_isfinite(a.x) && __builtin_isfinite(a.y) && __builtin_isfinite(a.z);
}

#if PT_WIDE_SIGNED && (defined(__FAST_MATH__) || __FINITE_MATH_ONLY__)
#error "PT_WIDE_SIGNED's one-compare child test needs IEEE f32 (subnormals kept, no finite-math): build without fast-math"
#endif
template <int KS, bool SORT, class Stk>
__device__ __forceinline__ bool wide_step(const float4* __restrict__ tree, int& node, Stk& st, int& sp, v3 S, v3 inv,
                                          float lim) {
  const float4* q = tree + kWideStride * node;
  int ref[4];
  float key[4];  // hitAABB's distance of a hit child (PT_WIDE_SIGNED: its entry t0), +inf otherwise
  int nh = 0;
#if PT_WIDE_SIGNED
  // For a ray whose inv components are all finite (the kernels hand the others to the cooperative walk) and a box
  // with lo <= hi (a tree with a NaN coordinate in a child box is not walked 4-wide: capi.hip), the near plane of an
  // axis is the lo plane when inv >= 0 (+0 included) and the hi plane otherwise: (b - o) * inv rounds monotonically
  // in b, so slab's min(fx, nx) IS that plane's value and its max(fx, nx) the other's — the same floats, picked by
  // which float4 is loaded instead of by 6 min / max per child. hitAABB's d > 0 is t1 >= t0 && t1 > 0 (d is t0 when
  // t0 > 0, then t1 >= t0 > 0; else d is t1). Sort key: the entry t0 (the order only decides which hit child is
  // walked first: the candidate triangles, hence the closest t, a unique closest triangle, an exact tie met and every
  // any-hit verdict do not depend on it).
  {
    const int sx = inv.x < 0.0f, sy = inv.y < 0.0f, sz = inv.z < 0.0f;
    const float4 nx4 = q[sx], fx4 = q[1 - sx], ny4 = q[2 + sy], fy4 = q[3 - sy], nz4 = q[4 + sz], fz4 = q[5 - sz];
    float4 rf = q[6];
    const float anx[4] = {nx4.x, nx4.y, nx4.z, nx4.w}, afx[4] = {fx4.x, fx4.y, fx4.z, fx4.w};
    const float any_[4] = {ny4.x, ny4.y, ny4.z, ny4.w}, afy[4] = {fy4.x, fy4.y, fy4.z, fy4.w};
    const float anz[4] = {nz4.x, nz4.y, nz4.z, nz4.w}, afz[4] = {fz4.x, fz4.y, fz4.z, fz4.w};
    // t1 >= t0 && t1 > 0 && !(t0 > lim) as ONE compare: t1 > 0 is t1 >= the least subnormal (f32 subnormals are kept),
    // and lim > 0 (a shadow ray's maxd scaled + 2e-4, a bounce ray's best t scaled + 2e-4, or +inf), so with
    // t0c = max(t0, least subnormal) it is t0c <= min(t1, lim) (no NaN: finite planes and inv, or the +-inf planes of
    // an empty slot). An empty slot (pack_wide: lo = +inf, hi = -inf) has t0 = +inf, t1 = -inf: never hit, so the
    // slot's ref is not tested. The sort key is t0c (order among children entered at t0 <= 0 is free, see above).
    // (needs f32 subnormals kept: a build that flushes them would make tiny 0 and enter children with t1 == 0;
    // fast-math builds are refused below, and pt_init refuses a device whose walk code flushes, subnormal_probe)
    const float tiny = __builtin_bit_cast(float, 1u);
    float t0c[4], t1l[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float t1 = fminf((afx[c] - S.x) * inv.x, fminf((afy[c] - S.y) * inv.y, (afz[c] - S.z) * inv.z));
      const float t0 = fmaxf((anx[c] - S.x) * inv.x, fmaxf((any_[c] - S.y) * inv.y, (anz[c] - S.z) * inv.z));
      t0c[c] = fmaxf(t0, tiny);
      t1l[c] = fminf(t1, lim);
    }
    // the refs are needed only once a child is hit; without this use (after the box arithmetic, so the box loads'
    // arithmetic still overlaps the refs' arrival) the compiler loads them after the hit test: a second dependent
    // fetch per node step instead of one fetch of the node's seven float4
    asm volatile("" : "+v"(rf.x), "+v"(rf.y), "+v"(rf.z), "+v"(rf.w)
                 : "v"(t0c[0]), "v"(t0c[1]), "v"(t0c[2]), "v"(t0c[3]), "v"(t1l[0]), "v"(t1l[1]), "v"(t1l[2]),
                   "v"(t1l[3]));
    const int rr[4] = {__float_as_int(rf.x), __float_as_int(rf.y), __float_as_int(rf.z), __float_as_int(rf.w)};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const bool hit = t0c[c] <= t1l[c];
      key[c] = hit ? t0c[c] : __builtin_inff();
      ref[c] = hit ? rr[c] : kNone;
      nh += hit ? 1 : 0;
    }
  }
#else
  {
    const float4 lx = q[0], hx = q[1], ly = q[2], hy = q[3], lz = q[4], hz = q[5], rf = q[6];
    const float alx[4] = {lx.x, lx.y, lx.z, lx.w}, ahx[4] = {hx.x, hx.y, hx.z, hx.w};
    const float aly[4] = {ly.x, ly.y, ly.z, ly.w}, ahy[4] = {hy.x, hy.y, hy.z, hy.w};
    const float alz[4] = {lz.x, lz.y, lz.z, lz.w}, ahz[4] = {hz.x, hz.y, hz.z, hz.w};
    const int rr[4] = {__float_as_int(rf.x), __float_as_int(rf.y), __float_as_int(rf.z), __float_as_int(rf.w)};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float t0;
      const float dist = slab(S, inv, alx[c], aly[c], alz[c], ahx[c], ahy[c], ahz[c], &t0);
      const bool hit = rr[c] != kNone && dist > 0.0f && !(t0 > lim);
      key[c] = hit ? dist : __builtin_inff();
      ref[c] = hit ? rr[c] : kNone;
      nh += hit ? 1 : 0;
    }
  }
#endif
  if (nh == 0) {
    node = sp > 0 ? st.get(--sp) : kNone;
    return true;
  }
  if (sp + nh - 1 > KS) return false;
  if constexpr (SORT) {
    // sorting network on (key, slot): 5 compare-exchanges; stable for equal keys (slot order kept)
    auto cx = [&](int a, int b) __attribute__((always_inline)) {
      const bool sw = key[b] < key[a];
      const float ka = key[a], kb = key[b];
      const int ra = ref[a], rb = ref[b];
      key[a] = sw ? kb : ka;
      key[b] = sw ? ka : kb;
      ref[a] = sw ? rb : ra;
      ref[b] = sw ? ra : rb;
    };
    cx(0, 1);
    cx(2, 3);
    cx(0, 2);
    cx(1, 3);
    cx(1, 2);
    // hit children now lead in near-to-far order: push slots nh-1 .. 1, take slot 0
#pragma unroll
    for (int r = 3; r >= 1; --r)
      if (r < nh) st.put(sp++, ref[r]);
    node = ref[0];
  } else {
    // any order (any-hit): take the first hit slot, push the others
    int first = kNone;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (ref[c] == kNone) continue;
      if (first == kNone) first = ref[c];
      else st.put(sp++, ref[c]);
    }
    node = first;
  }
  return true;
}

// Returns 1 occluded, 0 visible, -1 when the stack would overflow (the caller
// re-traces that ray on the binary tree, whose depth the host bounds by kStack).
template <int STRIDE, int KS = kStack>
__device__ int anyhit4(const SceneDev& sc, int* __restrict__ stk, v3 S, v3 d, bool point, float maxd,
                       uint32_t* steps) {
  v3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  const float lim = point ? maxd * 1.0002f + 2.0e-4f : __builtin_inff();
  int sp = 0;
  int node = sc.root4;
  int leaf = kNone;
  uint32_t nvis = 0;
  if (node < 0) { leaf = node; node = kNone; }
  while (node != kNone || leaf != kNone) {
    while (node >= 0) {
      nvis += PT_NODE_VISIT;
      const float4* q = sc.bvh4 + kWideStride * node;
      const float4 lx = q[0], hx = q[1], ly = q[2], hy = q[3], lz = q[4], hz = q[5], rf = q[6];
      const float alx[4] = {lx.x, lx.y, lx.z, lx.w}, ahx[4] = {hx.x, hx.y, hx.z, hx.w};
      const float aly[4] = {ly.x, ly.y, ly.z, ly.w}, ahy[4] = {hy.x, hy.y, hy.z, hy.w};
      const float alz[4] = {lz.x, lz.y, lz.z, lz.w}, ahz[4] = {hz.x, hz.y, hz.z, hz.w};
      const int ref[4] = {__float_as_int(rf.x), __float_as_int(rf.y), __float_as_int(rf.z), __float_as_int(rf.w)};
      int next = kNone;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float t0;
        float dist = slab(S, inv, alx[c], aly[c], alz[c], ahx[c], ahy[c], ahz[c], &t0);
        const bool hit = ref[c] != kNone && dist > 0.0f && !(t0 > lim);
        if (hit) {
          if (next == kNone) {
            next = ref[c];
          } else {
            if (sp == KS) return -1;
            stk[sp++ * STRIDE] = ref[c];
          }
        }
      }
      node = next != kNone ? next : (sp > 0 ? stk[--sp * STRIDE] : kNone);
      if (node < 0 && node != kNone && leaf == kNone) {  // postpone this leaf, keep walking
        leaf = node;
        node = sp > 0 ? stk[--sp * STRIDE] : kNone;
      }
      if (!__any(leaf == kNone)) break;
    }
    while (leaf != kNone) {
      int first = ref_leaf_first(leaf), cnt = ref_leaf_count(leaf);
      nvis += (uint32_t)cnt;
      if (leaf_scan(sc.tri_geom, first, cnt, S, d, [&](int, float t) {  // :905-909 for point lights
            return t < PT_INF && (!point || length(sub(add(S, muls(d, t)), S)) < maxd);
          })) {
        if (steps) *steps = nvis;
        return 1;
      }
      leaf = kNone;
      if (node < 0 && node != kNone) {
        leaf = node;
        node = sp > 0 ? stk[--sp * STRIDE] : kNone;
      }
    }
  }
  if (steps) *steps = nvis;
  return 0;
}

struct Hit {
  bool isHit;
  v3 P, normal, viewDir;
  Mat m;
};

// texture2DArray(material_array, vec3(u, v, layer)) (:331-364): RGBA8 UNORM texels (c / 255), GL_LINEAR,
// GL_CLAMP_TO_EDGE, one level (main.cpp:186-195), the layer rounded and clamped as GL does; the shared
// bilinear addressing of glsl_builtins.h. With no array bound the fetch reads 0.
__device__ __forceinline__ float unorm8(uint32_t t, int c) { return (float)((t >> (8 * c)) & 255u) / 255.0f; }
__device__ __forceinline__ void tex_array(const SceneDev& sc, float u, float v, int layer, float* out) {
  if (!sc.texarr) {
    out[0] = out[1] = out[2] = out[3] = 0.0f;
    return;
  }
  layer = clampi(layer, 0, sc.tex_layers - 1);
  const Bilin b = bilin_setup(u, v, sc.tex_w, sc.tex_h);
  const uint32_t* L = sc.texarr + (size_t)layer * sc.tex_w * sc.tex_h;
  const uint32_t t00 = L[(size_t)b.y0 * sc.tex_w + b.x0], t10 = L[(size_t)b.y0 * sc.tex_w + b.x1];
  const uint32_t t01 = L[(size_t)b.y1 * sc.tex_w + b.x0], t11 = L[(size_t)b.y1 * sc.tex_w + b.x1];
  for (int c = 0; c < 4; ++c) out[c] = bilin_mix(b, unorm8(t00, c), unorm8(t10, c), unorm8(t01, c), unorm8(t11, c));
}

// Decode the closest hit (hitTriangle :243-268 normal; hitArray :315-366 material).
__device__ Hit decode_hit(const SceneDev& sc, int i, float t, v3 S, v3 d) {
  Hit h;
  h.isHit = true;
  float4 a = sc.tri_geom[4 * i], b = sc.tri_geom[4 * i + 1], c = sc.tri_geom[4 * i + 2], gn = sc.tri_geom[4 * i + 3];
  v3 p1 = xyz(a), p2 = xyz(b), p3 = xyz(c);
  bool inside = dot(xyz(gn), d) > 0.0f;
  v3 P = add(S, muls(d, t));
  const float4* r = sc.tri_shade + 9 * i;
  float4 r0 = r[0], r1 = r[1], r2 = r[2], r3 = r[3], r4 = r[4], r5 = r[5], r6 = r[6];
  v3 n1 = mk(r0.x, r0.y, r0.z), n2 = mk(r0.w, r1.x, r1.y), n3 = mk(r1.z, r1.w, r2.x);
  float alpha = ((-(P.x - p2.x)) * (p3.y - p2.y) + (P.y - p2.y) * (p3.x - p2.x)) /
                ((-(p1.x - p2.x)) * (p3.y - p2.y) + (p1.y - p2.y) * (p3.x - p2.x) + 1e-7f);
  float beta = ((-(P.x - p3.x)) * (p1.y - p3.y) + (P.y - p3.y) * (p1.x - p3.x)) /
               ((-(p2.x - p3.x)) * (p1.y - p3.y) + (p2.y - p3.y) * (p1.x - p3.x) + 1e-7f);
  float gama = (1.0f - alpha) - beta;
  v3 Ns = normalize(add(add(muls(n1, alpha), muls(n2, beta)), muls(n3, gama)));
  h.P = P;
  h.normal = inside ? neg(Ns) : Ns;
  h.viewDir = d;
  h.m.emissive = mk(r2.y, r2.z, r2.w);
  h.m.baseColor = mk(r3.x, r3.y, r3.z);
  h.m.subsurface = r3.w;
  h.m.metallic = r4.x;
  h.m.specular = r4.y;
  h.m.specularTint = r4.z;
  h.m.roughness = r4.w;
  h.m.sheen = r5.y;
  h.m.sheenTint = r5.z;
  h.m.clearcoat = r5.w;
  h.m.clearcoatGloss = r6.x;
  // texture-array branch (:315-364) of the closest hit (hitArray applies it per leaf to the leaf's closest
  // triangle; hitBVH compares distances only, so applying it once to the global closest is the same)
  const float4 r7 = r[7], r8 = r[8];
  const float u = (alpha * r7.x + beta * r7.z) + gama * r8.x;  // smooth_uv (:328), uv1 uv2 uv3
  const float v = (alpha * r7.y + beta * r7.w) + gama * r8.y;
  const int mat_id = (int)r6.w * 4;                           // objIndex * 4 (:330)
  if (h.m.baseColor.x < 0.0f || h.m.baseColor.y < 0.0f || h.m.baseColor.z < 0.0f) {
    float c[4];
    tex_array(sc, u, v, mat_id, c);
    h.m.baseColor = mk(c[0], c[1], c[2]);
  }
  if (h.m.metallic < 0.0f) {
    float c[4];
    tex_array(sc, u, v, mat_id + 1, c);
    h.m.metallic = c[0];
  }
  if (sc.use_normal_map) {  // :338-361, TBN from the triangle's edges and uv deltas
    v3 edge1 = sub(p2, p1), edge2 = sub(p3, p1);
    float du1 = r7.z - r7.x, dv1 = r7.w - r7.y, du2 = r8.x - r7.x, dv2 = r8.y - r7.y;
    float f = 1.0f / (du1 * dv2 - du2 * dv1);
    v3 tangent = normalize(mk(f * (dv2 * edge1.x - dv1 * edge2.x), f * (dv2 * edge1.y - dv1 * edge2.y),
                              f * (dv2 * edge1.z - dv1 * edge2.z)));
    v3 bitangent = cross(tangent, h.normal);
    float c[4];
    tex_array(sc, u, v, mat_id + 2, c);
    v3 tn = normalize(sub(muls(mk(c[0], c[1], c[2]), 2.0f), splat(1.0f)));
    h.normal = normalize(add(add(muls(tangent, tn.x), muls(bitangent, tn.y)), muls(h.normal, tn.z)));
  }
  if (h.m.roughness < 0.0f) {
    float c[4];
    tex_array(sc, u, v, mat_id + 3, c);
    h.m.roughness = c[0];
  }
  return h;
}

// ------------------------------------------------------------ Disney BRDF ---
__device__ __forceinline__ float sqr(float x) { return x * x; }
__device__ __forceinline__ float schlick(float u) {  // :524-528
  float m = f_clamp(1.0f - u, 0.0f, 1.0f);
  float m2 = m * m;
  return (m2 * m2) * m;
}
__device__ __forceinline__ float gtr1(float NdotH, float a) {  // :530-535
  if (a >= 1.0f) return 1.0f / PT_PI;
  float a2 = a * a;
  float t = 1.0f + ((a2 - 1.0f) * NdotH) * NdotH;
  return (a2 - 1.0f) / ((PT_PI * g_log(a2)) * t);
}
__device__ __forceinline__ float gtr2(float NdotH, float a) {  // :537-541
  float a2 = a * a;
  float t = 1.0f + ((a2 - 1.0f) * NdotH) * NdotH;
  return a2 / ((PT_PI * t) * t);
}
__device__ __forceinline__ float smith(float NdotV, float alphaG) {  // :547-551
  float a = alphaG * alphaG, b = NdotV * NdotV;
  return 1.0f / (NdotV + f_sqrt((a + b) - a * b));
}

__device__ v3 brdf_eval(v3 V, v3 N, v3 L, const Mat& m) {  // :620-669
  float NdotL = dot(N, L), NdotV = dot(N, V);
  if (NdotL < 0.0f || NdotV < 0.0f) return splat(0.0f);
  v3 H = normalize(add(L, V));
  float NdotH = dot(N, H), LdotH = dot(L, H);
  v3 Cd = m.baseColor;
  float Cdlum = (0.3f * Cd.x + 0.6f * Cd.y) + 0.1f * Cd.z;
  v3 Ctint = (Cdlum > 0.0f) ? divs(Cd, Cdlum) : splat(1.0f);
  v3 Cspec = muls(mixv(splat(1.0f), Ctint, m.specularTint), m.specular);
  v3 Cspec0 = mixv(muls(Cspec, 0.08f), Cd, m.metallic);
  v3 Csheen = mixv(splat(1.0f), Ctint, m.sheenTint);
  float Fd90 = 0.5f + ((2.0f * LdotH) * LdotH) * m.roughness;
  float FL = schlick(NdotL), FV = schlick(NdotV);
  float Fd = f_mix(1.0f, Fd90, FL) * f_mix(1.0f, Fd90, FV);
  float Fss90 = (LdotH * LdotH) * m.roughness;
  float Fss = f_mix(1.0f, Fss90, FL) * f_mix(1.0f, Fss90, FV);
  float ss = 1.25f * (Fss * (1.0f / (NdotL + NdotV) - 0.5f) + 0.5f);
  float Ds = gtr2(NdotH, f_max(0.001f, sqr(m.roughness)));
  float FH = schlick(LdotH);
  v3 Fs = mixv(Cspec0, splat(1.0f), FH);
  float Gs = smith(NdotL, m.roughness);
  Gs *= smith(NdotV, m.roughness);
  float Dr = gtr1(NdotH, f_mix(0.1f, 0.001f, m.clearcoatGloss));
  float Fr = f_mix(0.04f, 1.0f, FH);
  float Gr = smith(NdotL, 0.25f) * smith(NdotV, 0.25f);
  v3 Fsheen = muls(Csheen, FH * m.sheen);
  v3 diffuse = add(muls(Cd, (1.0f / PT_PI) * f_mix(Fd, ss, m.subsurface)), Fsheen);
  v3 specular = muls(muls(Fs, Gs), Ds);
  v3 clearcoat = splat((((0.25f * Gr) * Fr) * Dr) * m.clearcoat);
  return add(add(muls(diffuse, 1.0f - m.metallic), specular), clearcoat);
}

__device__ float brdf_pdf(v3 V, v3 N, v3 L, const Mat& m) {  // :837-874
  float NdotL = dot(N, L), NdotV = dot(N, V);
  if (NdotL < 0.0f || NdotV < 0.0f) return 0.0f;
  v3 H = normalize(add(L, V));
  float NdotH = dot(N, H), LdotH = dot(L, H);
  float Ds = gtr2(NdotH, f_max(0.001f, sqr(m.roughness)));
  float Dr = gtr1(NdotH, f_mix(0.1f, 0.001f, m.clearcoatGloss));
  float pd = NdotL / PT_PI;
  float ps = (Ds * NdotH) / (4.0f * LdotH);
  float pc = (Dr * NdotH) / (4.0f * LdotH);
  float rd = 1.0f - m.metallic, rs = 1.0f, rc = 0.25f * m.clearcoat;
  float rsum = (rd + rs) + rc;
  float pdf = ((rd / rsum) * pd + (rs / rsum) * ps) + (rc / rsum) * pc;
  return f_max(1e-10f, pdf);
}

__device__ __forceinline__ v3 to_hemi(v3 v, v3 N) {  // toNormalHemisphere :681-687
  v3 helper = (f_abs(N.x) > 0.999f) ? mk(0, 0, 1) : mk(1, 0, 0);
  v3 T = normalize(cross(N, helper));
  v3 B = normalize(cross(N, T));
  return add(add(muls(T, v.x), muls(B, v.y)), muls(N, v.z));
}

__device__ v3 sample_brdf(float xi1, float xi2, float xi3, v3 V, v3 N, const Mat& m) {  // :753-784
  float rd = 1.0f - m.metallic, rs = 1.0f, rc = 0.25f * m.clearcoat;
  float rsum = (rd + rs) + rc;
  float pdiff = rd / rsum, pspec = rs / rsum;
  if (xi3 <= pdiff) {  // SampleCosineHemisphere :699-710
    float r = f_sqrt(xi1);
    float th = (xi2 * 2.0f) * PT_PI;
    float x = r * g_cos(th), y = r * g_sin(th);
    float z = f_sqrt((1.0f - x * x) - y * y);
    return to_hemi(mk(x, y, z), N);
  }
  bool spec = (pdiff < xi3 && xi3 <= pdiff + pspec);
  bool coat = (pdiff + pspec < xi3);
  if (!spec && !coat) return mk(0, 1, 0);
  float phi = (2.0f * PT_PI) * xi1;
  float sp = g_sin(phi), cp = g_cos(phi);
  float ct;
  if (spec) {  // SampleGTR2 :713-730
    float a = f_max(0.001f, sqr(m.roughness));
    ct = f_sqrt((1.0f - xi2) / (1.0f + (a * a - 1.0f) * xi2));
  } else {  // SampleGTR1 :733-750
    float a = f_mix(0.1f, 0.001f, m.clearcoatGloss);
    ct = f_sqrt((1.0f - g_pow(a * a, 1.0f - xi2)) / (1.0f - a * a));
  }
  float st = f_sqrt(f_max(0.0f, 1.0f - ct * ct));
  v3 H = to_hemi(mk(st * cp, st * sp, ct), N);
  return reflect(neg(V), H);
}

// ------------------------------------------------------------- environment ---
__device__ __forceinline__ float4 tex_lin(const Tex& T, float u, float v) {
  Bilin b = bilin_setup(u, v, T.W, T.H);
  float4 c00 = T.p[(size_t)b.y0 * T.W + b.x0], c10 = T.p[(size_t)b.y0 * T.W + b.x1];
  float4 c01 = T.p[(size_t)b.y1 * T.W + b.x0], c11 = T.p[(size_t)b.y1 * T.W + b.x1];
  return f4(bilin_mix(b, c00.x, c10.x, c01.x, c11.x), bilin_mix(b, c00.y, c10.y, c01.y, c11.y),
            bilin_mix(b, c00.z, c10.z, c01.z, c11.z), 0.0f);
}
__device__ __forceinline__ void to_sph(v3 v, float* u, float* w) {  // :804-810
  float a = g_atan2(v.z, v.x), b = g_asin(v.y);
  a /= (2.0f * PT_PI);
  b /= PT_PI;
  a += 0.5f;
  b += 0.5f;
  *u = a;
  *w = 1.0f - b;
}
__device__ __forceinline__ v3 hdr_color(const PTParams& p, v3 L) {  // :813-817
  float u, v;
  to_sph(normalize(L), &u, &v);
  // the merged texture holds hdrMap's texels in .xyz: the same bits, and the environment is read from one array
  return xyz(tex_lin(p.hdr_pdf.p ? p.hdr_pdf : p.hdr, u, v));
}
__device__ __forceinline__ float hdr_pdf(const PTParams& p, v3 L) {  // :821-832
  float u, v;
  to_sph(normalize(L), &u, &v);
  float pdf = tex_lin(p.cache, u, v).z;
  float theta = PT_PI * (0.5f - v);
  float st = f_max(g_sin(theta), 1e-10f);
  float conv = (float)(p.hdrResolution * p.hdrResolution / 2) / (((2.0f * PT_PI) * PT_PI) * st);
  return pdf * conv;
}
// hdr_color(p, L) and hdr_pdf(p, L) of one direction: with the merged texture (PTParams::hdr_pdf) one bilinear fetch
// serves both — the same texels, weights and mixes as tex_lin on each texture, so the same bits.
__device__ __forceinline__ v3 hdr_color_pdf(const PTParams& p, v3 L, float* pdf) {
  if (!p.hdr_pdf.p) {
    *pdf = hdr_pdf(p, L);
    return hdr_color(p, L);
  }
  float u, v;
  to_sph(normalize(L), &u, &v);
  const Tex& T = p.hdr_pdf;
  Bilin b = bilin_setup(u, v, T.W, T.H);
  float4 c00 = T.p[(size_t)b.y0 * T.W + b.x0], c10 = T.p[(size_t)b.y0 * T.W + b.x1];
  float4 c01 = T.p[(size_t)b.y1 * T.W + b.x0], c11 = T.p[(size_t)b.y1 * T.W + b.x1];
  const float theta = PT_PI * (0.5f - v);
  const float st = f_max(g_sin(theta), 1e-10f);
  const float conv = (float)(p.hdrResolution * p.hdrResolution / 2) / (((2.0f * PT_PI) * PT_PI) * st);
  *pdf = bilin_mix(b, c00.w, c10.w, c01.w, c11.w) * conv;
  return mk(bilin_mix(b, c00.x, c10.x, c01.x, c11.x), bilin_mix(b, c00.y, c10.y, c01.y, c11.y),
            bilin_mix(b, c00.z, c10.z, c01.z, c11.z));
}
__device__ __forceinline__ v3 sample_hdr(const PTParams& p, float xi1, float xi2) {  // :787-799
  float4 c = tex_lin(p.cache, xi1, xi2);
  float yy = 1.0f - c.y;
  float phi = (2.0f * PT_PI) * (c.x - 0.5f);
  float th = PT_PI * (yy - 0.5f);
  return mk(g_cos(th) * g_cos(phi), g_sin(th), g_cos(th) * g_sin(phi));
}

}  // namespace ptk

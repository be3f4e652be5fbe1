// kernels_pt.hip — per-pixel path tracer with next-event estimation and the
// ray-cast G-buffer, for gfx950 (wave64, no RT hardware: traversal is VALU).
//
// Behaviour restated from shaders/path_tracing.frag (file:line cited per
// function). Engineering differences from the GLSL, all result-preserving:
//  * scene decoded once at bind time into float4 SoA records (pt_device.h) —
//    one 64-B node fetch tests both children, one 64-B record per triangle test;
//  * short traversal stack in LDS (column layout: conflict-free), near child
//    visited first exactly as hitBVH's push order (:407-420);
//  * closest-hit rays prune boxes whose entry lies beyond the current hit
//    (with a safety margin; the reference visits every intersected box, which
//    can only change the result through its strict '<' tie rule — a pruned box
//    holds no triangle nearer than the current hit);
//  * shadow rays are any-hit: the HDR test only asks isHit (:934), the point
//    test asks whether the closest hit is nearer than the light (:905-909);
//  * material/normal of the closest hit are decoded once after traversal (the
//    reference decodes per leaf; the values are a function of the triangle and
//    the hit point only).
// Built with -ffp-contract=off and the shared GLSL built-ins: the CPU oracle's
// restatement of the same shader reproduces these outputs bit for bit.
#include <hip/hip_runtime.h>

#include "glsl_builtins.h"
#include "pt_device.h"

using namespace glsl;

namespace ptk {

#define PT_PI 3.1415926f
#define PT_INF 114514.0f

__device__ __forceinline__ int prow(const Plane& P, int y) {
  int ly = y - P.row0;
  return ly < 0 ? 0 : (ly >= P.rows ? P.rows - 1 : ly);
}
__device__ __forceinline__ float4 pld(const Plane& P, int x, int y) { return P.p[(size_t)prow(P, y) * P.W + x]; }
__device__ __forceinline__ void pst(const Plane& P, int x, int y, float4 v) { P.p[(size_t)prow(P, y) * P.W + x] = v; }
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
__device__ __forceinline__ bool tri_hit(const float4* __restrict__ g, int i, v3 S, v3 d, float* t_out) {
  float4 a = g[4 * i], b = g[4 * i + 1], c = g[4 * i + 2], n = g[4 * i + 3];
  v3 p1 = xyz(a), p2 = xyz(b), p3 = xyz(c), N = xyz(n);
  float dn = dot(N, d);
  if (f_abs(dn) < 0.00001f) return false;
  float t = (a.w - dot(S, N)) / dn;
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

__device__ __forceinline__ int ref_leaf_first(int ref) { return (-(ref + 1)) >> 4; }
__device__ __forceinline__ int ref_leaf_count(int ref) { return (-(ref + 1)) & 15; }

// mode 0: closest hit (hitBVH :372-424); mode 1: any hit (HDR shadow);
// mode 2: any hit nearer than `maxd` by length(P - S) (point-light shadow).
template <int MODE>
__device__ int traverse(const SceneDev& sc, int* __restrict__ stk, v3 S, v3 d, float maxd, int prune,
                        float* t_best_out) {
  v3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  float tbest = PT_INF;
  int best = -1;
  int sp = 0;
  int node = sc.root_ref;
  const int lane = threadIdx.x;
  while (true) {
    if (node >= 0) {
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
        int nearc = (dl < dr) ? cl : cr;
        int farc = (dl < dr) ? cr : cl;
        stk[sp * kBlock + lane] = farc;
        ++sp;
        node = nearc;
      } else if (hl) {
        node = cl;
      } else if (hr) {
        node = cr;
      } else {
        if (sp == 0) break;
        --sp;
        node = stk[sp * kBlock + lane];
      }
    } else {
      int first = ref_leaf_first(node), cnt = ref_leaf_count(node);
      for (int i = first; i < first + cnt; ++i) {
        float t;
        if (!tri_hit(sc.tri_geom, i, S, d, &t)) continue;
        if (MODE == 0) {
          if (t < tbest) { tbest = t; best = i; }
        } else if (MODE == 1) {
          if (t < PT_INF) { *t_best_out = t; return i; }
        } else {
          if (t < PT_INF) {
            float sd = length(sub(add(S, muls(d, t)), S));
            if (sd < maxd) { *t_best_out = t; return i; }
          }
        }
      }
      if (sp == 0) break;
      --sp;
      node = stk[sp * kBlock + lane];
    }
  }
  *t_best_out = tbest;
  return best;
}

struct Hit {
  bool isHit;
  v3 P, normal, viewDir;
  Mat m;
};

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
  // texture-array branch (:331-364): no material array bound -> the fetch reads 0
  if (h.m.baseColor.x < 0.0f || h.m.baseColor.y < 0.0f || h.m.baseColor.z < 0.0f) h.m.baseColor = splat(0.0f);
  if (h.m.metallic < 0.0f) h.m.metallic = 0.0f;
  if (h.m.roughness < 0.0f) h.m.roughness = 0.0f;
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
  return xyz(tex_lin(p.hdr, u, v));
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
__device__ __forceinline__ v3 sample_hdr(const PTParams& p, float xi1, float xi2) {  // :787-799
  float4 c = tex_lin(p.cache, xi1, xi2);
  float yy = 1.0f - c.y;
  float phi = (2.0f * PT_PI) * (c.x - 0.5f);
  float th = PT_PI * (yy - 0.5f);
  return mk(g_cos(th) * g_cos(phi), g_sin(th), g_cos(th) * g_sin(phi));
}

// ------------------------------------------------------------ path tracer ---
__global__ void __launch_bounds__(kBlock) pathtrace_kernel(PTParams p) {
  __shared__ int stk[kStack * kBlock];
  int* s = stk;
  // 16x16 pixel tile per block; each wave owns an 8x8 sub-tile (ray coherence).
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  const int x = blockIdx.x * 16 + (wv & 1) * 8 + (ln & 7);
  const int y = p.y0 + blockIdx.y * 16 + (wv >> 1) * 8 + (ln >> 3);
  if (x >= p.W || y >= p.y1) return;

  uint32_t seed = ((uint32_t)x * 1973u + (uint32_t)y * 9277u + p.frameCounter * 26699u) | 1u;  // :433-436
  wang_hash(&seed);  // AA jitter rand() x2 (:1060), never applied
  wang_hash(&seed);
  // Cranley-Patterson shift (:497-515): per-pixel constant
  uint32_t ps = ((uint32_t)x * 1973u + (uint32_t)y * 9277u + (uint32_t)(114514 / 1919) * 26699u) | 1u;
  float cpu = u32_to_unit(wang_hash(&ps));
  float cpv = u32_to_unit(wang_hash(&ps));

  float pixx = (float)(2 * x + 1) / (float)p.W - 1.0f;
  float pixy = (float)(2 * y + 1) / (float)p.H - 1.0f;
  if (p.aspect_corrected) pixx = pixx * ((float)p.W / (float)p.H);
  const float* m = p.camRot;
  v3 S = mk(p.eye[0], p.eye[1], p.eye[2]);
  v3 d = normalize(mk((m[0] * pixx + m[4] * pixy) + (m[8] * -1.0f + m[12] * 0.0f),
                      (m[1] * pixx + m[5] * pixy) + (m[9] * -1.0f + m[13] * 0.0f),
                      (m[2] * pixx + m[6] * pixy) + (m[10] * -1.0f + m[14] * 0.0f)));
  v3 light = splat(0.0f), red = splat(1.0f);
  v3 firstE = splat(0.0f), firstA = splat(0.0f);

  for (int i = 0; i < p.max_depth; ++i) {
    float t;
    int tri = traverse<0>(p.scene, s, S, d, 0.0f, p.prune, &t);
    if (tri < 0) {
      light = add(light, mul(hdr_color(p, d), red));
      break;
    }
    Hit h = decode_hit(p.scene, tri, t, S, d);
    if (i == 0) { firstE = h.m.emissive; firstA = h.m.baseColor; }
    float xi1 = p.sobol_u[i] + cpu;
    if (xi1 > 1.0f) xi1 -= 1.0f;
    if (xi1 < 0.0f) xi1 += 1.0f;
    float xi2 = p.sobol_v[i] + cpv;
    if (xi2 > 1.0f) xi2 -= 1.0f;
    if (xi2 < 0.0f) xi2 += 1.0f;
    float xi3 = u32_to_unit(wang_hash(&seed));
    v3 V = neg(h.viewDir);
    v3 L = sample_brdf(xi1, xi2, xi3, V, h.normal, h.m);
    if (dot(h.normal, L) <= 0.0f) break;

    // shade (:948-968)
    v3 brdf = brdf_eval(V, h.normal, L, h.m);
    float bpdf = brdf_pdf(V, h.normal, L, h.m);
    // hdriLight (:922-946)
    float r1 = u32_to_unit(wang_hash(&seed));
    float r2 = u32_to_unit(wang_hash(&seed));
    v3 hd = sample_hdr(p, r1, r2);
    float hpdf = 0.0f;
    v3 hcalc = splat(0.0f);
    {
      float ts;
      if (traverse<1>(p.scene, s, h.P, hd, 0.0f, 0, &ts) < 0) {
        v3 hv = hdr_color(p, hd);
        v3 hb = brdf_eval(V, h.normal, hd, h.m);
        hpdf = hdr_pdf(p, hd);
        hcalc = divs(mul(muls(hb, f_abs(dot(hd, h.normal))), hv), hpdf);
      }
    }
    // calculatePointLight (:884-919)
    float ppdf = 0.0f;
    v3 pcalc = splat(0.0f);
    if (p.pointLightSize != 0) {
      ppdf = (2.0f * PT_PI) / (float)p.pointLightSize;
      int li = (int)(u32_to_unit(wang_hash(&seed)) * (float)p.pointLightSize);
      v3 lpos = splat(0.0f), lrad = splat(0.0f);
      if (li >= 0 && li < p.scene.nlights_buf) {  // out-of-range texelFetch reads 0
        const float* lp = p.scene.lights + 6 * li;
        lpos = mk(lp[0], lp[1], lp[2]);
        lrad = mk(lp[3], lp[4], lp[5]);
      }
      v3 ld = normalize(sub(lpos, h.P));
      float dist = length(sub(lpos, h.P));
      float ts;
      if (traverse<2>(p.scene, s, h.P, ld, dist, 0, &ts) < 0) {
        v3 plv = divs(lrad, dist * dist);
        v3 pb = brdf_eval(V, h.normal, ld, h.m);
        pcalc = divs(muls(mul(plv, pb), f_abs(dot(ld, h.normal))), ppdf);
      }
    }
    v3 cosb = muls(brdf, f_abs(dot(L, h.normal)));
    v3 bcalc = divs(mul(h.m.emissive, cosb), bpdf);
    float sw = ((hpdf + ppdf) + bpdf) + 1e-6f;
    float w1 = hpdf / sw, w2 = ppdf / sw, w3 = bpdf / sw;
    v3 hitLight = mul(red, add(add(muls(hcalc, w1), muls(pcalc, w2)), muls(bcalc, w3)));
    red = mul(red, divs(cosb, bpdf));
    light = add(light, hitLight);
    S = h.P;
    d = L;
  }
  light = vclamp(light, 0.0f, p.clamp_threshold);
  v3 color = splat(0.0f);
  if (!f_isnan(light.x) && !f_isnan(light.y) && !f_isnan(light.z)) color = light;
  if (p.accumulate && p.last.p) {  // :1116-1119
    float4 lc = pld(p.last, x, y);
    color = mixv(xyz(lc), color, 1.0f / (float)(p.frameCounter + 1u));
  }
  pst(p.color, x, y, f4(color.x, color.y, color.z, 1.0f));
  pst(p.emission, x, y, f4(firstE.x, firstE.y, firstE.z, 1.0f));
  pst(p.albedo, x, y, f4(firstA.x, firstA.y, firstA.z, 1.0f));
}

// --------------------------------------------------------------- G-buffer ---
struct MTr {
  float t, u, v;
  bool ok;
};
__device__ __forceinline__ MTr moller(v3 p1, v3 e1, v3 e2, v3 o, v3 d, bool bounds) {
  MTr r;
  r.ok = false;
  r.t = r.u = r.v = 0.0f;
  v3 pvec = cross(d, e2);
  float det = dot(e1, pvec);
  if (det > -1e-12f && det < 1e-12f) return r;
  float inv = 1.0f / det;
  v3 tvec = sub(o, p1);
  r.u = dot(tvec, pvec) * inv;
  v3 qvec = cross(tvec, e1);
  r.v = dot(d, qvec) * inv;
  r.t = dot(e2, qvec) * inv;
  if (bounds) {
    if (r.u < 0.0f || r.u > 1.0f) return r;
    if (r.v < 0.0f || r.u + r.v > 1.0f) return r;
    if (!(r.t > 0.0f)) return r;
  }
  r.ok = true;
  return r;
}
__device__ __forceinline__ bool gb_box(v3 o, v3 inv, float ax, float ay, float az, float bx, float by, float bz,
                                       float lim, float* t0o) {
  // NaN slabs (0 * inf) leave the interval unchanged, as in the oracle's test
  float t0 = 0.0f, t1 = lim;
  const float lo[3] = {ax, ay, az}, hi[3] = {bx, by, bz}, oo[3] = {o.x, o.y, o.z}, ii[3] = {inv.x, inv.y, inv.z};
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    float ta = (lo[a] - oo[a]) * ii[a], tb = (hi[a] - oo[a]) * ii[a];
    if (ta > tb) { float tt = ta; ta = tb; tb = tt; }
    ta -= 1e-4f * (f_abs(ta) + 1.0f);
    tb += 1e-4f * (f_abs(tb) + 1.0f);
    t0 = ta > t0 ? ta : t0;
    t1 = tb < t1 ? tb : t1;
  }
  *t0o = t0;
  return t0 <= t1;
}
__device__ __forceinline__ v3 gb_dir(const GBufParams& p, int x, int y) {
  float px = (float)(2 * x + 1) / (float)p.W - 1.0f;
  float py = (float)(2 * y + 1) / (float)p.H - 1.0f;
  float dc0 = px / p.P00, dc1 = py / p.P11, dc2 = -1.0f;
  const float* R = p.invR;
  return mk((R[0] * dc0 + R[1] * dc1) + R[2] * dc2, (R[3] * dc0 + R[4] * dc1) + R[5] * dc2,
            (R[6] * dc0 + R[7] * dc1) + R[8] * dc2);
}
__device__ __forceinline__ void mat_vec4(const float* m, v3 P, float* o) {
  for (int r = 0; r < 4; ++r) o[r] = (m[r] * P.x + m[4 + r] * P.y) + (m[8 + r] * P.z + m[12 + r] * 1.0f);
}
__device__ __forceinline__ float lin_z(const GBufParams& p, v3 P) {
  float c[4];
  mat_vec4(p.M, P, c);
  float zw = (c[2] / c[3]) * 0.5f + 0.5f;
  float fw = 1.0f / c[3];
  return zw / fw;
}

__global__ void __launch_bounds__(kBlock) gbuffer_kernel(GBufParams p) {
  __shared__ int stk[kStack * kBlock];
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  const int x = blockIdx.x * 16 + (wv & 1) * 8 + (ln & 7);
  const int y = p.y0 + blockIdx.y * 16 + (wv >> 1) * 8 + (ln >> 3);
  if (x >= p.W || y >= p.y1) return;
  v3 o = mk(p.eye[0], p.eye[1], p.eye[2]);
  v3 d = gb_dir(p, x, y);
  v3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  float best = 3.0e38f;
  int besti = -1, bests = -1;
  float bu = 0.f, bv = 0.f;
  int sp = 0, node = p.root_ref;
  while (true) {
    if (node >= 0) {
      const float4* nd = p.bvh + 4 * node;
      float4 q0 = nd[0], q1 = nd[1], q2 = nd[2], q3 = nd[3];
      // conservative (widened) slab test: the box only culls, Moller-Trumbore decides
      float lim = best * 1.0002f + 2.0e-4f;
      float t0l, t0r;
      bool hl = gb_box(o, inv, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, lim, &t0l);
      bool hr = gb_box(o, inv, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, lim, &t0r);
      int cl = __float_as_int(q3.x), cr = __float_as_int(q3.y);
      if (hl && hr) {
        int nearc = (t0l < t0r) ? cl : cr, farc = (t0l < t0r) ? cr : cl;
        stk[sp * kBlock + threadIdx.x] = farc;
        ++sp;
        node = nearc;
      } else if (hl) node = cl;
      else if (hr) node = cr;
      else {
        if (sp == 0) break;
        --sp;
        node = stk[sp * kBlock + threadIdx.x];
      }
    } else {
      int first = ref_leaf_first(node), cnt = ref_leaf_count(node);
      for (int i = first; i < first + cnt; ++i) {
        const float4* g = p.geom + 7 * i;
        float4 a = g[0], e1 = g[1], e2 = g[2], ng = g[3];
        v3 p1 = xyz(a);
        if (!(dot(xyz(ng), sub(p1, o)) < 0.0f)) continue;  // back face culled (GL_BACK, CCW front)
        MTr h = moller(p1, xyz(e1), xyz(e2), o, d, true);
        if (!h.ok) continue;
        int oi = __float_as_int(a.w);
        if (h.t < best || (h.t == best && oi < besti)) {
          best = h.t;
          besti = oi;
          bests = i;
          bu = h.u;
          bv = h.v;
        }
      }
      if (sp == 0) break;
      --sp;
      node = stk[sp * kBlock + threadIdx.x];
    }
  }
  if (bests < 0) {
    float4 bg = f4(0.2f, 0.3f, 0.3f, 1.0f);  // glClearColor (main.cpp:62)
    pst(p.world, x, y, bg);
    pst(p.normal_depth, x, y, bg);
    pst(p.motion, x, y, bg);
    pst(p.fwidth, x, y, bg);
    if (p.fwidth_aux) p.fwidth_aux[(size_t)prow(p.fwidth, y) * p.W + x] = 0.3f;
    return;
  }
  const float4* g = p.geom + 7 * bests;
  v3 p1 = xyz(g[0]), e1 = xyz(g[1]), e2 = xyz(g[2]);
  v3 n1 = xyz(g[4]), n2 = xyz(g[5]), n3 = xyz(g[6]);
  auto interp = [&](float u, float v) {
    float w0 = (1.0f - u) - v;
    return add(add(muls(n1, w0), muls(n2, u)), muls(n3, v));
  };
  v3 P = add(o, muls(d, best));
  v3 N = interp(bu, bv);
  float lz = lin_z(p, P);
  float c[4], pc[4];
  mat_vec4(p.M, P, c);
  mat_vec4(p.PV, P, pc);
  float nowx = (c[0] / c[3]) * 0.5f + 0.5f, nowy = (c[1] / c[3]) * 0.5f + 0.5f;
  float prex = (pc[0] / pc[3]) * 0.5f + 0.5f, prey = (pc[1] / pc[3]) * 0.5f + 0.5f;
  v3 dx = gb_dir(p, x ^ 1, y), dy = gb_dir(p, x, y ^ 1);
  MTr hx = moller(p1, e1, e2, o, dx, false), hy = moller(p1, e1, e2, o, dy, false);
  v3 Nx = interp(hx.u, hx.v), Ny = interp(hy.u, hy.v);
  float zx = lin_z(p, add(o, muls(dx, hx.t)));
  float zy = lin_z(p, add(o, muls(dy, hy.t)));
  v3 fwN = add(mk(f_abs(Nx.x - N.x), f_abs(Nx.y - N.y), f_abs(Nx.z - N.z)),
               mk(f_abs(Ny.x - N.x), f_abs(Ny.y - N.y), f_abs(Ny.z - N.z)));
  float fwz = f_max(f_abs(zx - lz), f_abs(zy - lz));
  pst(p.world, x, y, f4(P.x, P.y, P.z, 1.0f));
  pst(p.normal_depth, x, y, f4(N.x, N.y, N.z, lz));
  pst(p.motion, x, y, f4(nowx - prex, nowy - prey, 0.0f, 1.0f));
  pst(p.fwidth, x, y, f4(length(fwN), fwz, lz, 1.0f));
  if (p.fwidth_aux) p.fwidth_aux[(size_t)prow(p.fwidth, y) * p.W + x] = fwz;
}

int launch_pathtrace(const PTParams& p, hipStream_t s) {
  if (p.y1 <= p.y0) return 0;
  dim3 grid((p.W + 15) / 16, (p.y1 - p.y0 + 15) / 16);
  hipLaunchKernelGGL(pathtrace_kernel, grid, dim3(kBlock), 0, s, p);
  return (int)hipGetLastError();
}
int launch_gbuffer(const GBufParams& p, hipStream_t s) {
  if (p.y1 <= p.y0) return 0;
  dim3 grid((p.W + 15) / 16, (p.y1 - p.y0 + 15) / 16);
  hipLaunchKernelGGL(gbuffer_kernel, grid, dim3(kBlock), 0, s, p);
  return (int)hipGetLastError();
}

}  // namespace ptk

// capi.hip — implementation of include/ptsvgf.h: the GL-plumbing-shaped C ABI
// (Utils/render_pass.h:82-182, Utils/shader.h:21-67, Utils/help_func.h:22-32)
// over HIP device memory and the gfx950 kernels.
//
// GL semantics kept:
//  * RenderPass uniforms are set by name; an unknown name is silently ignored;
//  * set_texture_uniform binds to the pass's next texture slot; a sampler that
//    was never bound reads texture unit 0, i.e. the texture most recently bound
//    to slot 0 by any pass (GL's global unit state);
//  * draw() is ordered after every previous draw (one in-order HIP stream);
//  * scene texture buffers are decoded once per (buffer, version) into the
//    kernels' SoA records (pt_device.h) on first use, like a driver upload.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <algorithm>
#include <array>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/ptsvgf.h"
#include "../../include/ptsvgf_scene.h"
#include "glsl_builtins.h"
#include "pt_device.h"

namespace {

using namespace ptk;

enum ProgKind {
  PK_PATHTRACE = 1,
  PK_REPROJECT,
  PK_VARIANCE,
  PK_ATROUS,
  PK_MODULATE,
  PK_BLIT,
  PK_SAVE,
  PK_OUTPUT,
  PK_TAA,
  PK_RASTER
};

struct Texture {
  uint32_t target = PT_TEXTURE_2D;
  int W = 0, H = 0;      // logical (global) size
  int row0 = 0, rows = 0;  // stored rows (band)
  int layers = 0;
  bool owned = true;
  void* dev = nullptr;
  size_t bytes = 0;
  std::vector<uint8_t> host;  // buffers: host copy for decoding
  uint64_t version = 1;
  float* aux = nullptr;  // compact depth-fwidth side plane
  bool aux_valid = false;
  unsigned char* tflags = nullptr;  // a-trous per-tile surface flags derived from aux (atrous_tile_flags)
  size_t tflags_cap = 0;
  uint64_t tflags_ver = 0;          // texture version / rows they were derived for
  int tflags_y0 = 0, tflags_y1 = -1;
  bool lbvh = false;     // written by pt_bvh_build (the device copy is authoritative: get_scene decodes it there)
};

struct Uniform {
  int type = 0;  // 1 float 2 int 3 uint 4 bool 5 vec3 6 mat4
  float f[16] = {0};
  int i = 0;
  uint32_t u = 0;
};

struct RasterScene {
  float4* geom = nullptr;
  float4* nrm = nullptr;
  float4* bvh = nullptr;
  int root_ref = 0;
  int stack_need = 0;
  int ntris = 0;
};

// Scratch of the tile-binned G-buffer (launch_gbuffer_raster), per rasterize pass, sized by its triangles and band.
struct RasterBins {
  void* base = nullptr;
  int ntris = 0, ntiles = 0, pair_cap = 0, big_cap = 0;
  int4* tri_box = nullptr;
  float* tri_tmin = nullptr;
  int *tile_count = nullptr, *tile_off = nullptr, *pairs = nullptr, *big = nullptr, *ctr = nullptr;
};

struct WFBuffers {
  void* base = nullptr;  // one allocation carved into the WFState arrays
  size_t n = 0;          // pixels per frame
  int nb = 1;            // frames (pt_pass_draw_batch): per-pixel arrays for nb * n pixels, lists and counters per frame
  WFState stb[kMaxBatch]{};  // frame b's state: per-pixel arrays at pid offset b * n; stb[0] == st
  WFState st{};
  int* spill = nullptr;  // deep reference trees: stack entries past the LDS stack (WFState::spill)
  int spill_levels = 0;
  size_t spill_cols = 0;
};

// Spill columns for a tree needing `need` stack entries (> the LDS stack): (need - kSpillKS + 1) entries per
// pixel of the band, allocated on first use and kept while the depth fits.
int wf_spill(WFBuffers& b, int need) {
  const int levels = need - kSpillKS + 1;
  const size_t m = b.n * (size_t)b.nb;  // columns of the batch's pixels (global pids)
  if (levels <= 0) {
    for (int f = 0; f < b.nb; ++f) {
      b.stb[f].spill = nullptr;
      b.stb[f].spill_stride = 0;
    }
    b.st = b.stb[0];
    return PT_OK;
  }
  if (!b.spill || b.spill_levels < levels || b.spill_cols != m) {
    if (b.spill) (void)hipFree(b.spill);
    b.spill = nullptr;
    if (hipMalloc((void**)&b.spill, (size_t)levels * m * sizeof(int)) != hipSuccess) return PT_ERR_HIP;
    b.spill_levels = levels;
    b.spill_cols = m;
  }
  for (int f = 0; f < b.nb; ++f) {  // frame f's local pid p is column f * n + p
    b.stb[f].spill = b.spill + (size_t)f * b.n;
    b.stb[f].spill_stride = m;
  }
  b.st = b.stb[0];
  return PT_OK;
}

int wf_alloc(WFBuffers& b, int W, int rows, int nb = 1) {
  const size_t n = (size_t)W * (size_t)rows;
  if (b.base && b.n == n && b.nb == nb) return PT_OK;
  if (b.base) { (void)hipFree(b.base); b.base = nullptr; }
  const size_t m = n * (size_t)nb;  // pixels of the batch
  const size_t f4 = m * 16, al = 256;
  const size_t nl = (size_t)wf_list_capacity(W, rows) * 8;  // 8 list segments
  auto up = [&](size_t v) { return (v + al - 1) / al * al; };
  const size_t lists = up(nl * 4 * kLiveBins) * 2 + up(nl * 4 * (1 + kPointBins));
  size_t total = up(f4) * 10 + up(m * 8) + up(m * 4) + up(m) * 2 + lists * nb + up(m * 8) + up(m * 4) +
                 up((size_t)nb * kWfCounters * 4);
  if (hipMalloc(&b.base, total) != hipSuccess) { b.base = nullptr; return PT_ERR_HIP; }
  char* c = (char*)b.base;
  WFState s0{};
  float4** f4p[10] = {&s0.ray_o, &s0.ray_d, &s0.light, &s0.red, &s0.pend0,
                      &s0.pend1, &s0.pend2, &s0.pend3, &s0.sh_h, &s0.sh_p};
  for (auto q : f4p) { *q = (float4*)c; c += up(f4); }
  s0.hit = (int2*)c; c += up(m * 8);
  s0.seed = (uint32_t*)c; c += up(m * 4);
  s0.occ_h = (uint8_t*)c; c += up(m);
  s0.occ_p = (uint8_t*)c; c += up(m);
  s0.straggler = (int*)c; c += up(m * 8);  // both shadow kinds of one bounce (a batch's: frame 0's pointer)
  s0.strag_c = (int*)c; c += up(m * 4);    // bounce rays of one bounce
  int* counters = (int*)c; c += up((size_t)nb * kWfCounters * 4);  // contiguous: one memset per draw
  for (int f = 0; f < nb; ++f) {
    WFState st = s0;
    const size_t o = (size_t)f * n;
    st.ray_o = s0.ray_o + o;
    st.ray_d = s0.ray_d + o;
    st.light = s0.light + o;
    st.red = s0.red + o;
    st.pend0 = s0.pend0 + o;
    st.pend1 = s0.pend1 + o;
    st.pend2 = s0.pend2 + o;
    st.pend3 = s0.pend3 + o;
    st.sh_h = s0.sh_h + o;
    st.sh_p = s0.sh_p + o;
    st.hit = s0.hit + o;
    st.seed = s0.seed + o;
    st.occ_h = s0.occ_h + o;
    st.occ_p = s0.occ_p + o;
    st.straggler = s0.straggler + 2 * o;
    st.strag_c = s0.strag_c + o;
    st.counters = counters + (size_t)f * kWfCounters;
    st.list0 = (int*)c; c += up(nl * 4 * kLiveBins);
    st.list1 = (int*)c; c += up(nl * 4 * kLiveBins);
    st.shadow_list = (int*)c; c += up(nl * 4 * (1 + kPointBins));
    b.stb[f] = st;
  }
  b.st = b.stb[0];
  b.n = n;
  b.nb = nb;
  return PT_OK;
}

// Cost-ordered tile dispatch state of one traversal pass (TileSched, pt_device.h).
struct TileOrder {
  uint32_t* cost = nullptr;  // per-tile cost recorded by the current launch
  int* perm = nullptr;       // dispatch order computed from the previous launch
  int n = 0;
  bool ordered = false;      // perm holds a valid order for n tiles
};

struct Pass {
  uint32_t program = 0;
  WFBuffers wf;
  TileOrder order;
  int W = 0, H = 0;
  std::vector<uint32_t> att;
  bool bound = false, final_pass = false;
  int slot = 0;
  std::unordered_map<std::string, uint32_t> tex;
  std::unordered_map<std::string, Uniform> uni;
  int y_begin = -1, y_end = -1;
  RasterScene raster;
  uint32_t raster_src = 0;  // pt_raster_pass_share: draw this rasterize pass's triangles and tree instead
  RasterBins bins;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool timed = false;
  uint32_t* row_cost = nullptr;  // pt_pass_set_row_cost (not owned)
  uint32_t* motion_max = nullptr;  // pt_pass_set_motion_bound (not owned)
  struct HdrMerged* hdr_reads = nullptr;  // the merged environment the draw being issued reads (pt_params)
  unsigned long long* stats = nullptr;  // pt_pass_set_trace_stats (not owned)
  int stats_n = 0;                      // counters that buffer holds (pt_pass_set_trace_stats_n)
};

struct SceneGPU {
  float4* geom = nullptr;
  float4* shade = nullptr;
  float4* bvh = nullptr;
  float4* bvh4 = nullptr;
  float4* bvh_any = nullptr;  // any-hit tree over the reference leaves (build_anyhit_tree)
  float4* leaves = nullptr;   // the reference leaves: (box lo, leaf ref bits), (box hi, 0) (wf_primary_raster)
  int nleaves = 0;
  int root_any = 0, need_any = 0;
  bool has4 = false;  // bvh4: the 4-wide form of bvh_any (pack_wide)
  bool nan4 = false;  // a child box of bvh4 has a NaN coordinate (PT_WIDE_SIGNED walks need lo <= hi: not walked)
  int root4 = 0, need4 = 0, root4c = 0;  // root4c: the closest-hit walks' root (SceneDev::root4c)
  // refine_leaves' fine boxes are padded for rays whose origin lies within kFineEyeReach x the scene's largest vertex
  // coordinate; an eye further out (pt_params) walks the reference tree instead
  float fine_eye_limit = INFINITY;
  int stack_need = 0;
  int root_ref = 0;
  int ntris = 0;
  uint64_t tri_ver = 0, node_ver = 0;
};

// The environment map with its importance cache's pdf channel beside it (PTParams::hdr_pdf): built on the device
// when a path-tracing draw binds an hdrMap and an hdrCache of one size, rebuilt when either changes (versions), freed
// with either texture.
struct HdrMerged {
  float4* buf = nullptr;
  const void *hdr_dev = nullptr, *cache_dev = nullptr;
  uint64_t vh = 0, vc = 0;
  int W = 0, H = 0;
  hipEvent_t built = nullptr;                  // recorded after the merge that wrote buf, on the stream that ran it
  std::map<hipStream_t, hipEvent_t> uses;      // per draw stream: recorded after its latest draw that read buf
  // buffers a rebuild retired, each with its readers' events: reused (never freed mid-run, so no call blocks the
  // device) once every event has completed
  std::vector<std::pair<float4*, std::vector<hipEvent_t>>> spare;
};

// drops a merged environment: its buffers (the caller has synchronised the streams that read them) and events
void free_hdr_merged(HdrMerged& m) {
  if (m.buf) (void)hipFree(m.buf);
  for (auto& sp : m.spare) {
    (void)hipFree(sp.first);
    for (hipEvent_t e : sp.second) (void)hipEventDestroy(e);
  }
  for (auto& u : m.uses) (void)hipEventDestroy(u.second);
  if (m.built) (void)hipEventDestroy(m.built);
  m = HdrMerged{};
}

struct Lib {
  bool init = false;
  int device = 0;
  hipStream_t own = nullptr, stream = nullptr;
  uint32_t next = 1;
  std::map<uint32_t, int> programs;
  std::map<uint32_t, std::unique_ptr<Texture>> textures;
  std::map<uint32_t, std::unique_ptr<Pass>> passes;
  std::map<std::pair<uint32_t, uint32_t>, SceneGPU> scenes;
  std::map<std::pair<uint32_t, uint32_t>, HdrMerged> hdr_merged;  // keyed by (hdrMap, hdrCache) handles
  std::map<hipStream_t, ptk::WfFork> forks;  // per draw stream: the path tracer's side stream (uniform trace_fork)
  uint32_t unit0 = 0;  // GL texture unit 0 binding (global)
  int band_w = 0, band_h = 0, band_y0 = 0, band_y1 = 0, band_row0 = 0, band_rows = 0;
  bool profiling = false;
};

Lib g;
thread_local std::string g_err;
std::recursive_mutex g_mu;

int err(int code, const std::string& m) {
  g_err = m;
  return code;
}
int hip_err(hipError_t e, const char* what) {
  return err(PT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}
#define HIPCHK(x)                                    \
  do {                                               \
    hipError_t e_ = (x);                             \
    if (e_ != hipSuccess) return hip_err(e_, #x);    \
  } while (0)

std::string basename_of(const char* p) {
  std::string s(p ? p : "");
  size_t k = s.find_last_of("/\\");
  return k == std::string::npos ? s : s.substr(k + 1);
}

Texture* tex_of(uint32_t h) {
  auto it = g.textures.find(h);
  return it == g.textures.end() ? nullptr : it->second.get();
}
Pass* pass_of(uint32_t h) {
  auto it = g.passes.find(h);
  return it == g.passes.end() ? nullptr : it->second.get();
}

int ensure_init() {
  if (g.init) return PT_OK;
  return err(PT_ERR_STATE, "pt_init() has not been called");
}

// ---------------------------------------------------------------- packing ---
struct NodeRaw {
  int left, right, n, index;
  float AA[3], BB[3];
};

constexpr int kRefStack = 256;  // path_tracing.frag:378

// *need: deepest interior level (root = 1) = the most stack entries a walk holds
int pack_bvh(const float* node_enc, int nnodes, std::vector<float4>& out, int* root_ref, int ntris, int* need) {
  if (nnodes < 2) return err(PT_ERR_FORMAT, "BVH needs the dummy node 0 and a root node 1");
  std::vector<NodeRaw> nd(nnodes);
  for (int i = 0; i < nnodes; ++i) {
    const float* f = node_enc + (size_t)i * 12;
    nd[i].left = (int)f[0];
    nd[i].right = (int)f[1];
    nd[i].n = (int)f[3];
    nd[i].index = (int)f[4];
    for (int k = 0; k < 3; ++k) { nd[i].AA[k] = f[6 + k]; nd[i].BB[k] = f[9 + k]; }
  }
  std::vector<int> idx(nnodes, -1);
  std::vector<int> order;
  // iterative DFS (depth check: stack needs one slot per interior level)
  struct Item { int id, depth; };
  std::vector<Item> st;
  auto leaf_ref = [&](int id, int* ref) -> int {
    const NodeRaw& n = nd[id];
    if (n.n > 15) return err(PT_ERR_FORMAT, "BVH leaf holds more than 15 triangles");
    if (n.index < 0 || n.index + n.n > ntris) return err(PT_ERR_FORMAT, "BVH leaf range out of bounds");
    *ref = -(n.index * 16 + n.n) - 1;
    return PT_OK;
  };
  *need = 0;
  if (nd[1].n > 0) {
    int r;
    if (leaf_ref(1, &r) != PT_OK) return PT_ERR_FORMAT;
    *root_ref = r;
    out.clear();
    return PT_OK;
  }
  st.push_back({1, 1});
  while (!st.empty()) {
    Item it = st.back();
    st.pop_back();
    // the reference walks with int stack[256] (path_tracing.frag:378); deeper trees are undefined there
    if (it.depth >= kRefStack) return err(PT_ERR_FORMAT, "BVH deeper than the reference's stack[256]");
    *need = std::max(*need, it.depth);
    idx[it.id] = (int)order.size();
    order.push_back(it.id);
    const NodeRaw& n = nd[it.id];
    if (n.left <= 0 || n.right <= 0 || n.left >= nnodes || n.right >= nnodes)
      return err(PT_ERR_FORMAT, "BVH interior node with an invalid child");
    if (nd[n.right].n <= 0) st.push_back({n.right, it.depth + 1});
    if (nd[n.left].n <= 0) st.push_back({n.left, it.depth + 1});
  }
  out.assign(order.size() * 4, float4{0, 0, 0, 0});
  for (size_t k = 0; k < order.size(); ++k) {
    const NodeRaw& n = nd[order[k]];
    const NodeRaw& L = nd[n.left];
    const NodeRaw& R = nd[n.right];
    int rl, rr;
    if (L.n > 0) { if (leaf_ref(n.left, &rl) != PT_OK) return PT_ERR_FORMAT; } else rl = idx[n.left];
    if (R.n > 0) { if (leaf_ref(n.right, &rr) != PT_OK) return PT_ERR_FORMAT; } else rr = idx[n.right];
    float4* q = &out[4 * k];
    q[0] = float4{L.AA[0], L.AA[1], L.AA[2], L.BB[0]};
    q[1] = float4{L.BB[1], L.BB[2], R.AA[0], R.AA[1]};
    q[2] = float4{R.AA[2], R.BB[0], R.BB[1], R.BB[2]};
    float a, b;
    memcpy(&a, &rl, 4);
    memcpy(&b, &rr, 4);
    q[3] = float4{a, b, 0, 0};
  }
  *root_ref = 0;
  return PT_OK;
}

// ------------------------------------------------------ binned SAH trees ---
// Trees whose answer does not depend on their shape, built for speed instead of
// reference compatibility (the reference's buildBVHwithSAH caps costs at INF =
// 114514 and falls back to median-x splits near the root of a 30k-triangle
// scene):
//  * the G-buffer tree over the raster triangles: its walk keeps the closest t
//    with ties to the lower original index and widened boxes only cull, so any
//    tree gives the same pixel;
//  * the any-hit (shadow) tree over the REFERENCE tree's leaves: its leaves are
//    exactly the reference leaves (same triangle ranges, same boxes) and every
//    interior box is an exact min/max union of them. A triangle is tested iff its
//    leaf box passes the slab test in either tree (an enclosing box passes
//    whenever an enclosed one does: slab rounding is monotone), so shadow
//    verdicts are those of the reference tree.
// A primitive is one triangle (G-buffer) or one reference leaf (any-hit).
struct SahPrim {
  float lo[3], hi[3];
  int weight;  // triangles it holds (SAH intersection cost)
  int ref;     // leaf ref it emits alone (any-hit tree), or its index (G-buffer)
};
struct SahNode {
  float lo[3], hi[3];
  int left = -1, right = -1;  // children (interior)
  int first = 0, n = 0;       // primitive range (leaf)
  int ref = 0;                // leaf: its ref, when `direct` (a fine leaf of refine_leaves) instead of leaf_ref()
  bool direct = false;
  bool keep = false;          // interior node whose box must be tested as is (a refined reference leaf): pack_wide
};

static float sah_area(const float* lo, const float* hi) {
  const float dx = std::max(hi[0] - lo[0], 0.0f), dy = std::max(hi[1] - lo[1], 0.0f), dz = std::max(hi[2] - lo[2], 0.0f);
  return dx * dy + dy * dz + dz * dx;
}

// Exact (full-sweep) SAH split of pr[l, r): per axis the primitives sorted by centroid, every cut priced; pr is
// left sorted along the best axis and *m is the cut. Returns the best cost (INFINITY: no split).
static float sah_sweep(std::vector<SahPrim>& pr, int l, int r, int* m) {
  const int n = r - l;
  std::vector<float> rarea((size_t)n);
  std::vector<int> rw((size_t)n);
  float best = INFINITY;
  int bax = -1, bcut = 0;
  auto by_axis = [&](int a) {
    std::sort(pr.begin() + l, pr.begin() + r, [a](const SahPrim& x, const SahPrim& y) {
      const float cx = x.lo[a] + x.hi[a], cy = y.lo[a] + y.hi[a];
      return cx < cy || (cx == cy && x.ref < y.ref);
    });
  };
  for (int a = 0; a < 3; ++a) {
    by_axis(a);
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    int w = 0;
    for (int i = n - 1; i >= 1; --i) {
      const SahPrim& q = pr[l + i];
      for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], q.lo[k]); hi[k] = std::max(hi[k], q.hi[k]); }
      w += q.weight;
      rarea[i] = sah_area(lo, hi);
      rw[i] = w;
    }
    for (int k = 0; k < 3; ++k) { lo[k] = INFINITY; hi[k] = -INFINITY; }
    w = 0;
    for (int i = 0; i + 1 < n; ++i) {
      const SahPrim& q = pr[l + i];
      for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], q.lo[k]); hi[k] = std::max(hi[k], q.hi[k]); }
      w += q.weight;
      const float c = sah_area(lo, hi) * w + rarea[i + 1] * rw[i + 1];
      if (c < best) { best = c; bax = a; bcut = i + 1; }
    }
  }
  if (bax < 0) return INFINITY;
  if (bax != 2) by_axis(bax);
  *m = l + bcut;
  return best;
}

// Build-quality switch (PTSVGF_SAH_SWEEP, read once): 1 (default) = exact sweep SAH, 0 = 16-bin SAH
// (measured 4K 6.885 -> 6.79 ms, 1080p 2.72 -> 2.64 ms with the sweep, tools/exp_env_ab.sh).
static bool sah_use_sweep() {
  static const bool on = [] {
    const char* e = getenv("PTSVGF_SAH_SWEEP");
    return !e || atoi(e) != 0;
  }();
  return on;
}

// 16-bin SAH over primitive centroids (cost: 1 per node visit, `weight` per primitive test), or the exact sweep.
// max_leaf: the most primitives a leaf may hold (leaves also stop at 15 triangles, the leaf ref's limit).
static int ceil_log2(int n) {
  int k = 0;
  while ((1 << k) < n) ++k;
  return k;
}

// depth: this node's level (root = 1). Once the SAH splits could take the tree past the LDS stack, the rest of the
// range is halved by index (sorted along the widest centroid axis), so every tree fits the stack: interior levels
// stay below kStack - 1 whatever the geometry (coincident centroids make SAH peel one primitive per level).
// reserve: stack levels kept free below the leaves (the any-hit tree's fine subtrees, refine_leaves)
static int sah_build(std::vector<SahPrim>& pr, int l, int r, int max_leaf, std::vector<SahNode>& nodes, int depth = 1,
                     int reserve = 0) {
  const int id = (int)nodes.size();
  nodes.emplace_back();
  SahNode nd;
  float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int a = 0; a < 3; ++a) { nd.lo[a] = INFINITY; nd.hi[a] = -INFINITY; }
  int w = 0;
  for (int i = l; i < r; ++i) {
    for (int a = 0; a < 3; ++a) {
      nd.lo[a] = std::min(nd.lo[a], pr[i].lo[a]);
      nd.hi[a] = std::max(nd.hi[a], pr[i].hi[a]);
      const float c = 0.5f * (pr[i].lo[a] + pr[i].hi[a]);
      clo[a] = std::min(clo[a], c);
      chi[a] = std::max(chi[a], c);
    }
    w += pr[i].weight;
  }
  const int n = r - l;
  constexpr int kBins = 16;
  float best = INFINITY;
  int bax = -1, bsplit = 0, msweep = -1;
  const bool sweep = sah_use_sweep();
  if (sweep && n > 1) {
    best = sah_sweep(pr, l, r, &msweep);
    if (best < INFINITY) bax = 0;
  }
  if (!sweep && n > 1) {
    for (int a = 0; a < 3; ++a) {
      const float ext = chi[a] - clo[a];
      if (!(ext > 0.0f)) continue;
      float blo[kBins][3], bhi[kBins][3];
      int bw[kBins] = {0}, bn[kBins] = {0};
      for (int b = 0; b < kBins; ++b)
        for (int k = 0; k < 3; ++k) { blo[b][k] = INFINITY; bhi[b][k] = -INFINITY; }
      for (int i = l; i < r; ++i) {
        const float c = 0.5f * (pr[i].lo[a] + pr[i].hi[a]);
        const int b = std::min(kBins - 1, (int)((c - clo[a]) / ext * kBins));
        ++bn[b];
        bw[b] += pr[i].weight;
        for (int k = 0; k < 3; ++k) { blo[b][k] = std::min(blo[b][k], pr[i].lo[k]); bhi[b][k] = std::max(bhi[b][k], pr[i].hi[k]); }
      }
      float rlo[kBins][3], rhi[kBins][3];
      int rw[kBins], rn[kBins];
      for (int b = kBins - 1; b >= 0; --b) {
        for (int k = 0; k < 3; ++k) {
          rlo[b][k] = b + 1 < kBins ? std::min(rlo[b + 1][k], blo[b][k]) : blo[b][k];
          rhi[b][k] = b + 1 < kBins ? std::max(rhi[b + 1][k], bhi[b][k]) : bhi[b][k];
        }
        rw[b] = (b + 1 < kBins ? rw[b + 1] : 0) + bw[b];
        rn[b] = (b + 1 < kBins ? rn[b + 1] : 0) + bn[b];
      }
      float llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
      int lw = 0, ln = 0;
      for (int b = 0; b + 1 < kBins; ++b) {
        for (int k = 0; k < 3; ++k) { llo[k] = std::min(llo[k], blo[b][k]); lhi[k] = std::max(lhi[k], bhi[b][k]); }
        lw += bw[b];
        ln += bn[b];
        if (ln == 0 || rn[b + 1] == 0) continue;
        const float c = sah_area(llo, lhi) * lw + sah_area(rlo[b + 1], rhi[b + 1]) * rw[b + 1];
        if (c < best) { best = c; bax = a; bsplit = b; }
      }
    }
  }
  const float area = sah_area(nd.lo, nd.hi);
  const bool fits = n <= max_leaf && w <= 15;
  if (n == 1 || (fits && (bax < 0 || !(area > 0.0f) || 1.0f + best / area >= (float)w))) {
    nd.first = l;
    nd.n = n;
    nodes[id] = nd;
    return id;
  }
  int m;
  if (depth + ceil_log2(n) + reserve >= kStack - 2) {  // depth cap: balanced halves from here on
    int ax = 0;
    for (int a = 1; a < 3; ++a)
      if (chi[a] - clo[a] > chi[ax] - clo[ax]) ax = a;
    std::sort(pr.begin() + l, pr.begin() + r, [ax](const SahPrim& x, const SahPrim& y) {
      const float cx = x.lo[ax] + x.hi[ax], cy = y.lo[ax] + y.hi[ax];
      return cx < cy || (cx == cy && x.ref < y.ref);
    });
    m = l + n / 2;
  } else if (sweep && msweep > l) {
    m = msweep;
  } else if (!sweep && bax >= 0) {
    const float ext = chi[bax] - clo[bax];
    m = (int)(std::partition(pr.begin() + l, pr.begin() + r, [&](const SahPrim& q) {
          const float c = 0.5f * (q.lo[bax] + q.hi[bax]);
          return std::min(kBins - 1, (int)((c - clo[bax]) / ext * kBins)) <= bsplit;
        }) - pr.begin());
  } else {
    m = l + n / 2;  // coincident centroids: halve the range
  }
  nd.left = sah_build(pr, l, m, max_leaf, nodes, depth + 1, reserve);
  nd.right = sah_build(pr, m, r, max_leaf, nodes, depth + 1, reserve);
  nodes[id] = nd;
  return id;
}

// Treelet restructuring of a built SahNode tree (PTSVGF_TREELET = passes, read once; default 1, 0 = off): for every interior node,
// bottom up, its treelet of up to 7 leaves (the root's descendants, the largest interior one opened first) is rebuilt
// as the binary tree of least SAH cost over those leaves (a dynamic program over the 127 leaf subsets), when that
// is cheaper. Boxes are unions again afterwards, so every walk's candidates stay the reference's (the containment
// argument of pack_wide); a tree that would grow past the stack's depth budget is left as it was.
// Bench scene (profiles/r06/treelet/): SAH cost / root area 121.56 -> 117.50 with one pass (117.00 with three); at 4K
// shadow visits -2.4 % / -3.1 % (default / surface view), bounce visits -1.0 % / -0.3 % (three passes: the surface
// view's shadow visits +0.4 %, so one pass); same bits; same box, three alternating repetitions: 227.7 / 228.4 / 227.6
// -> 225.8 / 228.1 / 227.7 fps at 4K (within noise), surface view 79.35 / 78.48 / 79.37 -> 80.02 / 80.63 / 80.13.
static int treelet_passes() {
  static const int n = [] {
    const char* e = getenv("PTSVGF_TREELET");
    return e ? std::max(0, atoi(e)) : 1;
  }();
  return n;
}

static void post_order(const std::vector<SahNode>& nodes, int root, std::vector<int>& order) {
  order.clear();
  std::vector<std::pair<int, bool>> st{{root, false}};
  while (!st.empty()) {
    auto [id, done] = st.back();
    st.pop_back();
    if (done || nodes[id].n > 0) { order.push_back(id); continue; }
    st.push_back({id, true});
    st.push_back({nodes[id].right, false});
    st.push_back({nodes[id].left, false});
  }
}

// SAH cost of node id's subtree (interior: its area + its children's; leaf: area x triangles), sah_build's model
static double sah_tree_cost(const std::vector<SahNode>& nodes, const std::vector<SahPrim>& pr, std::vector<double>& c) {
  std::vector<int> order;
  post_order(nodes, 0, order);
  c.assign(nodes.size(), 0.0);
  for (int id : order) {
    const SahNode& x = nodes[id];
    const double a = sah_area(x.lo, x.hi);
    if (x.n > 0) {
      int w = 0;
      for (int i = x.first; i < x.first + x.n; ++i) w += pr[i].weight;
      c[id] = a * w;
    } else {
      c[id] = a + c[x.left] + c[x.right];
    }
  }
  return c[0];
}

static int tree_depth(const std::vector<SahNode>& nodes) {
  int best = 0;
  std::vector<std::pair<int, int>> st{{0, 1}};
  while (!st.empty()) {
    auto [id, d] = st.back();
    st.pop_back();
    best = std::max(best, d);
    if (nodes[id].n == 0) {
      st.push_back({nodes[id].left, d + 1});
      st.push_back({nodes[id].right, d + 1});
    }
  }
  return best;
}

static void treelet_optimize(std::vector<SahNode>& nodes, const std::vector<SahPrim>& pr, int passes, int reserve,
                             double* sah_before = nullptr, double* sah_after = nullptr) {
  if (passes <= 0 || nodes.empty() || nodes[0].n > 0) {
    std::vector<double> c;
    const double v = nodes.empty() ? 0.0 : sah_tree_cost(nodes, pr, c) / std::max(1e-30, (double)sah_area(nodes[0].lo, nodes[0].hi));
    if (sah_before) *sah_before = v;
    if (sah_after) *sah_after = v;
    return;
  }
  const std::vector<SahNode> orig = nodes;
  constexpr int KMAX = 10;
  static const int K = [KMAX] {  // treelet leaves (PTSVGF_TREELET_LEAVES, 3..10, default 7)
    const char* e = getenv("PTSVGF_TREELET_LEAVES");
    return e ? std::min(KMAX, std::max(3, atoi(e))) : 7;
  }();
  std::vector<double> cost;
  const double before = sah_tree_cost(nodes, pr, cost);
  std::vector<int> order;
  for (int pass = 0; pass < passes; ++pass) {
    bool changed = false;
    post_order(nodes, 0, order);
    for (int r : order) {
      if (nodes[r].n > 0) continue;
      // its subtree may have changed below (children come first in post order)
      cost[r] = sah_area(nodes[r].lo, nodes[r].hi) + cost[nodes[r].left] + cost[nodes[r].right];
      int T[KMAX], nt = 2, I[KMAX], ni = 1;
      T[0] = nodes[r].left;
      T[1] = nodes[r].right;
      I[0] = r;
      while (nt < K) {  // open the largest interior treelet leaf
        int b = -1;
        float ba = -1.0f;
        for (int i = 0; i < nt; ++i)
          if (nodes[T[i]].n == 0) {
            const float a = sah_area(nodes[T[i]].lo, nodes[T[i]].hi);
            if (a > ba) { ba = a; b = i; }
          }
        if (b < 0) break;
        const int x = T[b];
        I[ni++] = x;
        T[b] = nodes[x].left;
        T[nt++] = nodes[x].right;
      }
      if (nt < 3) continue;
      const int full = (1 << nt) - 1;
      static thread_local std::vector<double> area(1 << KMAX), best(1 << KMAX);
      static thread_local std::vector<int> split(1 << KMAX);
      for (int S = 1; S <= full; ++S) {
        float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int i = 0; i < nt; ++i)
          if (S >> i & 1)
            for (int k = 0; k < 3; ++k) {
              lo[k] = std::min(lo[k], nodes[T[i]].lo[k]);
              hi[k] = std::max(hi[k], nodes[T[i]].hi[k]);
            }
        area[S] = sah_area(lo, hi);
        if ((S & (S - 1)) == 0) {
          int i = 0;
          while (!(S >> i & 1)) ++i;
          best[S] = cost[T[i]];
          split[S] = 0;
          continue;
        }
        double b = INFINITY;
        int bp = 0;
        const int low = S & -S;  // P holds S's lowest leaf: each unordered split once
        for (int P = (S - 1) & S; P > 0; P = (P - 1) & S) {
          if (!(P & low)) continue;
          const double c = best[P] + best[S ^ P];
          if (c < b) { b = c; bp = P; }
        }
        best[S] = area[S] + b;
        split[S] = bp;
      }
      if (!(best[full] < cost[r] * (1.0 - 1e-6))) continue;
      // rebuild: the treelet's interior nodes I (r stays the root), leaves T
      int next = 1;
      std::function<int(int, bool)> make = [&](int S, bool root) -> int {
        if ((S & (S - 1)) == 0) {
          int i = 0;
          while (!(S >> i & 1)) ++i;
          return T[i];
        }
        const int id = root ? r : I[next++];
        const int L = make(split[S], false), R = make(S ^ split[S], false);
        SahNode nd = nodes[id];
        nd.n = 0;
        nd.left = L;
        nd.right = R;
        for (int k = 0; k < 3; ++k) {
          nd.lo[k] = std::min(nodes[L].lo[k], nodes[R].lo[k]);
          nd.hi[k] = std::max(nodes[L].hi[k], nodes[R].hi[k]);
        }
        nodes[id] = nd;
        cost[id] = sah_area(nd.lo, nd.hi) + cost[L] + cost[R];
        return id;
      };
      make(full, true);
      changed = true;
    }
    if (!changed) break;
  }
  const double after = sah_tree_cost(nodes, pr, cost);
  const int depth = tree_depth(nodes);
  const bool keep = depth + reserve < kStack - 2;
  if (!keep) nodes = orig;
  const double root_area = std::max(1e-30, (double)sah_area(orig[0].lo, orig[0].hi));
  if (sah_before) *sah_before = before / root_area;
  if (sah_after) *sah_after = (keep ? after : before) / root_area;
  if (getenv("PTSVGF_WIDE_STATS"))
    fprintf(stderr, "ptsvgf: treelet restructuring (%d passes): SAH cost / root area %.4f -> %.4f, depth %d%s\n", passes,
            before / std::max(1e-30, (double)sah_area(orig[0].lo, orig[0].hi)),
            after / std::max(1e-30, (double)sah_area(orig[0].lo, orig[0].hi)), depth,
            keep ? "" : " (too deep for the stack: not used)");
}

// Pack a SahNode tree in pack_bvh's layout (DFS order, 4 x float4 per interior node).
// leaf_ref(first, n) gives the ref of a leaf holding primitives [first, first + n).
static int pack_sah(const std::vector<SahNode>& nodes, const std::function<int(int, int)>& leaf_ref,
                    std::vector<float4>& out, int* root_ref, int* need) {
  *need = 0;
  out.clear();
  if (nodes[0].n > 0) {
    *root_ref = leaf_ref(nodes[0].first, nodes[0].n);
    return PT_OK;
  }
  std::vector<int> idx(nodes.size(), -1), order;
  struct Item { int id, depth; };
  std::vector<Item> st{{0, 1}};
  while (!st.empty()) {
    const Item it = st.back();
    st.pop_back();
    if (it.depth >= kStack) return err(PT_ERR_FORMAT, "SAH tree deeper than the traversal stack");
    *need = std::max(*need, it.depth);
    idx[it.id] = (int)order.size();
    order.push_back(it.id);
    const SahNode& n = nodes[it.id];
    if (nodes[n.right].n == 0) st.push_back({n.right, it.depth + 1});
    if (nodes[n.left].n == 0) st.push_back({n.left, it.depth + 1});
  }
  out.assign(order.size() * 4, float4{0, 0, 0, 0});
  for (size_t k = 0; k < order.size(); ++k) {
    const SahNode& n = nodes[order[k]];
    const SahNode& L = nodes[n.left];
    const SahNode& R = nodes[n.right];
    const int rl = L.n > 0 ? (L.direct ? L.ref : leaf_ref(L.first, L.n)) : idx[n.left];
    const int rr = R.n > 0 ? (R.direct ? R.ref : leaf_ref(R.first, R.n)) : idx[n.right];
    float4* q = &out[4 * k];
    q[0] = float4{L.lo[0], L.lo[1], L.lo[2], L.hi[0]};
    q[1] = float4{L.hi[1], L.hi[2], R.lo[0], R.lo[1]};
    q[2] = float4{R.lo[2], R.hi[0], R.hi[1], R.hi[2]};
    float a, b;
    memcpy(&a, &rl, 4);
    memcpy(&b, &rr, 4);
    q[3] = float4{a, b, 0, 0};
  }
  *root_ref = 0;
  return PT_OK;
}

static int ref_first_of(int ref) { return (-(ref + 1)) >> 4; }
static int ref_count_of(int ref) { return (-(ref + 1)) & 15; }

// 4-wide form of a SahNode tree (the traversal kernels' WIDE walks): each 4-wide node holds up to four descendants of
// one binary node, the largest interior child opened first, never a `keep` node (a refined reference leaf keeps its
// exact box as a child box, refine_leaves). An opened node's box is only skipped, and it encloses the boxes that
// replace it (a union, or the widened fine boxes below a reference leaf, which only cull): a ray passing a kept box
// passed the skipped one too (slab rounding is monotone under containment), so the candidate triangles, and with
// them every closest t and any-hit verdict, are the binary tree's. Exact ties are re-walked on the reference tree.
// Layout (kWideStride x float4: 7 used = 112 B, padded to 128 B at 8): lo.x[4] hi.x[4] lo.y[4] hi.y[4] lo.z[4] hi.z[4] refs[4]; refs >= 0 node index,
// < 0 leaf, kNoneRef an empty slot. *need: the most stack entries a walk can hold (sum over a path of the
// children pushed beside the one taken); the kernels check pushes against their stack anyway.
// Which binary nodes a 4-wide node opens (PTSVGF_WIDE_COLLAPSE, read once): 0 = greedy (until round 6), the largest
// interior child opened until four slots are used; 1 = SAH-optimal, a dynamic program over the binary tree that picks
// the grouping with the least summed surface area of 4-wide nodes (each such node is one node step of a walk that
// reaches it; the leaves, hence their triangle tests, are the same either way); 2 = SAH-optimal for the any-hit
// (shadow) walks and greedy for the closest-hit walks, two trees in one buffer (SceneDev::root4c; the default);
// 3 = the reverse. Every form keeps `keep` nodes closed, so each is result-preserving by the argument above.
// Measured at 4K (profiles/r06/wide_collapse/, one box, two alternating repetitions): greedy 225.2 / 227.2 fps,
// surface view 78.0 / 78.3; SAH-optimal for both 231.1 / 229.6 and 76.6 / 76.1 (shadow visits -1.5 % / -7.1 %, but
// the surface view's closest-hit visits +7.8 %: the nearest-first, pruned walk is not what the area sum prices);
// mode 2 228.0 / 228.4 and 79.3 / 78.7. Same bits in every mode (planes digest, the wide-tree parity tests).
static int wide_collapse_mode() {
  static const int m = [] {
    const char* e = getenv("PTSVGF_WIDE_COLLAPSE");
    return e ? atoi(e) : 2;
  }();
  return m;
}

// The dynamic program of wide_collapse_mode() 1. For a binary node x: best[x] = A(x) + D(x, 4) (x as a 4-wide node);
// S(x, j) = the least cost of x's subtree given j slots of the enclosing 4-wide node (one slot: x itself, a leaf at
// cost 0 or a 4-wide node at best[x]; more: opened, its children sharing the slots); D(x, i) = min over j of
// S(left, j) + S(right, i - j), in one pass over the nodes in post order.
struct WideCollapse {
  std::vector<float> best;
  std::vector<std::array<float, 5>> S, D;
  std::vector<std::array<signed char, 5>> dsplit;  // D(x, i): slots given to the left child
  std::vector<std::array<bool, 5>> sopen;          // S(x, j): opened (else one slot)
  explicit WideCollapse(const std::vector<SahNode>& nodes) {
    const size_t n = nodes.size();
    best.assign(n, 0.0f);
    S.assign(n, {});
    D.assign(n, {});
    dsplit.assign(n, {});
    sopen.assign(n, {});
    std::vector<int> order;  // children before parents (ids need not be: treelet_optimize reuses them)
    post_order(nodes, 0, order);
    for (int k : order) {
      const SahNode& x = nodes[k];
      const bool leaf = x.n > 0;
      if (!leaf) {
        for (int i = 2; i <= 4; ++i) {
          float b = INFINITY;
          int bj = 1;
          for (int j = 1; j < i; ++j) {
            const float c = S[x.left][j] + S[x.right][i - j];
            if (c < b) { b = c; bj = j; }
          }
          D[k][i] = b;
          dsplit[k][i] = (signed char)bj;
        }
        best[k] = sah_area(x.lo, x.hi) + D[k][4];
      }
      const float slot = leaf ? 0.0f : best[k];
      for (int j = 1; j <= 4; ++j) {
        const bool open = !leaf && !x.keep && j >= 2 && D[k][j] < slot;
        S[k][j] = open ? D[k][j] : slot;
        sopen[k][j] = open;
      }
    }
  }
  // the children of a 4-wide node rooted at binary node id
  int children(const std::vector<SahNode>& nodes, int id, int* ch) const {
    int nc = 0;
    std::function<void(int, int)> cover = [&](int x, int j) {
      if (!sopen[x][j]) { ch[nc++] = x; return; }
      expand(nodes, x, j, cover);
    };
    expand(nodes, id, 4, cover);
    return nc;
  }
  void expand(const std::vector<SahNode>& nodes, int x, int i, const std::function<void(int, int)>& cover) const {
    const int j = dsplit[x][i];
    cover(nodes[x].left, j);
    cover(nodes[x].right, i - j);
  }
};

static int pack_wide(const std::vector<SahNode>& nodes, const std::function<int(int, int)>& leaf_ref,
                     std::vector<float4>& out, int* root_ref, int* need, bool dp, double* area_out = nullptr) {
  out.clear();
  *need = 0;
  auto ref_of = [&](const SahNode& L) { return L.direct ? L.ref : leaf_ref(L.first, L.n); };
  if (nodes[0].n > 0) {
    *root_ref = ref_of(nodes[0]);
    return PT_OK;
  }
  std::unique_ptr<WideCollapse> wc(dp ? new WideCollapse(nodes) : nullptr);
  static const int order_key = [] {
    const char* e = getenv("PTSVGF_WIDE_ORDER_KEY");
    return e ? atoi(e) : 0;
  }();
  std::vector<double> tris_below(nodes.size(), 0.0);  // triangles in each subtree (order_key 1 / 2)
  if (order_key) {
    std::vector<int> po;
    post_order(nodes, 0, po);
    for (int id : po) {
      const SahNode& x = nodes[id];
      tris_below[id] = x.n > 0 ? (double)ref_count_of(ref_of(x)) : tris_below[x.left] + tris_below[x.right];
    }
  }
  double area_sum = 0.0;  // summed surface area of the 4-wide nodes (PTSVGF_WIDE_STATS)
  std::function<int(int, int)> build = [&](int id, int acc) -> int {
    int ch[4] = {nodes[id].left, nodes[id].right, -1, -1};
    int nc = 2;
    area_sum += sah_area(nodes[id].lo, nodes[id].hi);
    if (dp) nc = wc->children(nodes, id, ch);
    while (!dp && nc < 4) {  // open the largest interior child that may be opened
      int best = -1;
      float ba = -1.0f;
      for (int c = 0; c < nc; ++c) {
        const SahNode& n = nodes[ch[c]];
        const float a = sah_area(n.lo, n.hi);
        if (n.n == 0 && !n.keep && a > ba) { ba = a; best = c; }
      }
      if (best < 0) break;
      const int b = ch[best];
      for (int c = nc; c > best + 1; --c) ch[c] = ch[c - 1];
      ch[best] = nodes[b].left;
      ch[best + 1] = nodes[b].right;
      ++nc;
    }
#if PT_WIDE_ORDER
    // slot order = build order: the first interior child is stored right after this node (depth first), so the
    // second cache line of this node's fetch holds most of it. Put the child a ray most likely enters there (largest
    // surface area). Slots only order ties between equally near children; the candidates, hence every result, are
    // the same.
    // PTSVGF_WIDE_ORDER_KEY (read once; A/B): 0 = area (default), 1 = triangles below, 2 = area x triangles below
    std::stable_sort(ch, ch + nc, [&](int x, int y) {
      const double ax = sah_area(nodes[x].lo, nodes[x].hi), ay = sah_area(nodes[y].lo, nodes[y].hi);
      if (order_key == 1) return tris_below[x] > tris_below[y];
      if (order_key == 2) return ax * tris_below[x] > ay * tris_below[y];
      return ax > ay;
    });
#endif
    const int k = (int)(out.size() / ptk::kWideStride);
    out.resize(out.size() + ptk::kWideStride, float4{0, 0, 0, 0});
    {  // empty slots: lo = +inf, hi = -inf, a box no ray enters (wide_step's signed test needs no slot check)
      float* q = (float*)&out[ptk::kWideStride * (size_t)k];
      for (int a = 0; a < 3; ++a)
        for (int c = nc; c < 4; ++c) {
          q[8 * a + c] = INFINITY;
          q[8 * a + 4 + c] = -INFINITY;
        }
    }
    const int here = acc + nc - 1;
    *need = std::max(*need, here + 1);
    int refs[4] = {kNoneRef, kNoneRef, kNoneRef, kNoneRef};
    for (int c = 0; c < nc; ++c) {
      const SahNode& n = nodes[ch[c]];
      float* q = (float*)&out[ptk::kWideStride * (size_t)k];
      for (int a = 0; a < 3; ++a) { q[8 * a + c] = n.lo[a]; q[8 * a + 4 + c] = n.hi[a]; }
      refs[c] = n.n > 0 ? ref_of(n) : build(ch[c], here);  // may reallocate `out`
    }
    memcpy(&out[ptk::kWideStride * (size_t)k + 6], refs, 16);
    return k;
  };
  build(0, 0);
  *root_ref = 0;
  if (area_out) *area_out = area_sum / std::max(1e-30, (double)sah_area(nodes[0].lo, nodes[0].hi));
  if (getenv("PTSVGF_WIDE_STATS"))
    fprintf(stderr, "ptsvgf: 4-wide tree (%s collapse): %zu nodes, summed node area / root area %.4f, stack need %d\n",
            dp ? "SAH-optimal" : "greedy", out.size() / ptk::kWideStride,
            area_sum / std::max(1e-30, (double)sah_area(nodes[0].lo, nodes[0].hi)), *need);
  return PT_OK;
}

// Fine leaves under the reference leaves (PTSVGF_FINE_LEAVES = F, the largest fine leaf; 0 = off). A reference leaf
// holds up to 8 triangles (BVH.h:77, main.cpp:96) in one box; every ray that passes that box tests all of them. Here
// each reference leaf of more than F triangles becomes an interior node over contiguous sub-ranges of its triangles
// (index order kept, so a fine leaf is a valid leaf ref), cut by SAH on their boxes, down to <= F triangles.
// Result-preserving: the reference leaf's own box is still tested exactly (it is the box the parent stores for this
// child), and a fine box is the min/max box of its triangles widened by `pad` (2^-12 of the largest coordinate
// magnitude, ~500x the float rounding of hitTriangle's hit point and of the slab arithmetic), so a ray that
// hitTriangle (:215-272) accepts for one of those triangles passes it: the fine boxes only cull triangles that cannot
// be hit, and the candidate set (and with it every closest t and any-hit verdict) is the reference leaf's. Exact ties
// are re-walked on the reference tree as before. Leaves with a non-finite vertex coordinate stay whole.
// The rounding of the hit point grows with the ray origin's magnitude and the hit distance, not with the vertices:
// bounce and shadow rays start on the scene (|origin| <= mag), primary rays at the eye. The pad covers eyes within
// kFineEyeReach x max(mag, 1) per coordinate (the rounding then stays >= 32x below the pad); pt_params walks the
// reference tree (no fine boxes) for an eye beyond that.
constexpr float kFineEyeReach = 64.0f;
static int fine_leaf_max() {
  static const int f = [] {
    const char* e = getenv("PTSVGF_FINE_LEAVES");
    return e ? std::max(0, atoi(e)) : 4;
  }();
  return f;
}

static int fine_subtree(const float* tri_enc, const float* tlo, const float* thi, int a, int b, int F, float pad,
                        std::vector<SahNode>& nodes, int forced_id = -1) {
  const int id = forced_id >= 0 ? forced_id : (int)nodes.size();
  if (forced_id < 0) nodes.emplace_back();
  SahNode nd = forced_id >= 0 ? nodes[forced_id] : SahNode{};
  auto box = [&](int u, int v, float* lo, float* hi) {
    for (int k = 0; k < 3; ++k) { lo[k] = INFINITY; hi[k] = -INFINITY; }
    for (int i = u; i < v; ++i)
      for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], tlo[3 * i + k]); hi[k] = std::max(hi[k], thi[3 * i + k]); }
    for (int k = 0; k < 3; ++k) { lo[k] -= pad; hi[k] += pad; }
  };
  if (forced_id < 0) box(a, b, nd.lo, nd.hi);  // the subtree root keeps the reference leaf's exact box
  if (b - a <= F) {
    nd.n = b - a;
    nd.direct = true;
    nd.ref = -(a * 16 + (b - a)) - 1;
    nodes[id] = nd;
    return id;
  }
  float best = INFINITY;
  int m = a + (b - a) / 2;
  for (int c = a + 1; c < b; ++c) {
    float l0[3], l1[3], r0[3], r1[3];
    box(a, c, l0, l1);
    box(c, b, r0, r1);
    const float cost = sah_area(l0, l1) * (c - a) + sah_area(r0, r1) * (b - c);
    if (cost < best) { best = cost; m = c; }
  }
  nd.n = 0;
  nd.direct = false;
  nd.left = fine_subtree(tri_enc, tlo, thi, a, m, F, pad, nodes);
  nd.right = fine_subtree(tri_enc, tlo, thi, m, b, F, pad, nodes);
  nodes[id] = nd;
  return id;
}

// Returns the coordinate magnitude the pad was sized for (0: no fine leaves).
static float refine_leaves(std::vector<SahNode>& nodes, const std::vector<SahPrim>& pr, const float* tri_enc,
                           int ntris, int F) {
  if (F <= 0 || !tri_enc) return 0.0f;
  std::vector<float> tlo((size_t)ntris * 3), thi((size_t)ntris * 3);
  std::vector<char> finite((size_t)ntris);
  float mag = 0.0f;
  for (int i = 0; i < ntris; ++i) {
    const float* f = tri_enc + (size_t)i * 45;  // Triangle_encoded: p1 p2 p3 first (Triangle.h:12-24)
    bool ok = true;
    for (int k = 0; k < 3; ++k) {
      const float v0 = f[k], v1 = f[3 + k], v2 = f[6 + k];
      ok = ok && std::isfinite(v0) && std::isfinite(v1) && std::isfinite(v2);
      tlo[3 * i + k] = std::min(v0, std::min(v1, v2));
      thi[3 * i + k] = std::max(v0, std::max(v1, v2));
    }
    finite[i] = ok;
    if (ok)
      for (int k = 0; k < 9; ++k) mag = std::max(mag, std::fabs(f[k]));
  }
  const float pad = std::max(mag, 1.0f) * (1.0f / 4096.0f);
  const size_t n0 = nodes.size();
  bool any = false;
  for (size_t id = 0; id < n0; ++id) {
    if (nodes[id].n <= 0) continue;
    const int ref = pr[nodes[id].first].ref;
    const int first = ref_first_of(ref), cnt = ref_count_of(ref);
    if (cnt <= F) continue;
    bool ok = true;
    for (int i = first; i < first + cnt; ++i) ok = ok && finite[i];
    if (!ok) continue;
    SahNode root = nodes[id];  // exact reference-leaf box, stored by the parent for this child
    root.n = 0;
    root.keep = true;
    nodes[id] = root;
    fine_subtree(tri_enc, tlo.data(), thi.data(), first, first + cnt, F, pad, nodes, (int)id);
    any = true;
  }
  return any ? std::max(mag, 1.0f) : 0.0f;
}

// Any-hit tree over the leaves of the reference tree (see above), with fine leaves under them (refine_leaves).
int build_anyhit_tree(const float* node_enc, int nnodes, int ntris, const float* tri_enc, std::vector<float4>& out,
                      int* root_ref, int* need, std::vector<float4>* wide = nullptr, int* root_wide = nullptr,
                      int* need_wide = nullptr, float* fine_mag = nullptr, int* root_closest = nullptr,
                      int collapse = -1, int treelet = -1, double* stats = nullptr) {
  // collapse / treelet: PTSVGF_WIDE_COLLAPSE / PTSVGF_TREELET when < 0; stats (pt_tree_check): SAH cost / root area
  // before and after the treelet pass, summed 4-wide node area / root area of the any-hit and closest-hit trees
  if (collapse < 0) collapse = wide_collapse_mode();
  if (treelet < 0) treelet = treelet_passes();
  double st_[4] = {0, 0, 0, 0};
  double* st = stats ? stats : st_;
  std::vector<SahPrim> pr;
  for (int i = 1; i < nnodes; ++i) {
    const float* f = node_enc + (size_t)i * 12;
    const int n = (int)f[3], first = (int)f[4];
    if (n <= 0) continue;
    if (n > 15 || first < 0 || first + n > ntris) return err(PT_ERR_FORMAT, "BVH leaf out of range");
    SahPrim q;
    for (int a = 0; a < 3; ++a) { q.lo[a] = f[6 + a]; q.hi[a] = f[9 + a]; }
    q.weight = n;
    q.ref = -(first * 16 + n) - 1;
    pr.push_back(q);
  }
  if (pr.empty()) return err(PT_ERR_FORMAT, "BVH without leaves");
  std::vector<SahNode> nodes;
  nodes.reserve(2 * pr.size());
  const int F = fine_leaf_max();
  sah_build(pr, 0, (int)pr.size(), 1, nodes, 1, F > 0 ? ceil_log2(16) : 0);  // a fine subtree is <= 4 levels deep
  treelet_optimize(nodes, pr, treelet, F > 0 ? ceil_log2(16) : 0, &st[0], &st[1]);
  const float mag = refine_leaves(nodes, pr, tri_enc, ntris, F);
  if (fine_mag) *fine_mag = mag;
  auto leaf_ref = [&](int first, int) { return pr[first].ref; };
  const int rc = pack_sah(nodes, leaf_ref, out, root_ref, need);
  if (rc != PT_OK || !wide) return rc;
  const int mode = collapse;
  const int rw = pack_wide(nodes, leaf_ref, *wide, root_wide, need_wide, mode == 1 || mode == 2, &st[2]);
  st[3] = st[2];
  if (root_closest) *root_closest = *root_wide;
  if (rw != PT_OK || !root_closest || (mode != 2 && mode != 3) || *root_wide < 0) return rw;
  // the closest-hit walks' tree, appended: its node indices shifted past the any-hit tree's
  std::vector<float4> second;
  int root2 = 0, need2 = 0;
  const int r2 = pack_wide(nodes, leaf_ref, second, &root2, &need2, mode == 3, &st[3]);
  if (r2 != PT_OK) return r2;
  const int base = (int)(wide->size() / ptk::kWideStride);
  for (size_t k = 0; k + ptk::kWideStride <= second.size(); k += ptk::kWideStride) {
    int refs[4];
    memcpy(refs, &second[k + 6], 16);
    for (int c = 0; c < 4; ++c)
      if (refs[c] >= 0) refs[c] += base;
    memcpy(&second[k + 6], refs, 16);
  }
  *root_closest = root2 + base;
  wide->insert(wide->end(), second.begin(), second.end());
  *need_wide = std::max(*need_wide, need2);
  return PT_OK;
}

// pt_tree_check (include/ptsvgf.h): the trees build_anyhit_tree makes for a reference tree, checked on the host
// against the properties the walks' result preservation rests on. Host only: no device, no pt_init.
struct TreeCheck {
  const float* node_enc;
  int nnodes;
  const float* tri_enc;
  int ntris;
  std::vector<int> cover;  // per triangle: leaves of the checked tree holding it
  std::vector<char> inref; // per triangle: held by a reference leaf
  std::map<std::array<uint32_t, 6>, int> refbox;  // reference leaf boxes (bits) -> triangle count
  bool contain_ok = true, leaf_ok = true;
  int depth = 0;
  static std::array<uint32_t, 6> key(const float* lo, const float* hi) {
    std::array<uint32_t, 6> k;
    for (int a = 0; a < 3; ++a) { memcpy(&k[a], &lo[a], 4); memcpy(&k[3 + a], &hi[a], 4); }
    return k;
  }
  void init() {
    cover.assign((size_t)ntris, 0);
    inref.assign((size_t)ntris, 0);
    for (int i = 1; i < nnodes; ++i) {
      const float* f = node_enc + (size_t)i * 12;
      const int n = (int)f[3], first = (int)f[4];
      if (n <= 0) continue;
      for (int t = first; t < first + n && t < ntris; ++t) inref[(size_t)t] = 1;
      refbox[key(f + 6, f + 9)] = n;
    }
  }
  static bool inside(const float* lo, const float* hi, const float* plo, const float* phi) {
    for (int a = 0; a < 3; ++a)
      if (lo[a] < plo[a] || hi[a] > phi[a]) return false;
    return true;
  }
  // a leaf ref below a box: its triangles marked; each triangle's vertex box inside the box
  void leaf(int ref, const float* lo, const float* hi) {
    const int first = ref_first_of(ref), cnt = ref_count_of(ref);
    for (int t = first; t < first + cnt; ++t) {
      if (t < 0 || t >= ntris) { leaf_ok = false; continue; }
      ++cover[(size_t)t];
      const float* v = tri_enc + (size_t)t * 45;
      for (int a = 0; a < 3; ++a) {
        const float tl = std::min(v[a], std::min(v[3 + a], v[6 + a])), th = std::max(v[a], std::max(v[3 + a], v[6 + a]));
        if (std::isfinite(tl) && std::isfinite(th) && (tl < lo[a] || th > hi[a])) contain_ok = false;
      }
    }
  }
  // a child slot box (lo, hi) holding a subtree; `fine`: the box is a reference leaf's (its fine boxes, widened, need
  // not lie inside it: each fine leaf's box must hold its triangles instead)
  bool is_ref_leaf_box(const float* lo, const float* hi) const { return refbox.count(key(lo, hi)) != 0; }
  bool partition_ok() const {
    for (int t = 0; t < ntris; ++t)
      if (cover[(size_t)t] != (inref[(size_t)t] ? 1 : 0)) return false;
    return true;
  }
  void walk_binary(const std::vector<float4>& bvh, int ref, const float* lo, const float* hi, bool fine, int d) {
    depth = std::max(depth, d);
    if (ref < 0) { leaf(ref, lo, hi); return; }
    const float* q = (const float*)&bvh[4 * (size_t)ref];
    const float L0[3] = {q[0], q[1], q[2]}, L1[3] = {q[3], q[4], q[5]};
    const float R0[3] = {q[6], q[7], q[8]}, R1[3] = {q[9], q[10], q[11]};
    int rl, rr;
    memcpy(&rl, &q[12], 4);
    memcpy(&rr, &q[13], 4);
    for (int s = 0; s < 2; ++s) {
      const float* cl = s ? R0 : L0;
      const float* ch = s ? R1 : L1;
      if (!fine && lo && !inside(cl, ch, lo, hi)) contain_ok = false;
      walk_binary(bvh, s ? rr : rl, cl, ch, fine || is_ref_leaf_box(cl, ch), d + 1);
    }
  }
  void walk_wide(const std::vector<float4>& w, int ref, const float* lo, const float* hi, bool fine, int d) {
    depth = std::max(depth, d);
    if (ref < 0) { leaf(ref, lo, hi); return; }
    const float* q = (const float*)&w[(size_t)ptk::kWideStride * ref];
    int refs[4];
    memcpy(refs, q + 24, 16);
    for (int c = 0; c < 4; ++c) {
      if (refs[c] == kNoneRef) continue;
      const float cl[3] = {q[c], q[8 + c], q[16 + c]}, ch[3] = {q[4 + c], q[12 + c], q[20 + c]};
      if (!fine && lo && !inside(cl, ch, lo, hi)) contain_ok = false;
      walk_wide(w, refs[c], cl, ch, fine || is_ref_leaf_box(cl, ch), d + 1);
    }
  }
};

int tree_check(const float* node_enc, int nnodes, const float* tri_enc, int ntris, int collapse, int treelet,
               double* out, int nout) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  if (!node_enc || !tri_enc || !out || nnodes < 2 || ntris < 1) return err(PT_ERR_ARG, "trees and output needed");
  if (nout < PT_TREE_CHECK_COUNT) return err(PT_ERR_ARG, "output holds fewer than PT_TREE_CHECK_COUNT values");
  if (collapse < 0 || collapse > 3 || treelet < 0) return err(PT_ERR_ARG, "collapse in 0..3, treelet >= 0");
  std::vector<float4> bin, wide;
  int root_any = 0, need_any = 0, root4 = 0, need4 = 0, root4c = 0;
  float mag = 0.0f;
  double st[4] = {0, 0, 0, 0};
  const int rc = build_anyhit_tree(node_enc, nnodes, ntris, tri_enc, bin, &root_any, &need_any, &wide, &root4, &need4,
                                   &mag, &root4c, collapse, treelet, st);
  if (rc != PT_OK) return rc;
  double ok[3];
  int depth[3];
  bool contain = true;
  for (int k = 0; k < 3; ++k) {
    TreeCheck tc{node_enc, nnodes, tri_enc, ntris};
    tc.init();
    if (k == 0) tc.walk_binary(bin, root_any, nullptr, nullptr, false, 1);
    else tc.walk_wide(wide, k == 1 ? root4 : root4c, nullptr, nullptr, false, 1);
    ok[k] = tc.partition_ok() && tc.leaf_ok ? 1.0 : 0.0;
    depth[k] = tc.depth;
    contain = contain && tc.contain_ok;
  }
  const double vals[PT_TREE_CHECK_COUNT] = {ok[0], ok[1], ok[2], contain ? 1.0 : 0.0, st[0], st[1], st[2], st[3],
                                            (double)(wide.size() / ptk::kWideStride), (double)depth[0],
                                            (double)need4, root4c != root4 ? 1.0 : 0.0};
  for (int i = 0; i < PT_TREE_CHECK_COUNT; ++i) out[i] = vals[i];
  return PT_OK;
}

void free_scene(SceneGPU& sg) {
  float4** bufs[6] = {&sg.geom, &sg.shade, &sg.bvh, &sg.bvh4, &sg.bvh_any, &sg.leaves};
  for (auto b : bufs) {
    if (*b) (void)hipFree(*b);
    *b = nullptr;
  }
}

template <class T>
int upload_vec(const std::vector<T>& v, T** dst) {
  if (*dst) { (void)hipFree(*dst); *dst = nullptr; }
  if (v.empty()) return PT_OK;
  HIPCHK(hipMalloc((void**)dst, v.size() * sizeof(T)));
  HIPCHK(hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return PT_OK;
}

// The reference tree's leaves with their own boxes (the primary-ray tile rasteriser's items). The caller has checked
// the leaf ranges (pack_bvh).
static int upload_leaves(const float* ne, size_t nnodes, SceneGPU& sg) {
  std::vector<float4> lv;
  for (size_t i = 1; i < nnodes; ++i) {
    const float* f = ne + i * 12;
    const int n = (int)f[3], first = (int)f[4];
    if (n <= 0) continue;
    const int ref = -(first * 16 + n) - 1;
    float rf;
    memcpy(&rf, &ref, 4);
    lv.push_back(float4{f[6], f[7], f[8], rf});
    lv.push_back(float4{f[9], f[10], f[11], 0.0f});
  }
  sg.nleaves = (int)(lv.size() / 2);
  return upload_vec(lv, &sg.leaves);
}

// A scene pt_bvh_build wrote (dynamic scenes): its triangles are decoded on the device (decode_tris: the host
// decode's built-ins, the same records), and its own tree (an LBVH, not the reference's SAH tree) serves every walk:
// no 4-wide or any-hit SAH tree is derived from it, so a rebuild costs the GPU build, this decode and the host
// packing of the node texels (DESIGN.md "Dynamic scenes").
int get_scene_lbvh(Texture* tris, Texture* nodes, SceneGPU& sg, SceneGPU** out) {
  const size_t ntris = tris->bytes / (45 * sizeof(float));
  const size_t nnodes = nodes->host.size() / (12 * sizeof(float));
  std::vector<float4> bvh;
  int root = 0;
  int rc = pack_bvh((const float*)nodes->host.data(), (int)nnodes, bvh, &root, (int)ntris, &sg.stack_need);
  if (rc != PT_OK) return rc;
  if ((rc = upload_leaves((const float*)nodes->host.data(), nnodes, sg)) != PT_OK) return rc;
  if (bvh.empty()) bvh.push_back(float4{0, 0, 0, 0});
  if ((rc = upload_vec(bvh, &sg.bvh)) != PT_OK) return rc;
  float4** opt[2] = {&sg.bvh4, &sg.bvh_any};
  for (auto b : opt)
    if (*b) { (void)hipFree(*b); *b = nullptr; }
  sg.has4 = false;
  sg.need_any = sg.root_any = sg.need4 = sg.root4 = sg.root4c = 0;  // no any-hit tree: its depth must not size the stack
  if (sg.geom) (void)hipFree(sg.geom);
  if (sg.shade) (void)hipFree(sg.shade);
  sg.geom = sg.shade = nullptr;
  HIPCHK(hipMalloc((void**)&sg.geom, std::max<size_t>(ntris, 1) * 4 * sizeof(float4)));
  HIPCHK(hipMalloc((void**)&sg.shade, std::max<size_t>(ntris, 1) * 9 * sizeof(float4)));
  HIPCHK((hipError_t)ptk::decode_tris((const float*)tris->dev, (int)ntris, sg.geom, sg.shade, g.stream));
  sg.root_ref = root;
  sg.ntris = (int)ntris;
  sg.tri_ver = tris->version;
  sg.node_ver = nodes->version;
  *out = &sg;
  return PT_OK;
}

int get_scene(Texture* tris, uint32_t th, Texture* nodes, uint32_t nh, SceneGPU** out) {
  SceneGPU& sg = g.scenes[{th, nh}];
  if (sg.geom && sg.tri_ver == tris->version && sg.node_ver == nodes->version) {
    *out = &sg;
    return PT_OK;
  }
  using namespace glsl;
  size_t ntris = tris->host.size() / (45 * sizeof(float));
  size_t nnodes = nodes->host.size() / (12 * sizeof(float));
  if (tris->lbvh && nodes->lbvh) return get_scene_lbvh(tris, nodes, sg, out);
  const float* te = (const float*)tris->host.data();
  std::vector<float4> geom(ntris * 4), shade(ntris * 9);
  for (size_t i = 0; i < ntris; ++i) {
    const float* f = te + i * 45;
    v3 p1 = mk(f[0], f[1], f[2]), p2 = mk(f[3], f[4], f[5]), p3 = mk(f[6], f[7], f[8]);
    v3 N = normalize(cross(sub(p2, p1), sub(p3, p1)));  // hitTriangle :227, same built-ins
    geom[4 * i + 0] = float4{p1.x, p1.y, p1.z, dot(N, p1)};
    geom[4 * i + 1] = float4{p2.x, p2.y, p2.z, 0.0f};
    geom[4 * i + 2] = float4{p3.x, p3.y, p3.z, 0.0f};
    geom[4 * i + 3] = float4{N.x, N.y, N.z, 0.0f};
    float4* s = &shade[9 * i];
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
  std::vector<float4> bvh, bvh4;
  int root = 0, root4 = 0, need4 = 0, root4c = 0;
  int rc = pack_bvh((const float*)nodes->host.data(), (int)nnodes, bvh, &root, (int)ntris, &sg.stack_need);
  if (rc != PT_OK) return rc;
  {  // optional: without it shadow and closest-hit rays walk the reference tree (binary, or its 4-wide form)
    std::vector<float4> any;
    sg.has4 = false;
    float fine_mag = 0.0f;
    sg.fine_eye_limit = INFINITY;
    if (build_anyhit_tree((const float*)nodes->host.data(), (int)nnodes, (int)ntris, te, any, &sg.root_any,
                          &sg.need_any, &bvh4, &root4, &need4, &fine_mag, &root4c) == PT_OK) {
      if (fine_mag > 0.0f) sg.fine_eye_limit = kFineEyeReach * fine_mag;
      if (any.empty()) any.push_back(float4{0, 0, 0, 0});
      if ((rc = upload_vec(any, &sg.bvh_any)) != PT_OK) return rc;
      if (bvh4.empty()) bvh4.push_back(float4{0, 0, 0, 0});
      if ((rc = upload_vec(bvh4, &sg.bvh4)) != PT_OK) return rc;
      sg.has4 = true;
      sg.root4 = root4;
      sg.root4c = root4c;
      sg.nan4 = false;
      for (size_t k = 0; k + ptk::kWideStride <= bvh4.size(); k += ptk::kWideStride) {
        const float* q = (const float*)&bvh4[k];
        int refs[4];
        memcpy(refs, q + 24, 16);
        for (int c = 0; c < 4; ++c)
          for (int i = 0; i < 6; ++i) sg.nan4 = sg.nan4 || (refs[c] != kNoneRef && std::isnan(q[4 * i + c]));
      }
      sg.need4 = need4;
      if (getenv("PTSVGF_SCENE_INFO"))  // diagnostics: the walks' working set (DESIGN.md "The traversal in round 4")
        fprintf(stderr, "ptsvgf scene: %zu triangles (geometry %zu B, shading %zu B), reference tree %zu B, any-hit "
                        "tree %zu B, 4-wide tree %zu nodes = %zu B, stack need %d / %d / %d\n",
                (size_t)ntris, (size_t)ntris * 64, (size_t)ntris * 144, bvh.size() * sizeof(float4),
                any.size() * sizeof(float4), bvh4.size() / ptk::kWideStride, bvh4.size() * sizeof(float4),
                sg.stack_need, sg.need_any, need4);
    } else {
      for (float4** b : {&sg.bvh_any, &sg.bvh4})
        if (*b) { (void)hipFree(*b); *b = nullptr; }
      sg.need_any = sg.root_any = sg.need4 = sg.root4 = sg.root4c = 0;
    }
  }
  if ((rc = upload_leaves((const float*)nodes->host.data(), nnodes, sg)) != PT_OK) return rc;
  if ((rc = upload_vec(geom, &sg.geom)) != PT_OK) return rc;
  if ((rc = upload_vec(shade, &sg.shade)) != PT_OK) return rc;
  if (bvh.empty()) bvh.push_back(float4{0, 0, 0, 0});
  if ((rc = upload_vec(bvh, &sg.bvh)) != PT_OK) return rc;
  sg.root_ref = root;
  sg.ntris = (int)ntris;
  sg.tri_ver = tris->version;
  sg.node_ver = nodes->version;
  *out = &sg;
  return PT_OK;
}

// -------------------------------------------------------------- bindings ---
const Uniform* U(Pass* p, const char* name, int type) {
  auto it = p->uni.find(name);
  if (it == p->uni.end()) return nullptr;
  return it->second.type == type ? &it->second : nullptr;
}
float uf(Pass* p, const char* n, float def) {
  const Uniform* u = U(p, n, 1);
  return u ? u->f[0] : def;
}
int ui(Pass* p, const char* n, int def) {
  auto it = p->uni.find(n);
  if (it == p->uni.end()) return def;
  if (it->second.type == 2 || it->second.type == 4) return it->second.i;
  if (it->second.type == 3) return (int)it->second.u;
  return def;
}
uint32_t uu(Pass* p, const char* n, uint32_t def) {
  auto it = p->uni.find(n);
  if (it == p->uni.end()) return def;
  if (it->second.type == 3) return it->second.u;
  if (it->second.type == 2 || it->second.type == 4) return (uint32_t)it->second.i;
  return def;
}

// A sampler the host bound by name (no texture-unit-0 fallback): optional inputs with no GL counterpart.
Texture* bound_sampler(Pass* p, const char* name) {
  auto it = p->tex.find(name);
  return it != p->tex.end() ? tex_of(it->second) : nullptr;
}
Texture* sampler(Pass* p, const char* name, uint32_t* handle = nullptr) {
  auto it = p->tex.find(name);
  uint32_t h = it != p->tex.end() ? it->second : g.unit0;
  if (handle) *handle = h;
  return tex_of(h);
}

int plane_of(Texture* t, Pass* p, Plane* out, const char* what) {
  if (!t || t->target != PT_TEXTURE_2D || !t->dev)
    return err(PT_ERR_MISSING_TEXTURE, std::string("pass needs 2-D texture '") + what + "'");
  if (t->W != p->W || t->H != p->H)
    return err(PT_ERR_ARG, std::string("texture '") + what + "' size differs from the pass size");
  out->p = (float4*)t->dev;
  out->aux = t->aux_valid ? t->aux : nullptr;
  out->W = t->W;
  out->row0 = t->row0;
  out->rows = t->rows;
  return PT_OK;
}
int att_plane(Pass* p, int k, Plane* out) {
  if ((int)p->att.size() <= k) return err(PT_ERR_ARG, "pass has too few color attachments");
  Texture* t = tex_of(p->att[k]);
  int rc = plane_of(t, p, out, "color attachment");
  if (rc != PT_OK) return rc;
  t->version++;
  t->aux_valid = false;
  return PT_OK;
}
#define TRY(x)                    \
  do {                            \
    int rc_ = (x);                \
    if (rc_ != PT_OK) return rc_; \
  } while (0)

void rows_of(Pass* p, int* y0, int* y1) {
  if (p->y_begin >= 0) {
    *y0 = p->y_begin;
    *y1 = p->y_end;
  } else if (g.band_h > 0 && p->W == g.band_w && p->H == g.band_h) {
    *y0 = g.band_y0;
    *y1 = g.band_y1;
  } else {
    *y0 = 0;
    *y1 = p->H;
  }
}

// sobol (path_tracing.frag:480-495): a per-frame uniform value
float sobol_host(uint32_t d, uint32_t i) {
  static const uint32_t V[8 * 32] = {
#include "sobol_v.inc"
  };
  uint32_t r = 0u;
  for (uint32_t j = 0u; i > 0u; i >>= 1u, j++)
    if ((i & 1u) == 1u) r ^= V[j + d * 32u];
  return (float)r * (1.0f / (float)0xFFFFFFFFu);
}

int copy_plane(Texture* dst, Texture* src, Pass* p, int y0, int y1) {
  if (!src || !dst || !src->dev || !dst->dev) return err(PT_ERR_MISSING_TEXTURE, "copy: unbound texture");
  if (src->W != dst->W || src->H != dst->H) return err(PT_ERR_ARG, "copy: size mismatch");
  (void)p;
  int a = std::max(y0, std::max(src->row0, dst->row0));
  int b = std::min(y1, std::min(src->row0 + src->rows, dst->row0 + dst->rows));
  if (b > a) {
    size_t rowb = (size_t)src->W * 16;
    HIPCHK(hipMemcpyAsync((char*)dst->dev + (size_t)(a - dst->row0) * rowb,
                          (char*)src->dev + (size_t)(a - src->row0) * rowb, (size_t)(b - a) * rowb,
                          hipMemcpyDeviceToDevice, g.stream));
  }
  dst->version++;
  dst->aux_valid = false;
  if (src->aux_valid && src->aux) {  // keep the compact side plane in step with its texture
    if (!dst->aux) HIPCHK(hipMalloc((void**)&dst->aux, (size_t)dst->W * dst->rows * 4));
    if (b > a) {
      size_t rb = (size_t)src->W * 4;
      HIPCHK(hipMemcpyAsync((char*)dst->aux + (size_t)(a - dst->row0) * rb, (char*)src->aux + (size_t)(a - src->row0) * rb,
                            (size_t)(b - a) * rb, hipMemcpyDeviceToDevice, g.stream));
    }
    dst->aux_valid = true;
  }
  return PT_OK;
}

// Cost-ordered dispatch (TileSched): the launch records per-tile costs into o.cost and
// runs in the order the previous launch's costs gave (once one exists for this tile
// count); tile_order_finish then sorts the new costs for the next launch.
int tile_order_begin(Pass* p, int ntiles, TileSched* out) {
  TileOrder& o = p->order;
  memset(out, 0, sizeof(*out));
  if (ui(p, "tile_order", 1) == 0 || ntiles <= 0) return PT_OK;  // A/B switch: raster order
  if (o.n != ntiles) {
    if (o.cost) (void)hipFree(o.cost);
    if (o.perm) (void)hipFree(o.perm);
    o.cost = nullptr;
    o.perm = nullptr;
    o.n = 0;
    o.ordered = false;
    HIPCHK(hipMalloc((void**)&o.cost, (size_t)ntiles * 4));
    HIPCHK(hipMalloc((void**)&o.perm, (size_t)ntiles * 4));
    HIPCHK(hipMemsetAsync(o.cost, 0, (size_t)ntiles * 4, g.stream));
    o.n = ntiles;
  }
  out->cost = o.cost;
  out->perm = o.ordered ? o.perm : nullptr;
  out->perm_next = o.perm;
  out->ntiles = ntiles;
  return PT_OK;
}

int tile_order_finish(Pass* p, const TileSched& t) {
  if (!t.cost) return PT_OK;
  int rc = launch_tile_sort(p->order.cost, p->order.perm, p->order.n, g.stream);
  if (rc) return hip_err((hipError_t)rc, "tile order sort");
  p->order.ordered = true;
  return PT_OK;
}

// Scratch of a tile rasteriser (Bins, pt_device.h): allocated once per (items, band) size, its tile counts zeroed
// then (every later launch leaves them at zero: the scatter decrements each one it counted, an overflowed launch's
// fallback clears them); the counters are cleared per launch. `cap` > 0 lowers the pair list's capacity (tests).
int bins_for(RasterBins& b, int n, int W, int y0, int y1, int cap, Bins* out) {
  const int ntiles = ((W + kRTile - 1) / kRTile) * ((std::max(0, y1 - y0) + kRTile - 1) / kRTile);
  if (!b.base || b.ntris != n || b.ntiles != ntiles) {
    if (b.base) (void)hipFree(b.base);
    b = RasterBins{};
    const int pair_cap = (int)std::min<long long>(std::max<long long>(256LL * n, 1 << 22), 1 << 28);
    const int large_cap = std::max(n, 1);
    auto up = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const size_t o_box = 0, o_tmin = o_box + up((size_t)std::max(n, 1) * 16),
                 o_cnt = o_tmin + up((size_t)std::max(n, 1) * 4), o_off = o_cnt + up((size_t)ntiles * 4),
                 o_pairs = o_off + up(((size_t)ntiles + 1) * 4), o_big = o_pairs + up((size_t)pair_cap * 4),
                 o_ctr = o_big + up((size_t)large_cap * 4), total = o_ctr + 256;
    HIPCHK(hipMalloc(&b.base, total));
    char* c = (char*)b.base;
    b.tri_box = (int4*)(c + o_box);
    b.tri_tmin = (float*)(c + o_tmin);
    b.tile_count = (int*)(c + o_cnt);
    b.tile_off = (int*)(c + o_off);
    b.pairs = (int*)(c + o_pairs);
    b.big = (int*)(c + o_big);
    b.ctr = (int*)(c + o_ctr);
    b.ntris = n;
    b.ntiles = ntiles;
    b.pair_cap = pair_cap;
    b.big_cap = large_cap;
    HIPCHK(hipMemsetAsync(b.tile_count, 0, (size_t)ntiles * 4, g.stream));
  }
  HIPCHK(hipMemsetAsync(b.ctr, 0, 16, g.stream));
  Bins& k = *out;
  k.n = n;
  k.box = b.tri_box;
  k.tmin = b.tri_tmin;
  k.tile_count = b.tile_count;
  k.tile_off = b.tile_off;
  k.pairs = b.pairs;
  k.pair_cap = cap > 0 ? std::min(b.pair_cap, cap) : b.pair_cap;
  k.large = b.big;
  k.large_cap = b.big_cap;
  k.ctr = b.ctr;
  k.W = W;
  k.y0 = y0;
  k.y1 = y1;
  return PT_OK;
}

// ------------------------------------------------------------- draw calls ---
// PTParams of a path-tracing pass's draw from its uniforms, samplers and attachments (the wavefront state aside).
int pt_params(Pass* p, PTParams& k, SceneGPU*& sg) {
  memset(&k, 0, sizeof(k));
  k.W = p->W;
  k.H = p->H;
  rows_of(p, &k.y0, &k.y1);
  TRY(att_plane(p, 0, &k.color));
  TRY(att_plane(p, 1, &k.emission));
  TRY(att_plane(p, 2, &k.albedo));
  uint32_t th, nh, lh;
  Texture* tt = sampler(p, "triangles", &th);
  Texture* nt = sampler(p, "nodes", &nh);
  Texture* lt = sampler(p, "pointLights", &lh);
  if (!tt || tt->target != PT_TEXTURE_BUFFER || !nt || nt->target != PT_TEXTURE_BUFFER)
    return err(PT_ERR_MISSING_TEXTURE, "path_tracing needs the 'triangles' and 'nodes' texture buffers");
  TRY(get_scene(tt, th, nt, nh, &sg));
  k.scene.tri_geom = sg->geom;
  k.scene.tri_shade = sg->shade;
  k.scene.bvh = sg->bvh;
  k.scene.root_ref = sg->root_ref;
  k.stack_need = sg->stack_need;
  const Uniform* e = U(p, "eye", 5);
  if (e) memcpy(k.eye, e->f, 12);
  // the any-hit / closest-hit SAH trees hold fine boxes padded for eyes within sg->fine_eye_limit (refine_leaves): an
  // eye further out walks the reference tree, whose boxes are the reference's own
  const bool eye_near = fabsf(k.eye[0]) <= sg->fine_eye_limit && fabsf(k.eye[1]) <= sg->fine_eye_limit &&
                        fabsf(k.eye[2]) <= sg->fine_eye_limit;
  if (ui(p, "shadow_tree", 1) && eye_near) {  // A/B switch: 0 = shadow rays walk the reference tree
    k.scene.bvh_any = sg->bvh_any;
    k.scene.root_any = sg->root_any;
    k.stack_need = std::max(k.stack_need, sg->need_any);
  }
  // wide_bvh = 1 (default): the traversal kernels walk the 4-wide form of the any-hit tree: 28 % fewer node + triangle
  // visits, same bits. With the library built without the SLP vectorizer: 4K 197.7 / 198.9 -> 203.9 / 203.3 fps,
  // surface view 65.4 / 65.2 -> 67.3 / 67.1 (profiles/r03/wide_ab.log; with SLP it measured no faster)
  k.scene.bvh4 = (k.scene.bvh_any && sg->has4 && !(PT_WIDE_SIGNED && sg->nan4) && ui(p, "wide_bvh", 1)) ? sg->bvh4
                                                                                                     : nullptr;
  k.scene.root4 = sg->root4;
  k.scene.root4c = sg->root4c;
  k.scene.ntris = sg->ntris;
  k.scene.leaves = sg->leaves;
  k.scene.nleaves = sg->nleaves;
  if (lt && lt->target == PT_TEXTURE_BUFFER) {
    k.scene.lights = (const float*)lt->dev;
    k.scene.nlights_buf = (int)(lt->bytes / (6 * sizeof(float)));
  }
  // uniform sampler2DArray material_array (path_tracing.frag:331-364); unbound -> fetches read 0
  Texture* ma = sampler(p, "material_array");
  if (ma && ma->target == PT_TEXTURE_2D_ARRAY && ma->dev) {
    k.scene.texarr = (const uint32_t*)ma->dev;
    k.scene.tex_w = ma->W;
    k.scene.tex_h = ma->H;
    k.scene.tex_layers = ma->layers;
  }
  k.scene.use_normal_map = ui(p, "use_normal_map", 0);
  uint32_t hmh = 0, hch = 0;
  Texture* hm = sampler(p, "hdrMap", &hmh);
  Texture* hc = sampler(p, "hdrCache", &hch);
  if (!hm || !hc || !hm->dev || !hc->dev) return err(PT_ERR_MISSING_TEXTURE, "path_tracing needs hdrMap and hdrCache");
  k.hdr = Tex{(const float4*)hm->dev, hm->W, hm->H};
  k.cache = Tex{(const float4*)hc->dev, hc->W, hc->H};
  k.hdr_pdf = Tex{nullptr, 0, 0};
  // A/B switch hdr_merge (default 1): the NEE's radiance and pdf fetches at one direction from one merged texture
  if (ui(p, "hdr_merge", 1) && hm != hc && hm->W == hc->W && hm->H == hc->H && hm->target == PT_TEXTURE_2D &&
      hc->target == PT_TEXTURE_2D && hm->rows == hm->H && hc->rows == hc->H) {
    // Built on the draw's stream, but read by the path tracers of every frame in flight on other streams. A rebuild
    // (first bind, an uploaded hdrMap / hdrCache) writes a buffer no draw still reads: the current one is retired with
    // its readers' events (HdrMerged::uses, recorded after each draw that read it) and a retired buffer whose readers
    // have all finished is taken, or a new one. Every draw's stream waits for the merge's event before reading. No host
    // wait, so a rebuild never blocks on the device (e.g. on RCCL receives in flight for peers). Rebuilds are rare.
    // Staleness follows Texture::version, which uploads bump; a texture wrapped around external device memory
    // (pt_texture2d_wrap) is not tracked, so new contents there must be re-bound (a new handle) to be merged.
    HdrMerged& m = g.hdr_merged[{hmh, hch}];
    const bool stale = !m.buf || m.W != hm->W || m.H != hm->H || m.hdr_dev != hm->dev || m.cache_dev != hc->dev ||
                       m.vh != hm->version || m.vc != hc->version;
    if (stale) {
      if (m.buf && (m.W != hm->W || m.H != hm->H)) {  // a new size (rarer still): the old buffers go once idle
        HIPCHK(hipDeviceSynchronize());
        free_hdr_merged(m);
      }
      if (m.buf) {
        std::vector<hipEvent_t> readers;
        for (auto& u : m.uses) readers.push_back(u.second);
        m.uses.clear();
        m.spare.emplace_back(m.buf, std::move(readers));
        m.buf = nullptr;
      }
      for (size_t i = 0; i < m.spare.size() && !m.buf; ++i) {
        bool idle = true;
        for (hipEvent_t e : m.spare[i].second) idle = idle && hipEventQuery(e) == hipSuccess;
        if (!idle) continue;
        m.buf = m.spare[i].first;
        for (hipEvent_t e : m.spare[i].second) (void)hipEventDestroy(e);
        m.spare.erase(m.spare.begin() + i);
      }
      if (!m.buf) HIPCHK(hipMalloc((void**)&m.buf, (size_t)hm->W * hm->H * sizeof(float4)));
      m.W = hm->W;
      m.H = hm->H;
      if (!m.built) HIPCHK(hipEventCreateWithFlags(&m.built, hipEventDisableTiming));
      const int rc = ptk::launch_hdr_merge((const float4*)hm->dev, (const float4*)hc->dev, m.buf, m.W * m.H, g.stream);
      if (rc) return hip_err((hipError_t)rc, "hdr merge");
      HIPCHK(hipEventRecord(m.built, g.stream));
      m.hdr_dev = hm->dev;
      m.cache_dev = hc->dev;
      m.vh = hm->version;
      m.vc = hc->version;
    }
    HIPCHK(hipStreamWaitEvent(g.stream, m.built, 0));  // (a no-op wait once the merge has run)
    p->hdr_reads = &m;
    k.hdr_pdf = Tex{m.buf, m.W, m.H};
  }
  k.hdrResolution = ui(p, "hdrResolution", hm->W);
  k.pointLightSize = ui(p, "pointLightSize", 0);
  k.frameCounter = uu(p, "frameCounter", 0);
  const Uniform* cr = U(p, "cameraRotate", 6);
  if (cr) memcpy(k.camRot, cr->f, 64);
  else { k.camRot[0] = k.camRot[5] = k.camRot[10] = k.camRot[15] = 1.0f; }
  k.accumulate = ui(p, "accumulate", 0);
  k.clamp_threshold = uf(p, "clamp_threshold", 0.0f);
  k.max_depth = ui(p, "max_tracing_depth", 0);
  if (k.max_depth > 4) return err(PT_ERR_ARG, "max_tracing_depth > 4 indexes past the 8 Sobol dimensions (:463)");
  k.aspect_corrected = ui(p, "aspect_corrected", 0);
  k.prune = ui(p, "prune", 1);
  // A/B switch: 1 = wavefront closest-hit rays walk bvh_any (ties re-walked on the reference tree)
  k.closest_tree = (k.prune && k.scene.bvh_any) ? ui(p, "closest_tree", 1) : 0;
  for (int b = 0; b < 4; ++b) {
    uint32_t i = k.frameCounter + 1u;
    uint32_t gc = i ^ (i >> 1);
    k.sobol_u[b] = sobol_host(2u * b, gc);
    k.sobol_v[b] = sobol_host(2u * b + 1u, gc);
  }
  if (k.accumulate) {
    Texture* lf = sampler(p, "lastFrame");
    if (lf) TRY(plane_of(lf, p, &k.last, "lastFrame"));
  }
  // optional primary-ray bound from this frame's G-buffer (wf_primary), result-preserving
  Texture* hp = bound_sampler(p, "gWorldPos");
  Texture* hn = bound_sampler(p, "gNormalAndLinearZ");
  if (hp && hn && ui(p, "primary_bound", 1)) {
    TRY(plane_of(hp, p, &k.hint_pos, "gWorldPos"));
    TRY(plane_of(hn, p, &k.hint_nd, "gNormalAndLinearZ"));
  }
  // tile subset (PTParams::tile_stride): this pass traces every tile_stride-th 16 x 16 tile of the band
  k.tile_stride = ui(p, "tile_stride", 1);
  k.tile_offset = ui(p, "tile_offset", 0);
  if (wf_subset_tiles(k.W, std::max(0, k.y1 - k.y0), k.tile_stride, k.tile_offset) < 0)
    return err(PT_ERR_ARG, "tile_offset must lie in [0, tile_stride)");
  return PT_OK;
}

// The wavefront-side fields of a path-tracing pass's PTParams: its wavefront state `st` (its own, or its frame's
// share of a batch's), counters, budgets, refill, cost-ordered tiles and the primary rasteriser's bins.
int pt_wf_setup(Pass* p, PTParams& k, SceneGPU* sg, const WFState& st) {
    k.wf = st;
    k.wf.row_cost = p->row_cost;
    k.wf.stats = p->stats;
    k.wf.stats_n = p->stats_n;
    // > 0: shadow rays past this many visits finish in the wave-cooperative walk (A/B switch; off: with frames
    // in flight it measured slower)
    k.wf.shadow_budget = (uint32_t)ui(p, "shadow_budget", 0);
    // > 0: bounce rays past this many visits finish in the wave-cooperative closest-hit walk (refill kernel only)
    k.wf.closest_budget = (uint32_t)ui(p, "closest_budget", 0);
    // percent of the bounce / shadow lists traced by lane-refill waves: 75 pays with frames in flight (the renderer
    // sets it then), 0 (default) keeps the shortest single-frame latency
    k.refill = std::min(100, std::max(0, ui(p, "trace_refill", 0)));
    k.refill_waves = std::max(0, ui(p, "refill_waves", 0));
    k.refill_grid = std::max(0, ui(p, "refill_grid", 0));
    k.list_grid = std::max(0, ui(p, "list_grid", 0));
    const int ntiles = wf_subset_tiles(k.W, std::max(0, k.y1 - k.y0), k.tile_stride, k.tile_offset);  // wf_primary's grid
    TRY(tile_order_begin(p, ntiles, &k.tiles));
    // primary rays by tile-binned rasterisation of the reference leaves (default; 0 = the per-pixel walk); the leaves
    // are binned to every tile of the band, a tile subset rasterises its own tiles
    if (ui(p, "primary_raster", 1)) {
      TRY(bins_for(p->bins, sg->nleaves, k.W, k.y0, k.y1, ui(p, "raster_pair_cap", 0), &k.leaf_bins));
      k.primary_raster = 1;
    }
    return PT_OK;
}

// The side stream and events of path-tracing draws issued on `s` (uniform trace_fork = 1), created on first use: one
// per draw stream, so frames in flight on different streams do not queue behind each other's shadow walks. An entry
// lives until its stream is released (pt_stream_release, which the host's stream pool calls when a renderer gives a
// stream back: ptsvgf.renderer.release_stream) or pt_shutdown, so a handle value a new stream reuses starts afresh.
const ptk::WfFork* wf_fork(Pass* p, hipStream_t s, int* rc) {
  *rc = PT_OK;
  if (!ui(p, "trace_fork", 0)) return nullptr;
  auto it = g.forks.find(s);
  if (it != g.forks.end()) return &it->second;
  ptk::WfFork f{};
  // the side stream runs on the draw stream's CUs (pt_stream_create_cu_masked): a CU mask that keeps CUs free of the
  // traversal launches must hold for the forked walk too
  hipError_t e = hipSuccess;
  int ncu = 0;
  uint32_t mask[16] = {};
  bool masked = false;
  if (s && hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, g.device) == hipSuccess && ncu > 0 &&
      ncu <= 512 && hipExtStreamGetCUMask(s, (uint32_t)((ncu + 31) / 32), mask) == hipSuccess)
    for (int i = 0; i < ncu; ++i) masked = masked || !((mask[i / 32] >> (i % 32)) & 1u);
  // and at the draw stream's queue priority (pt_stream_create_priority)
  int prio = 0;
  if (s) (void)hipStreamGetPriority(s, &prio);
  if (masked) e = hipExtStreamCreateWithCUMask(&f.side, (uint32_t)((ncu + 31) / 32), mask);
  else e = hipStreamCreateWithPriority(&f.side, hipStreamNonBlocking, prio);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&f.fork, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&f.join, hipEventDisableTiming);
  if (e != hipSuccess) {
    if (f.side) (void)hipStreamDestroy(f.side);
    if (f.fork) (void)hipEventDestroy(f.fork);
    *rc = hip_err(e, "trace_fork side stream");
    return nullptr;
  }
  return &(g.forks[s] = f);
}

// after a path-tracing draw that read a merged environment: its stream's use event, so a later rebuild knows when
// this draw no longer reads the buffer (HdrMerged::uses)
int note_hdr_read(Pass* p) {
  HdrMerged* m = p->hdr_reads;
  p->hdr_reads = nullptr;
  if (!m || !m->buf) return PT_OK;
  hipEvent_t& e = m->uses[g.stream];
  if (!e) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIPCHK(hipEventRecord(e, g.stream));
  return PT_OK;
}

int draw_pathtrace(Pass* p) {
  PTParams k;
  SceneGPU* sg = nullptr;
  TRY(pt_params(p, k, sg));
  int rc;
  if (ui(p, "pt_kernel", 0) == 1) {  // 1: single megakernel (kernels_pt.hip), kept for A/B
    if (k.tile_stride != 1) return err(PT_ERR_ARG, "tile subsets need the wavefront path tracer");
    if (k.stack_need >= kStack)
      return err(PT_ERR_ARG, "the megakernel (pt_kernel=1) walks a 32-entry LDS stack; this BVH is deeper: use the "
                             "wavefront path tracer (pt_kernel=0, the default)");
    rc = launch_pathtrace(k, g.stream);
  } else {                            // 0: wavefront (kernels_wavefront.hip), production
    TRY(wf_alloc(p->wf, k.W, std::max(0, k.y1 - k.y0)));
    if (wf_spill(p->wf, k.stack_need) != PT_OK) return err(PT_ERR_HIP, "spill stack allocation failed");
    TRY(pt_wf_setup(p, k, sg, p->wf.st));
    const ptk::WfFork* fk = wf_fork(p, g.stream, &rc);
    if (rc) return rc;
    rc = launch_pathtrace_wavefront(k, g.stream, fk);
    if (!rc && k.tiles.cost) p->order.ordered = true;
  }
  if (rc) return hip_err((hipError_t)rc, "pathtrace launch");
  return note_hdr_read(p);
}

// pt_pass_draw_batch: the frames of several path-tracing passes in one wavefront run whose list-driven traversals
// trace every frame's rays per launch. The first pass owns the shared state, sized for its "trace_batch" frames.
int draw_pathtrace_batch(Pass** ps, int n) {
  Pass* h = ps[0];
  PTParams k[kMaxBatch];
  SceneGPU* sg = nullptr;
  for (int b = 0; b < n; ++b) {
    SceneGPU* sb = nullptr;
    TRY(pt_params(ps[b], k[b], sb));
    if (b == 0) sg = sb;
    // the batched traversal launches take their lane-refill share and visit budgets from passes[0] (pt_wf_setup
    // sets k[b].refill and the budgets from these uniforms later): every pass of the batch must agree on them, each
    // compared at its effective value (the default pt_params / pt_wf_setup apply when a pass never set it)
    struct Same { const char* name; int dflt; };
    const Same same[] = {{"trace_refill", 0}, {"shadow_budget", 0}, {"closest_budget", 0}, {"wide_bvh", 1},
                         {"refill_waves", 0}, {"trace_fork", 0}, {"refill_grid", 0}, {"list_grid", 0}};
    bool agree = true;
    for (const Same& u : same) agree = agree && ui(ps[b], u.name, u.dflt) == ui(ps[0], u.name, u.dflt);
    if (sb != sg || k[b].W != k[0].W || k[b].y0 != k[0].y0 || k[b].y1 != k[0].y1 || k[b].max_depth != k[0].max_depth ||
        k[b].scene.bvh_any != k[0].scene.bvh_any || !agree)
      return err(PT_ERR_ARG, "a path-tracing batch needs one scene, size, band, depth and traversal settings");
    // a tile subset (tile_stride / tile_offset) is batched as a whole frame is, provided every frame traces the same
    // subset: the per-frame launches (primaries, bounce-0 shade, finalize) are sized by that subset's tile count
    if (ui(ps[b], "pt_kernel", 0) != 0 || k[b].accumulate || k[b].tile_stride != k[0].tile_stride ||
        k[b].tile_offset != k[0].tile_offset)
      return err(PT_ERR_ARG, "a path-tracing batch needs the wavefront path tracer, one tile subset, no accumulation");
  }
  const int cap = std::max(n, std::min(kMaxBatch, ui(h, "trace_batch", n)));
  TRY(wf_alloc(h->wf, k[0].W, std::max(0, k[0].y1 - k[0].y0), cap));
  if (wf_spill(h->wf, k[0].stack_need) != PT_OK) return err(PT_ERR_HIP, "spill stack allocation failed");
  for (int b = 0; b < n; ++b) TRY(pt_wf_setup(ps[b], k[b], sg, h->wf.stb[b]));
  int rc;
  const ptk::WfFork* fk = wf_fork(h, g.stream, &rc);
  if (rc) return rc;
  rc = launch_pathtrace_wavefront_batch(k, n, g.stream, fk);
  for (int b = 0; b < n && !rc; ++b)
    if (k[b].tiles.cost) ps[b]->order.ordered = true;
  if (rc) return hip_err((hipError_t)rc, "pathtrace batch launch");
  for (int b = 0; b < n; ++b) TRY(note_hdr_read(ps[b]));
  return PT_OK;
}

// The tile flags of a draw of p over rows [k.y0, k.y1): the rows the a-trous passes draw ("atrous_rows_begin" /
// "_end", e.g. a band's ghost-zone margin), default the G-buffer's own rows; they must lie inside them (a tile's flag is
// marked by the G-buffer pixels it holds). Allocates and zeroes them on the fwidth texture; k.tflags null when off.
static int gbuf_flags(Pass* p, Texture* fwt, GBufParams& k) {
  k.tf_y0 = ui(p, "atrous_rows_begin", -1) >= 0 ? ui(p, "atrous_rows_begin", -1) : k.y0;
  k.tf_y1 = ui(p, "atrous_rows_end", -1) >= 0 ? ui(p, "atrous_rows_end", -1) : k.y1;
  if (k.tf_y0 < k.y0 || k.tf_y1 > k.y1 || k.tf_y0 > k.tf_y1)
    return err(PT_ERR_ARG, "atrous_rows_begin / _end outside the G-buffer's rows");
  if (ui(p, "atrous_tile_flags", 1) && k.tf_y1 > k.tf_y0) {
    const size_t nb = ptk::atrous_flag_bytes(k.W, k.tf_y0, k.tf_y1);
    if (fwt->tflags_cap < nb) {
      if (fwt->tflags) (void)hipFree(fwt->tflags);
      fwt->tflags = nullptr;
      fwt->tflags_cap = 0;
      HIPCHK(hipMalloc((void**)&fwt->tflags, nb));
      fwt->tflags_cap = nb;
    }
    HIPCHK(hipMemsetAsync(fwt->tflags, 0, nb, g.stream));
    k.tflags = fwt->tflags;
    for (int si = 0; si < 5; ++si) k.tf_off[si] = (int)ptk::atrous_flag_offset(si, k.W, k.tf_y0, k.tf_y1);
    fwt->tflags_ver = fwt->version;
    fwt->tflags_y0 = k.tf_y0;
    fwt->tflags_y1 = k.tf_y1;
  } else {
    fwt->tflags_ver = 0;
  }
  return PT_OK;
}

int draw_raster(Pass* p) {
  Pass* src = p->raster_src ? pass_of(p->raster_src) : p;
  if (!src) return err(PT_ERR_STATE, "raster pass shares the triangles of a destroyed pass");
  if (src != p && src->raster_src)  // the source became a sharer itself: its own raster scene is stale
    return err(PT_ERR_STATE, "raster pass shares the triangles of a pass that now shares another pass's");
  const RasterScene& rs = src->raster;
  if (!rs.geom && rs.ntris > 0) return err(PT_ERR_STATE, "raster pass not bound");
  GBufParams k;
  memset(&k, 0, sizeof(k));
  k.W = p->W;
  k.H = p->H;
  rows_of(p, &k.y0, &k.y1);
  TRY(att_plane(p, 0, &k.world));
  TRY(att_plane(p, 1, &k.normal_depth));
  TRY(att_plane(p, 2, &k.motion));
  TRY(att_plane(p, 3, &k.fwidth));
  Texture* fwt = tex_of(p->att[3]);
  if (!fwt->aux) HIPCHK(hipMalloc((void**)&fwt->aux, (size_t)fwt->W * fwt->rows * 4));
  k.fwidth_aux = fwt->aux;
  // the a-trous per-tile surface flags of this G-buffer, marked by the G-buffer kernels as they write the pixels
  TRY(gbuf_flags(p, fwt, k));
  k.geom = rs.geom;
  k.nrm = rs.nrm;
  k.bvh = rs.bvh;
  k.root_ref = rs.root_ref;
  k.stack_need = rs.stack_need;
  float V[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1}, P[16], PV[16];
  memcpy(P, V, 64);
  memcpy(PV, V, 64);
  if (const Uniform* u = U(p, "view", 6)) memcpy(V, u->f, 64);
  if (const Uniform* u = U(p, "projection", 6)) memcpy(P, u->f, 64);
  if (const Uniform* u = U(p, "pre_viewproj", 6)) memcpy(PV, u->f, 64);
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) k.invR[r * 3 + c] = V[r * 4 + c];
  for (int r = 0; r < 3; ++r)
    k.eye[r] = -((k.invR[r * 3] * V[12] + k.invR[r * 3 + 1] * V[13]) + k.invR[r * 3 + 2] * V[14]);
  k.P00 = P[0];
  k.P11 = P[5];
  for (int c = 0; c < 4; ++c)
    for (int r = 0; r < 4; ++r)
      k.M[c * 4 + r] = ((P[0 * 4 + r] * V[c * 4 + 0] + P[1 * 4 + r] * V[c * 4 + 1]) + P[2 * 4 + r] * V[c * 4 + 2]) +
                       P[3 * 4 + r] * V[c * 4 + 3];
  memcpy(k.PV, PV, 64);
  if (rs.ntris == 0) k.root_ref = -1;  // empty leaf
  if (p->motion_max) {
    HIPCHK(hipMemsetAsync(p->motion_max, 0, sizeof(uint32_t), g.stream));
    k.motion_max = p->motion_max;
  }
  const int ntiles = ((k.W + 15) / 16) * ((std::max(0, k.y1 - k.y0) + 15) / 16);  // gbuffer_kernel's grid
  if (ui(p, "gbuffer_mode", 1) == 1) {  // tile-binned rasterisation (default); the ray cast on list overflow
    TRY(bins_for(p->bins, rs.ntris, k.W, k.y0, k.y1, ui(p, "raster_pair_cap", 0), &k.bins));
    int rc = launch_gbuffer_raster(k, g.stream);
    if (rc) return hip_err((hipError_t)rc, "gbuffer raster launch");
  } else {  // A/B: the ray cast with cost-ordered tiles
    TRY(tile_order_begin(p, ntiles, &k.tiles));
    int rc = launch_gbuffer(k, g.stream);
    if (rc) return hip_err((hipError_t)rc, "gbuffer launch");
    TRY(tile_order_finish(p, k.tiles));
  }
  fwt->aux_valid = true;
  return PT_OK;
}

int draw_svgf(Pass* p, int kind) {
  int y0, y1;
  rows_of(p, &y0, &y1);
  int rc = 0;
  if (kind == PK_REPROJECT) {
    ReprojParams k;
    memset(&k, 0, sizeof(k));
    k.W = p->W; k.H = p->H; k.y0 = y0; k.y1 = y1;
    TRY(plane_of(sampler(p, "gMotion"), p, &k.motion, "gMotion"));
    TRY(plane_of(sampler(p, "gColor"), p, &k.color, "gColor"));
    TRY(plane_of(sampler(p, "gAlbedo"), p, &k.albedo, "gAlbedo"));
    TRY(plane_of(sampler(p, "gEmission"), p, &k.emission, "gEmission"));
    TRY(plane_of(sampler(p, "gPrevIllum"), p, &k.prev_illum, "gPrevIllum"));
    TRY(plane_of(sampler(p, "gPrevMoments_HistoryLength"), p, &k.prev_moments, "gPrevMoments_HistoryLength"));
    TRY(plane_of(sampler(p, "gNormalAndLinearZ"), p, &k.nd, "gNormalAndLinearZ"));
    TRY(plane_of(sampler(p, "gPrevNormalAndLinearZ"), p, &k.prev_nd, "gPrevNormalAndLinearZ"));
    TRY(plane_of(sampler(p, "gNormalDepthFwidth"), p, &k.fwidth, "gNormalDepthFwidth"));
    TRY(att_plane(p, 0, &k.out_illum));
    TRY(att_plane(p, 1, &k.out_moments));
    k.inv_w = uf(p, "inv_screen_width", 0.0f);
    k.inv_h = uf(p, "inv_screen_height", 0.0f);
    k.depth_thr = uf(p, "depth_threshold", 0.0f);
    k.normal_thr = uf(p, "normal_threshold", 0.0f);
    k.block = ui(p, "reproj_block", 1);  // A/B (0: lin per tap): the same texels either way
    rc = launch_reproject(k, g.stream);
  } else if (kind == PK_VARIANCE) {
    VarianceParams k;
    memset(&k, 0, sizeof(k));
    k.W = p->W; k.H = p->H; k.y0 = y0; k.y1 = y1;
    TRY(plane_of(sampler(p, "gIllumination"), p, &k.illum, "gIllumination"));
    TRY(plane_of(sampler(p, "gMoments_HistoryLength"), p, &k.moments, "gMoments_HistoryLength"));
    TRY(plane_of(sampler(p, "gNormalAndLinearZ"), p, &k.nd, "gNormalAndLinearZ"));
    TRY(plane_of(sampler(p, "gNormalDepthFwidth"), p, &k.fwidth, "gNormalDepthFwidth"));
    TRY(att_plane(p, 0, &k.out));
    k.phi_color = uf(p, "gPhiColor", 0.0f);
    k.phi_normal = uf(p, "gPhiNormal", 0.0f);
    rc = launch_variance(k, g.stream);
  } else if (kind == PK_ATROUS) {
    AtrousParams k;
    memset(&k, 0, sizeof(k));
    k.W = p->W; k.H = p->H; k.y0 = y0; k.y1 = y1;
    TRY(plane_of(sampler(p, "gIllumination"), p, &k.illum, "gIllumination"));
    TRY(plane_of(sampler(p, "gNormalAndLinearZ"), p, &k.nd, "gNormalAndLinearZ"));
    TRY(plane_of(sampler(p, "gNormalDepthFwidth"), p, &k.fwidth, "gNormalDepthFwidth"));
    TRY(att_plane(p, 0, &k.out));
    if (k.out.p == k.illum.p) return err(PT_ERR_ARG, "a-trous output aliases its input (GL feedback loop)");
    k.step = ui(p, "gStepSize", 1);
    k.phi_color = uf(p, "gPhiColor", 0.0f);
    k.phi_normal = uf(p, "gPhiNormal", 0.0f);
    // production tiled kernel: per-tile surface flags, derived once per G-buffer from its depth-fwidth plane
    const int si = k.step == 1 ? 0 : k.step == 2 ? 1 : k.step == 4 ? 2 : k.step == 8 ? 3 : k.step == 16 ? 4 : -1;
    const int av = ui(p, "atrous_variant", 0);
    if (!ui(p, "exact", 0) && av == 0 && ui(p, "atrous_tile_flags", 1) && k.fwidth.aux &&
        si >= 0 && y1 > y0) {
      Texture* ft = sampler(p, "gNormalDepthFwidth");
      const size_t nb = ptk::atrous_flag_bytes(k.W, y0, y1);
      if (ft->tflags_cap < nb) {
        if (ft->tflags) (void)hipFree(ft->tflags);
        ft->tflags = nullptr;
        ft->tflags_cap = 0;
        HIPCHK(hipMalloc((void**)&ft->tflags, nb));
        ft->tflags_cap = nb;
        ft->tflags_ver = 0;
      }
      if (ft->tflags_ver != ft->version || ft->tflags_y0 != y0 || ft->tflags_y1 != y1) {
        const int frc = ptk::atrous_tile_flags(k.fwidth, k.W, y0, y1, ft->tflags, g.stream);
        if (frc) return hip_err((hipError_t)frc, "a-trous tile flags");
        ft->tflags_ver = ft->version;
        ft->tflags_y0 = y0;
        ft->tflags_y1 = y1;
      }
      k.tile_any = ft->tflags + ptk::atrous_flag_offset(si, k.W, y0, y1);
    }
    // fused modulate (fast driver, last iteration): "fuse_modulate" = 1, colour attachment 1 = the modulate target,
    // gAlbedo / gEmission bound; the production kernel writes it from its epilogue, the others launch modulate after
    if (ui(p, "fuse_modulate", 0)) {
      TRY(plane_of(sampler(p, "gAlbedo"), p, &k.albedo, "gAlbedo"));
      TRY(plane_of(sampler(p, "gEmission"), p, &k.emission, "gEmission"));
      TRY(att_plane(p, 1, &k.mod));
      const Plane* mp[3] = {&k.albedo, &k.emission, &k.mod};
      for (const Plane* q : mp)
        if (y0 < std::max(0, q->row0) || y1 > std::min(p->H, q->row0 + q->rows))
          return err(PT_ERR_ARG, "fused modulate: a plane does not store the draw's rows");
      if (k.mod.p == k.illum.p || k.mod.p == k.out.p) return err(PT_ERR_ARG, "fused modulate target aliases the a-trous planes");
    }
    if (ui(p, "exact", 0)) rc = launch_atrous_exact(k, g.stream);          // bit-exact form (tests)
    else if (ui(p, "atrous_variant", 0) == 1) rc = launch_atrous_simple(k, g.stream);  // A/B: generic
    else if (ui(p, "atrous_variant", 0) == 2) rc = launch_atrous_step(k, g.stream);    // A/B: step kernel
    else rc = launch_atrous_fast(k, g.stream);                             // LDS-tiled (production)
    if (rc == PT_OK && k.mod.p && (ui(p, "exact", 0) || ui(p, "atrous_variant", 0) != 0))
      rc = launch_modulate_after(k, g.stream);
  } else if (kind == PK_MODULATE) {
    ModulateParams k;
    memset(&k, 0, sizeof(k));
    k.W = p->W; k.H = p->H; k.y0 = y0; k.y1 = y1;
    TRY(plane_of(sampler(p, "gAlbedo"), p, &k.albedo, "gAlbedo"));
    TRY(plane_of(sampler(p, "gEmission"), p, &k.emission, "gEmission"));
    TRY(plane_of(sampler(p, "gIllumination"), p, &k.illum, "gIllumination"));
    TRY(plane_of(sampler(p, "gNormalAndLinearZ"), p, &k.nd, "gNormalAndLinearZ"));
    TRY(att_plane(p, 0, &k.out));
    rc = launch_modulate(k, g.stream);
  } else if (kind == PK_OUTPUT) {
    OutputParams k;
    memset(&k, 0, sizeof(k));
    k.W = p->W; k.H = p->H; k.y0 = y0; k.y1 = y1;
    TRY(plane_of(sampler(p, "texPass0"), p, &k.in, "texPass0"));
    if (p->att.empty()) return PT_OK;  // default framebuffer: nothing to keep
    TRY(att_plane(p, 0, &k.out));
    rc = launch_output(k, g.stream);
  } else if (kind == PK_TAA) {
    TAAParams k;
    memset(&k, 0, sizeof(k));
    k.W = p->W; k.H = p->H; k.y0 = y0; k.y1 = y1;
    TRY(plane_of(sampler(p, "currentColor"), p, &k.cur, "currentColor"));
    TRY(plane_of(sampler(p, "previousColor"), p, &k.prev, "previousColor"));
    TRY(plane_of(sampler(p, "velocityTexture"), p, &k.vel, "velocityTexture"));
    TRY(plane_of(sampler(p, "normal_depth"), p, &k.nd, "normal_depth"));
    TRY(att_plane(p, 0, &k.out));
    k.frameCounter = uu(p, "frameCounter", 0);
    rc = launch_taa(k, g.stream);
  } else if (kind == PK_BLIT) {
    if (p->att.empty()) return err(PT_ERR_ARG, "bilt pass without attachment");
    TRY(copy_plane(tex_of(p->att[0]), sampler(p, "in_texture"), p, y0, y1));
  } else if (kind == PK_SAVE) {
    const char* names[5] = {"texPass0", "texPass1", "texPass2", "accColor", "taaOutput"};
    for (int i = 0; i < 5 && i < (int)p->att.size(); ++i)
      TRY(copy_plane(tex_of(p->att[i]), sampler(p, names[i]), p, y0, y1));
  }
  return rc ? hip_err((hipError_t)rc, "kernel launch") : PT_OK;
}

Uniform* set_u(uint32_t pass, const char* name, int type, int* rc) {
  *rc = ensure_init();
  if (*rc != PT_OK) return nullptr;
  Pass* p = pass_of(pass);
  if (!p) { *rc = err(PT_ERR_INVALID_HANDLE, "invalid pass"); return nullptr; }
  if (!name) { *rc = err(PT_ERR_ARG, "null uniform name"); return nullptr; }
  Uniform& u = p->uni[name];
  u.type = type;
  return &u;
}

}  // namespace

// ================================================================= C ABI ===
ptk::LbvhWork g_lbvh;  // GPU BVH builder scratch (grows, reused across rebuilds)

// Replace a texbuffer's contents with `bytes` of device data (device + host copy), as a fresh upload would.
static int texbuffer_take(Texture* t, const void* dev_src, size_t bytes) {
  if (t->bytes != bytes || !t->dev) {
    if (t->owned && t->dev) (void)hipFree(t->dev);
    t->dev = nullptr;
    if (bytes) HIPCHK(hipMalloc(&t->dev, bytes));
    t->owned = true;
  }
  t->bytes = bytes;
  t->W = (int)(bytes / 12);
  t->host.resize(bytes);
  if (bytes) {
    HIPCHK(hipMemcpyAsync(t->dev, dev_src, bytes, hipMemcpyDeviceToDevice, g.stream));
    HIPCHK(hipMemcpyAsync(t->host.data(), dev_src, bytes, hipMemcpyDeviceToHost, g.stream));
  }
  t->version++;
  t->lbvh = true;
  return PT_OK;
}

extern "C" {

int pt_tree_check(const float* node_enc, int nnodes, const float* tri_enc, int ntris, int collapse, int treelet,
                  double* out, int nout) {
  return tree_check(node_enc, nnodes, tri_enc, ntris, collapse, treelet, out, nout);
}

const char* pt_last_error(void) { return g_err.c_str(); }
int pt_version(void) { return 1; }

int pt_init(int device) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  if (g.init) return PT_OK;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return err(PT_ERR_NO_DEVICE, "no HIP device visible");
  if (device < 0 || device >= n) return err(PT_ERR_ARG, "device index out of range");
  HIPCHK(hipSetDevice(device));
  HIPCHK(hipStreamCreateWithFlags(&g.own, hipStreamNonBlocking));
  if (PT_WIDE_SIGNED) {
    const int sub = ptk::subnormal_probe(g.own);
    if (sub != 1) {
      (void)hipStreamDestroy(g.own);
      g.own = nullptr;
      return sub == 0 ? err(PT_ERR_STATE, "walk kernels flush f32 subnormals: PT_WIDE_SIGNED needs them kept")
                      : err(PT_ERR_HIP, "subnormal probe failed");
    }
  }
  g.stream = g.own;
  g.device = device;
  g.init = true;
  return PT_OK;
}

int pt_shutdown(void) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  if (!g.init) return PT_OK;
  (void)hipDeviceSynchronize();
  for (auto& kv : g.textures) {
    Texture* t = kv.second.get();
    if (t->owned && t->dev) (void)hipFree(t->dev);
    if (t->aux) (void)hipFree(t->aux);
    if (t->tflags) (void)hipFree(t->tflags);
  }
  for (auto& kv : g.passes) {
    Pass* p = kv.second.get();
    if (p->raster.geom) (void)hipFree(p->raster.geom);
    if (p->raster.nrm) (void)hipFree(p->raster.nrm);
    if (p->raster.bvh) (void)hipFree(p->raster.bvh);
    if (p->bins.base) (void)hipFree(p->bins.base);
    if (p->wf.base) (void)hipFree(p->wf.base);
    if (p->wf.spill) (void)hipFree(p->wf.spill);
    if (p->order.cost) (void)hipFree(p->order.cost);
    if (p->order.perm) (void)hipFree(p->order.perm);
    if (p->ev0) (void)hipEventDestroy(p->ev0);
    if (p->ev1) (void)hipEventDestroy(p->ev1);
  }
  for (auto& kv : g.scenes) free_scene(kv.second);
  for (auto& kv : g.hdr_merged) free_hdr_merged(kv.second);
  g.hdr_merged.clear();
  for (auto& kv : g.forks) {
    (void)hipEventDestroy(kv.second.fork);
    (void)hipEventDestroy(kv.second.join);
    (void)hipStreamDestroy(kv.second.side);
  }
  g.forks.clear();
  if (g_lbvh.base) (void)hipFree(g_lbvh.base);
  g_lbvh = ptk::LbvhWork{};
  if (g.own) (void)hipStreamDestroy(g.own);
  g = Lib();
  return PT_OK;
}

int pt_set_stream(void* s) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  TRY(ensure_init());
  // s is used as given: NULL is the HIP default (null) stream, which is torch's default stream.
  g.stream = (hipStream_t)s;
  return PT_OK;
}

int pt_stream_release(void* s) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  TRY(ensure_init());
  hipStream_t st = (hipStream_t)s;
  if (st == g.own) return err(PT_ERR_ARG, "the library's own stream is not released");
  auto it = g.forks.find(st);
  if (it != g.forks.end()) {  // its side stream's work was joined into st; wait for that side stream only
    (void)hipStreamSynchronize(it->second.side);
    (void)hipEventDestroy(it->second.fork);
    (void)hipEventDestroy(it->second.join);
    (void)hipStreamDestroy(it->second.side);
    g.forks.erase(it);
  }
  for (auto& kv : g.hdr_merged) {  // the stream's last read of a merged environment: done before the entry goes
    auto u = kv.second.uses.find(st);
    if (u == kv.second.uses.end()) continue;
    (void)hipEventSynchronize(u->second);
    (void)hipEventDestroy(u->second);
    kv.second.uses.erase(u);
  }
  if (g.stream == st) g.stream = g.own;
  return PT_OK;
}

int pt_stream_create_cu_masked(uint32_t words, const uint32_t* mask, void** out) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  TRY(ensure_init());
  if (!mask || !out || words == 0) return err(PT_ERR_ARG, "CU mask and output needed");
  hipStream_t s = nullptr;
  HIPCHK(hipExtStreamCreateWithCUMask(&s, words, mask));  // (the size counts uint32 words)
  *out = (void*)s;
  return PT_OK;
}

int pt_stream_create_priority(int priority, void** out) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  TRY(ensure_init());
  if (!out) return err(PT_ERR_ARG, "output needed");
  int least = 0, greatest = 0;
  HIPCHK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  // numerically lower = higher priority; clamp into [greatest, least]
  priority = std::min(std::max(priority, std::min(least, greatest)), std::max(least, greatest));
  hipStream_t s = nullptr;
  HIPCHK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority));
  *out = (void*)s;
  return PT_OK;
}

int pt_stream_priority_range(int* least, int* greatest) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  TRY(ensure_init());
  if (!least || !greatest) return err(PT_ERR_ARG, "null output");
  HIPCHK(hipDeviceGetStreamPriorityRange(least, greatest));
  return PT_OK;
}

int pt_stream_destroy(void* s) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  TRY(ensure_init());
  if (!s) return err(PT_ERR_ARG, "null stream");
  TRY(pt_stream_release(s));
  HIPCHK(hipStreamSynchronize((hipStream_t)s));
  HIPCHK(hipStreamDestroy((hipStream_t)s));
  return PT_OK;
}

int pt_device_cus(int* n) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  TRY(ensure_init());
  if (!n) return err(PT_ERR_ARG, "null output");
  HIPCHK(hipDeviceGetAttribute(n, hipDeviceAttributeMultiprocessorCount, g.device));
  return PT_OK;
}

int pt_use_own_stream(void) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  TRY(ensure_init());
  g.stream = g.own;
  return PT_OK;
}

int pt_sync(void) {
  TRY(ensure_init());
  HIPCHK(hipStreamSynchronize(g.stream));
  return PT_OK;
}

int pt_set_band(int fw, int fh, int y0, int y1, int row0, int rows) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  if (fw <= 0 || fh <= 0 || y0 < 0 || y1 > fh || y0 >= y1 || row0 < 0 || rows <= 0 || row0 + rows > fh ||
      row0 > y0 || row0 + rows < y1)
    return err(PT_ERR_ARG, "pt_set_band: inconsistent band");
  g.band_w = fw; g.band_h = fh; g.band_y0 = y0; g.band_y1 = y1; g.band_row0 = row0; g.band_rows = rows;
  return PT_OK;
}

int pt_set_profiling(int on) {
  g.profiling = on != 0;
  return PT_OK;
}

int pt_program_create(const char* frag, const char* vert, uint32_t* out) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  TRY(ensure_init());
  if (!out) return err(PT_ERR_ARG, "null out pointer");
  std::string f = basename_of(frag), v = basename_of(vert);
  static const std::map<std::string, int> kinds = {
      {"path_tracing.frag", PK_PATHTRACE}, {"svgf_reproject.frag", PK_REPROJECT},
      {"svgf_variance.frag", PK_VARIANCE}, {"svgf_Atrous.frag", PK_ATROUS},
      {"svgf_modulate.frag", PK_MODULATE}, {"bilt.frag", PK_BLIT},
      {"save_frame_data.frag", PK_SAVE},   {"output_pass.frag", PK_OUTPUT},
      {"taa.frag", PK_TAA},                {"rasterize_frag.frag", PK_RASTER}};
  auto it = kinds.find(f);
  if (it == kinds.end()) return err(PT_ERR_UNKNOWN_PROGRAM, "no HIP kernel for fragment shader '" + f + "'");
  const char* want = it->second == PK_RASTER ? "rasterize_vert.vert" : "vert.vert";
  if (v != want) return err(PT_ERR_UNKNOWN_PROGRAM, "'" + f + "' must be linked with '" + want + "'");
  uint32_t h = g.next++;
  g.programs[h] = it->second;
  *out = h;
  return PT_OK;
}

static int new_texture(std::unique_ptr<Texture> t, uint32_t* out) {
  uint32_t h = g.next++;
  g.textures[h] = std::move(t);
  *out = h;
  return PT_OK;
}

int pt_texture2d_create(int w, int h, uint32_t* out) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  TRY(ensure_init());
  if (w <= 0 || h <= 0 || !out) return err(PT_ERR_ARG, "pt_texture2d_create: bad size");
  auto t = std::make_unique<Texture>();
  t->W = w;
  t->H = h;
  if (g.band_h > 0 && w == g.band_w && h == g.band_h) {
    t->row0 = g.band_row0;
    t->rows = g.band_rows;
  } else {
    t->row0 = 0;
    t->rows = h;
  }
  t->bytes = (size_t)w * t->rows * 16;
  HIPCHK(hipMalloc(&t->dev, t->bytes));
  HIPCHK(hipMemsetAsync(t->dev, 0, t->bytes, g.stream));  // GL leaves it undefined; the build zeroes
  return new_texture(std::move(t), out);
}

int pt_texture2d_wrap(void* ptr, int w, int h, uint32_t* out) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  TRY(ensure_init());
  if (!ptr || w <= 0 || h <= 0 || !out) return err(PT_ERR_ARG, "pt_texture2d_wrap: bad argument");
  auto t = std::make_unique<Texture>();
  t->W = w;
  t->H = h;
  if (g.band_h > 0 && w == g.band_w && h == g.band_h) {
    t->row0 = g.band_row0;
    t->rows = g.band_rows;
  } else {
    t->rows = h;
  }
  t->bytes = (size_t)w * t->rows * 16;
  t->dev = ptr;
  t->owned = false;
  return new_texture(std::move(t), out);
}

int pt_texture2d_upload(uint32_t tex, int w, int h, uint32_t fmt, const float* data) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  TRY(ensure_init());
  Texture* t = tex_of(tex);
  if (!t || t->target != PT_TEXTURE_2D) return err(PT_ERR_INVALID_HANDLE, "invalid 2-D texture");
  if (!data) return err(PT_ERR_ARG, "null data");
  if (fmt != PT_RGB32F && fmt != PT_RGBA32F && fmt != PT_RGB && fmt != PT_RGBA)
    return err(PT_ERR_FORMAT, "upload format must be RGB32F or RGBA32F");
  int nch = (fmt == PT_RGB32F || fmt == PT_RGB) ? 3 : 4;
  if (w != t->W || h != t->H) {  // glTexImage2D respecifies the image
    if (t->owned && t->dev) HIPCHK(hipFree(t->dev));
    if (!t->owned) return err(PT_ERR_ARG, "cannot resize a wrapped texture");
    t->W = w; t->H = h; t->row0 = 0; t->rows = h;
    if (g.band_h > 0 && w == g.band_w && h == g.band_h) { t->row0 = g.band_row0; t->rows = g.band_rows; }
    t->bytes = (size_t)w * t->rows * 16;
    HIPCHK(hipMalloc(&t->dev, t->bytes));
  }
  std::vector<float4> buf((size_t)w * t->rows);
  for (int r = 0; r < t->rows; ++r) {
    const float* src = data + ((size_t)(t->row0 + r) * w) * nch;
    for (int x = 0; x < w; ++x) {
      const float* q = src + (size_t)x * nch;
      buf[(size_t)r * w + x] = float4{q[0], q[1], q[2], nch == 4 ? q[3] : 1.0f};
    }
  }
  HIPCHK(hipMemcpyAsync(t->dev, buf.data(), t->bytes, hipMemcpyHostToDevice, g.stream));
  HIPCHK(hipStreamSynchronize(g.stream));
  t->version++;
  t->aux_valid = false;
  return PT_OK;
}

int pt_texture_upload_rgba(uint32_t tex, const float* data, size_t bytes) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  TRY(ensure_init());
  Texture* t = tex_of(tex);
  if (!t || t->target != PT_TEXTURE_2D) return err(PT_ERR_INVALID_HANDLE, "invalid 2-D texture");
  if (!data || bytes != t->bytes) return err(PT_ERR_ARG, "upload size must equal the stored rows");
  HIPCHK(hipMemcpyAsync(t->dev, data, bytes, hipMemcpyHostToDevice, g.stream));
  HIPCHK(hipStreamSynchronize(g.stream));
  t->version++;
  t->aux_valid = false;
  return PT_OK;
}

int pt_texbuffer_create(const void* data, size_t bytes, uint32_t fmt, uint32_t* out) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  TRY(ensure_init());
  if (fmt != PT_RGB32F) return err(PT_ERR_FORMAT, "texture buffers are RGB32F (main.cpp:142,151,168)");
  if ((!data && bytes) || bytes % 12 || !out) return err(PT_ERR_ARG, "texbuffer size must be whole RGB32F texels");
  auto t = std::make_unique<Texture>();
  t->target = PT_TEXTURE_BUFFER;
  t->bytes = bytes;
  t->W = (int)(bytes / 12);
  t->H = 1;
  t->rows = 1;
  if (bytes) {
    t->host.assign((const uint8_t*)data, (const uint8_t*)data + bytes);
    HIPCHK(hipMalloc(&t->dev, bytes));
    HIPCHK(hipMemcpy(t->dev, data, bytes, hipMemcpyHostToDevice));
  }
  return new_texture(std::move(t), out);
}

int pt_bvh_build(uint32_t tri_in, int leaf_n, int ploc_radius, uint32_t tri_out, uint32_t node_out, int* out_nodes,
                 float* out_ms) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  TRY(ensure_init());
  Texture *ti = tex_of(tri_in), *to = tex_of(tri_out), *no = tex_of(node_out);
  if (!ti || !to || !no || ti->target != PT_TEXTURE_BUFFER || to->target != PT_TEXTURE_BUFFER ||
      no->target != PT_TEXTURE_BUFFER)
    return err(PT_ERR_ARG, "pt_bvh_build: tri_in, tri_out and node_out must be texture buffers");
  if (tri_in == tri_out || tri_in == node_out || tri_out == node_out)
    return err(PT_ERR_ARG, "pt_bvh_build: tri_in, tri_out and node_out must be three different buffers");
  if (leaf_n < 1 || leaf_n > 15) return err(PT_ERR_ARG, "pt_bvh_build: leaf_n must be in [1, 15]");
  if (ploc_radius < 0 || ploc_radius > 256) return err(PT_ERR_ARG, "pt_bvh_build: ploc_radius must be in [0, 256]");
  if (ti->bytes == 0 || ti->bytes % (45 * sizeof(float)) || !ti->dev)
    return err(PT_ERR_FORMAT, "pt_bvh_build: tri_in must hold whole Triangle_encoded records (45 floats)");
  const size_t nt = ti->bytes / (45 * sizeof(float));
  if (nt > (1u << 24)) return err(PT_ERR_ARG, "pt_bvh_build: more than 2^24 triangles (float-encoded indices)");
  const int n = (int)nt;
  float *tbuf = nullptr, *nbuf = nullptr;
  HIPCHK(hipMalloc(&tbuf, nt * 45 * sizeof(float)));
  if (hipMalloc(&nbuf, (size_t)2 * n * 12 * sizeof(float)) != hipSuccess) {
    (void)hipFree(tbuf);
    return err(PT_ERR_HIP, "pt_bvh_build: out of device memory");
  }
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (out_ms) {
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, g.stream);
  }
  int nodes = 0;
  int rc = ptk::lbvh_build(g_lbvh, (const float*)ti->dev, ptk::kTriEncoded, n, leaf_n, ploc_radius, tbuf, nbuf,
                           nullptr, &nodes, g.stream);
  if (out_ms) {
    (void)hipEventRecord(e1, g.stream);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(out_ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
  }
  if (rc == 0) rc = texbuffer_take(to, tbuf, nt * 45 * sizeof(float));
  else rc = hip_err((hipError_t)rc, "lbvh_build");
  if (rc == PT_OK) rc = texbuffer_take(no, nbuf, (size_t)nodes * 12 * sizeof(float));
  if (rc == PT_OK) {
    hipError_t e = hipStreamSynchronize(g.stream);
    if (e != hipSuccess) rc = hip_err(e, "pt_bvh_build");
  }
  (void)hipFree(tbuf);
  (void)hipFree(nbuf);
  if (rc == PT_OK && out_nodes) *out_nodes = nodes;
  return rc;
}

int pt_texarray_create(int w, int h, int layers, uint32_t* out) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  TRY(ensure_init());
  if (w <= 0 || h <= 0 || layers <= 0 || !out) return err(PT_ERR_ARG, "pt_texarray_create: bad size");
  auto t = std::make_unique<Texture>();
  t->target = PT_TEXTURE_2D_ARRAY;
  t->W = w; t->H = h; t->rows = h; t->layers = layers;
  t->bytes = (size_t)w * h * layers * 4;
  HIPCHK(hipMalloc(&t->dev, t->bytes));
  HIPCHK(hipMemset(t->dev, 0, t->bytes));
  return new_texture(std::move(t), out);
}

int pt_texarray_upload_layer(uint32_t tex, int layer, int w, int h, int ch, const uint8_t* data) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  TRY(ensure_init());
  Texture* t = tex_of(tex);
  if (!t || t->target != PT_TEXTURE_2D_ARRAY) return err(PT_ERR_INVALID_HANDLE, "invalid texture array");
  if (!data || layer < 0 || layer >= t->layers || w > t->W || h > t->H || (ch != 3 && ch != 4))
    return err(PT_ERR_ARG, "pt_texarray_upload_layer: bad argument");
  // glTexSubImage3D at the origin (help_func.h:12): a w x h sub-rectangle of the layer
  std::vector<uint8_t> row((size_t)w * 4);
  for (int y = 0; y < h; ++y) {
    for (int x = 0; x < w; ++x) {
      const uint8_t* q = data + ((size_t)y * w + x) * ch;
      row[4 * x] = q[0]; row[4 * x + 1] = q[1]; row[4 * x + 2] = q[2]; row[4 * x + 3] = ch == 4 ? q[3] : 255;
    }
    HIPCHK(hipMemcpy((char*)t->dev + (((size_t)layer * t->H + y) * t->W) * 4, row.data(), row.size(),
                     hipMemcpyHostToDevice));
  }
  t->version++;
  return PT_OK;
}

int pt_texture_readback(uint32_t tex, float* out, size_t bytes) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  TRY(ensure_init());
  Texture* t = tex_of(tex);
  if (!t || !t->dev) return err(PT_ERR_INVALID_HANDLE, "invalid texture");
  if (!out || bytes < t->bytes) return err(PT_ERR_ARG, "readback buffer too small");
  HIPCHK(hipDeviceSynchronize());  // every stream: a frame may be in flight on another renderer's stream
  HIPCHK(hipMemcpy(out, t->dev, t->bytes, hipMemcpyDeviceToHost));
  return PT_OK;
}

int pt_texture_device_ptr(uint32_t tex, void** out) {
  Texture* t = tex_of(tex);
  if (!t || !out) return err(PT_ERR_INVALID_HANDLE, "invalid texture");
  *out = t->dev;
  return PT_OK;
}

int pt_texture_info(uint32_t tex, int* w, int* h, int* row0) {
  Texture* t = tex_of(tex);
  if (!t) return err(PT_ERR_INVALID_HANDLE, "invalid texture");
  if (w) *w = t->W;
  if (h) *h = t->rows;
  if (row0) *row0 = t->row0;
  return PT_OK;
}

int pt_texture_destroy(uint32_t tex) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  auto it = g.textures.find(tex);
  if (it == g.textures.end()) return err(PT_ERR_INVALID_HANDLE, "invalid texture");
  (void)hipStreamSynchronize(g.stream);
  if (it->second->owned && it->second->dev) (void)hipFree(it->second->dev);
  if (it->second->aux) (void)hipFree(it->second->aux);
  if (it->second->tflags) (void)hipFree(it->second->tflags);
  g.textures.erase(it);
  for (auto hm = g.hdr_merged.begin(); hm != g.hdr_merged.end();) {  // merged environments built from it
    if (hm->first.first == tex || hm->first.second == tex) {
      (void)hipDeviceSynchronize();  // its readers may run on any stream
      free_hdr_merged(hm->second);
      hm = g.hdr_merged.erase(hm);
    } else {
      ++hm;
    }
  }
  // the device scenes decoded from this buffer (keyed by (triangles, nodes) handles) go with it
  for (auto sc = g.scenes.begin(); sc != g.scenes.end();) {
    if (sc->first.first == tex || sc->first.second == tex) {
      free_scene(sc->second);
      sc = g.scenes.erase(sc);
    } else {
      ++sc;
    }
  }
  return PT_OK;
}

int pt_pass_create(uint32_t program, int w, int h, uint32_t* out) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  TRY(ensure_init());
  if (!g.programs.count(program)) return err(PT_ERR_INVALID_HANDLE, "invalid program");
  if (w <= 0 || h <= 0 || !out) return err(PT_ERR_ARG, "pt_pass_create: bad size");
  auto p = std::make_unique<Pass>();
  p->program = program;
  p->W = w;
  p->H = h;
  uint32_t hnd = g.next++;
  g.passes[hnd] = std::move(p);
  *out = hnd;
  return PT_OK;
}

int pt_pass_add_color_attachment(uint32_t pass, uint32_t tex) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  Pass* p = pass_of(pass);
  if (!p) return err(PT_ERR_INVALID_HANDLE, "invalid pass");
  if (!tex_of(tex)) return err(PT_ERR_INVALID_HANDLE, "invalid texture");
  p->att.push_back(tex);
  return PT_OK;
}

int pt_pass_bind(uint32_t pass, int final_pass) {
  Pass* p = pass_of(pass);
  if (!p) return err(PT_ERR_INVALID_HANDLE, "invalid pass");
  p->bound = true;
  p->final_pass = final_pass != 0;
  return PT_OK;
}

int pt_raster_pass_bind(uint32_t pass, const float* verts, size_t n_floats) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  TRY(ensure_init());
  Pass* p = pass_of(pass);
  if (!p) return err(PT_ERR_INVALID_HANDLE, "invalid pass");
  if (g.programs[p->program] != PK_RASTER) return err(PT_ERR_ARG, "not a rasterize pass");
  if (n_floats % 18) return err(PT_ERR_ARG, "vertex list must be whole triangles of pos3+nrm3");
  int ntris = (int)(n_floats / 18);
  p->raster.ntris = ntris;
  p->raster_src = 0;
  p->bound = true;
  if (ntris == 0) return PT_OK;
  // SAH tree over the raster triangles (sah_build: the walk's answer does not depend on the tree);
  // geom in leaf order, objIndex = original index (the depth-test tie rule)
  std::vector<SahPrim> pr((size_t)ntris);
  for (int i = 0; i < ntris; ++i) {
    const float* q = verts + (size_t)i * 18;
    for (int a = 0; a < 3; ++a) {
      pr[i].lo[a] = std::min(q[a], std::min(q[6 + a], q[12 + a]));
      pr[i].hi[a] = std::max(q[a], std::max(q[6 + a], q[12 + a]));
    }
    pr[i].weight = 1;
    pr[i].ref = i;
  }
  std::vector<SahNode> tree;
  tree.reserve(2 * (size_t)ntris);
  sah_build(pr, 0, ntris, 8, tree);  // leaves of <= 8 (measured: 2 and 4 slower, tools/exp_tree_ab.sh)
  using namespace glsl;
  std::vector<float4> geom((size_t)ntris * 4), nrm((size_t)ntris * 3);
  for (int k = 0; k < ntris; ++k) {
    const int oi = pr[k].ref;
    const float* f = verts + (size_t)oi * 18;
    v3 p1 = mk(f[0], f[1], f[2]), p2 = mk(f[6], f[7], f[8]), p3 = mk(f[12], f[13], f[14]);
    v3 e1 = sub(p2, p1), e2 = sub(p3, p1), ng = cross(e1, e2);
    float oif;
    memcpy(&oif, &oi, 4);
    float4* q = &geom[(size_t)k * 4];
    q[0] = float4{p1.x, p1.y, p1.z, oif};
    q[1] = float4{e1.x, e1.y, e1.z, 0};
    q[2] = float4{e2.x, e2.y, e2.z, 0};
    q[3] = float4{ng.x, ng.y, ng.z, 0};
    float4* n = &nrm[(size_t)k * 3];
    n[0] = float4{f[3], f[4], f[5], 0};
    n[1] = float4{f[9], f[10], f[11], 0};
    n[2] = float4{f[15], f[16], f[17], 0};
  }
  std::vector<float4> bvh;
  int root = 0;
  TRY(pack_sah(tree, [](int first, int n) { return -(first * 16 + n) - 1; }, bvh, &root, &p->raster.stack_need));
  if (bvh.empty()) bvh.push_back(float4{0, 0, 0, 0});
  TRY(upload_vec(geom, &p->raster.geom));
  TRY(upload_vec(nrm, &p->raster.nrm));
  TRY(upload_vec(bvh, &p->raster.bvh));
  p->raster.root_ref = root;
  return PT_OK;
}

int pt_raster_pass_bind_device(uint32_t pass, const void* dverts, size_t n_floats, int ploc_radius) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  TRY(ensure_init());
  Pass* p = pass_of(pass);
  if (!p) return err(PT_ERR_INVALID_HANDLE, "invalid pass");
  if (g.programs[p->program] != PK_RASTER) return err(PT_ERR_ARG, "not a rasterize pass");
  if (n_floats % 18) return err(PT_ERR_ARG, "vertex list must be whole triangles of pos3+nrm3");
  if (ploc_radius < 0 || ploc_radius > 256) return err(PT_ERR_ARG, "ploc_radius must be in [0, 256]");
  if (n_floats / 18 > (1u << 24)) return err(PT_ERR_ARG, "more than 2^24 raster triangles");
  const int ntris = (int)(n_floats / 18);
  if (ntris > 0 && !dverts) return err(PT_ERR_ARG, "null device vertex list");
  p->raster.ntris = ntris;
  p->raster_src = 0;
  p->bound = true;
  if (ntris == 0) return PT_OK;
  float* nbuf = nullptr;
  int* order = nullptr;
  HIPCHK(hipMalloc(&nbuf, (size_t)2 * ntris * 12 * sizeof(float)));
  if (hipMalloc(&order, (size_t)ntris * sizeof(int)) != hipSuccess) {
    (void)hipFree(nbuf);
    return err(PT_ERR_HIP, "pt_raster_pass_bind_device: out of device memory");
  }
  auto release = [&]() { (void)hipFree(nbuf); (void)hipFree(order); };
  int nodes = 0;
  int rc = ptk::lbvh_build(g_lbvh, (const float*)dverts, ptk::kRasterVerts, ntris, 8, ploc_radius, nullptr, nbuf,
                           order, &nodes, g.stream);
  if (rc) { release(); return hip_err((hipError_t)rc, "raster lbvh_build"); }
  std::vector<float> hn((size_t)nodes * 12);
  if (hipMemcpy(hn.data(), nbuf, hn.size() * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess) {
    release();
    return err(PT_ERR_HIP, "pt_raster_pass_bind_device: node readback");
  }
  std::vector<float4> bvh;
  int root = 0, need = 0;
  rc = pack_bvh(hn.data(), nodes, bvh, &root, ntris, &need);
  if (rc != PT_OK || need >= kStack) {
    // the G-buffer walk's stack holds kStack entries: a deeper device tree (coincident centroids) takes the host
    // bind, whose SAH builder caps the depth; the G-buffer does not depend on the tree
    std::vector<float> hv(n_floats);
    const bool ok = hipMemcpy(hv.data(), dverts, n_floats * sizeof(float), hipMemcpyDeviceToHost) == hipSuccess;
    release();
    if (!ok) return err(PT_ERR_HIP, "pt_raster_pass_bind_device: vertex readback");
    return pt_raster_pass_bind(pass, hv.data(), n_floats);
  }
  if (p->raster.geom) (void)hipFree(p->raster.geom);
  if (p->raster.nrm) (void)hipFree(p->raster.nrm);
  p->raster.geom = p->raster.nrm = nullptr;
  if (hipMalloc((void**)&p->raster.geom, (size_t)ntris * 4 * sizeof(float4)) != hipSuccess ||
      hipMalloc((void**)&p->raster.nrm, (size_t)ntris * 3 * sizeof(float4)) != hipSuccess) {
    release();
    return err(PT_ERR_HIP, "pt_raster_pass_bind_device: out of device memory");
  }
  rc = ptk::decode_raster((const float*)dverts, order, ntris, p->raster.geom, p->raster.nrm, g.stream);
  if (rc) { release(); return hip_err((hipError_t)rc, "decode_raster"); }
  if (bvh.empty()) bvh.push_back(float4{0, 0, 0, 0});
  if ((rc = upload_vec(bvh, &p->raster.bvh)) != PT_OK) { release(); return rc; }
  p->raster.root_ref = root;
  p->raster.stack_need = need;
  // draws of other frames may run on other streams: the records are complete when this returns
  const hipError_t e = hipStreamSynchronize(g.stream);
  release();
  if (e != hipSuccess) return hip_err(e, "pt_raster_pass_bind_device");
  return PT_OK;
}

int pt_raster_pass_share(uint32_t pass, uint32_t src_pass) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  TRY(ensure_init());
  Pass *p = pass_of(pass), *s = pass_of(src_pass);
  if (!p || !s) return err(PT_ERR_INVALID_HANDLE, "invalid pass");
  if (g.programs[p->program] != PK_RASTER || g.programs[s->program] != PK_RASTER)
    return err(PT_ERR_ARG, "pt_raster_pass_share: both passes must be rasterize passes");
  if (pass == src_pass || s->raster_src) return err(PT_ERR_ARG, "pt_raster_pass_share: share from an own-bound pass");
  p->raster_src = src_pass;
  p->bound = true;
  return PT_OK;
}

int pt_raster_pass_adopt(uint32_t pass, int y_begin, int y_end) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  TRY(ensure_init());
  Pass* p = pass_of(pass);
  if (!p) return err(PT_ERR_INVALID_HANDLE, "invalid pass");
  if (g.programs[p->program] != PK_RASTER) return err(PT_ERR_ARG, "pt_raster_pass_adopt: not a rasterize pass");
  if (p->att.size() < 4) return err(PT_ERR_STATE, "pt_raster_pass_adopt: the pass has no G-buffer attachments");
  GBufParams k;
  memset(&k, 0, sizeof(k));
  k.W = p->W;
  k.H = p->H;
  if (y_begin < 0 || y_end > p->H || y_begin > y_end) return err(PT_ERR_ARG, "pt_raster_pass_adopt: bad rows");
  k.y0 = y_begin;
  k.y1 = y_end;
  for (int i = 0; i < 4; ++i) {  // the attachments now hold new texels (their versions move on, as after a draw)
    Plane* dst[4] = {&k.world, &k.normal_depth, &k.motion, &k.fwidth};
    TRY(att_plane(p, i, dst[i]));
  }
  Texture* fwt = tex_of(p->att[3]);
  for (int i : {1, 3}) {
    const Texture* t = tex_of(p->att[i]);
    if (y_begin < t->row0 || y_end > t->row0 + t->rows)
      return err(PT_ERR_ARG, "pt_raster_pass_adopt: rows outside the attachments' stored rows");
  }
  if (!fwt->aux) HIPCHK(hipMalloc((void**)&fwt->aux, (size_t)fwt->W * fwt->rows * 4));
  k.fwidth_aux = fwt->aux;
  TRY(gbuf_flags(p, fwt, k));
  const int rc = ptk::launch_gbuffer_adopt(k, g.stream);
  if (rc) return hip_err((hipError_t)rc, "pt_raster_pass_adopt");
  fwt->aux_valid = true;
  return PT_OK;
}

int pt_tiles_count(int frame_w, int tile_y0, int stride, int offset, int y_begin, int y_end, int64_t* out_pixels) {
  if (!out_pixels || frame_w <= 0 || frame_w % 16 || stride < 1 || offset < 0 || offset >= stride || y_begin > y_end ||
      y_begin < tile_y0)
    return err(PT_ERR_ARG, "pt_tiles_count: width a multiple of 16, 0 <= offset < stride, tile_y0 <= y_begin <= y_end");
  *out_pixels = ptk::shard_pixels(frame_w, tile_y0, stride, offset, y_begin, y_end);
  return PT_OK;
}

int pt_tiles_copy(const uint32_t* tex, int ntex, int tile_y0, int stride, const PtTileSeg* segs, int nseg, int unpack) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  TRY(ensure_init());
  if (!tex || ntex < 1 || ntex > 4 || (nseg > 0 && !segs) || nseg < 0 || stride < 1)
    return err(PT_ERR_ARG, "pt_tiles_copy: 1..4 textures, segments, stride >= 1");
  ptk::ShardCopy c;
  memset(&c, 0, sizeof(c));
  c.tile_y0 = tile_y0;
  c.stride = stride;
  c.nplanes = ntex;
  c.unpack = unpack ? 1 : 0;
  Texture* ts[4] = {nullptr, nullptr, nullptr, nullptr};
  for (int j = 0; j < ntex; ++j) {
    Texture* t = tex_of(tex[j]);
    if (!t || t->target != PT_TEXTURE_2D || !t->dev) return err(PT_ERR_INVALID_HANDLE, "pt_tiles_copy: invalid texture");
    if (j > 0 && t->W != ts[0]->W) return err(PT_ERR_ARG, "pt_tiles_copy: textures of different widths");
    if (t->W % 16) return err(PT_ERR_ARG, "pt_tiles_copy: the frame width must be a multiple of 16");
    ts[j] = t;
    c.plane[j] = (float4*)t->dev;
    c.row0[j] = t->row0;
  }
  c.W = ts[0]->W;
  for (int s = 0; s < nseg; ++s) {
    const PtTileSeg& q = segs[s];
    if (q.offset < 0 || q.offset >= stride || q.y_begin < tile_y0 || q.y_begin > q.y_end || (!q.packed && q.y_end > q.y_begin))
      return err(PT_ERR_ARG, "pt_tiles_copy: bad segment");
    for (int j = 0; j < ntex; ++j)
      if (q.y_end > q.y_begin && (q.y_begin < ts[j]->row0 || q.y_end > ts[j]->row0 + ts[j]->rows))
        return err(PT_ERR_ARG, "pt_tiles_copy: segment rows outside a texture's stored rows");
  }
  for (int s0 = 0; s0 < nseg; s0 += ptk::kShardSegs) {  // one launch per kShardSegs segments
    c.nseg = std::min(ptk::kShardSegs, nseg - s0);
    for (int s = 0; s < c.nseg; ++s) {
      const PtTileSeg& q = segs[s0 + s];
      c.seg[s] = ptk::ShardSeg{q.y_begin, q.y_end, q.offset, (float4*)q.packed};
    }
    const int rc = ptk::launch_shard_copy(c, g.stream);
    if (rc) return hip_err((hipError_t)rc, "pt_tiles_copy");
  }
  if (unpack)
    for (int j = 0; j < ntex; ++j) ts[j]->version++;  // new texels, as after a draw
  return PT_OK;
}

int pt_pass_reset_texture_slot(uint32_t pass) {
  Pass* p = pass_of(pass);
  if (!p) return err(PT_ERR_INVALID_HANDLE, "invalid pass");
  p->slot = 0;
  return PT_OK;
}

int pt_pass_set_texture(uint32_t pass, uint32_t target, uint32_t tex, const char* name) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  Pass* p = pass_of(pass);
  if (!p) return err(PT_ERR_INVALID_HANDLE, "invalid pass");
  Texture* t = tex_of(tex);
  if (!t) return err(PT_ERR_INVALID_HANDLE, "invalid texture");
  if (!name) return err(PT_ERR_ARG, "null sampler name");
  if (target != t->target) return err(PT_ERR_FORMAT, "texture bound to the wrong target");
  if (p->slot == 0) g.unit0 = tex;  // glActiveTexture(GL_TEXTURE0 + slot) is global state
  p->slot++;
  p->tex[name] = tex;
  return PT_OK;
}

int pt_pass_set_uniform_mat4(uint32_t pass, const char* name, const float* m) {
  int rc;
  Uniform* u = set_u(pass, name, 6, &rc);
  if (!u) return rc;
  if (!m) return err(PT_ERR_ARG, "null matrix");
  memcpy(u->f, m, 64);
  return PT_OK;
}
int pt_pass_set_uniform_float(uint32_t pass, const char* name, float v) {
  int rc;
  Uniform* u = set_u(pass, name, 1, &rc);
  if (!u) return rc;
  u->f[0] = v;
  return PT_OK;
}
int pt_pass_set_uniform_int(uint32_t pass, const char* name, int v) {
  int rc;
  Uniform* u = set_u(pass, name, 2, &rc);
  if (!u) return rc;
  u->i = v;
  return PT_OK;
}
int pt_pass_set_uniform_uint(uint32_t pass, const char* name, uint32_t v) {
  int rc;
  Uniform* u = set_u(pass, name, 3, &rc);
  if (!u) return rc;
  u->u = v;
  return PT_OK;
}
int pt_pass_set_uniform_bool(uint32_t pass, const char* name, int v) {
  int rc;
  Uniform* u = set_u(pass, name, 4, &rc);
  if (!u) return rc;
  u->i = v != 0;
  return PT_OK;
}
int pt_pass_set_uniform_vec3(uint32_t pass, const char* name, const float* v) {
  int rc;
  Uniform* u = set_u(pass, name, 5, &rc);
  if (!u) return rc;
  if (!v) return err(PT_ERR_ARG, "null vector");
  memcpy(u->f, v, 12);
  return PT_OK;
}

int pt_pass_set_rows(uint32_t pass, int y0, int y1) {
  Pass* p = pass_of(pass);
  if (!p) return err(PT_ERR_INVALID_HANDLE, "invalid pass");
  if (y0 < 0 && y1 < 0) { p->y_begin = p->y_end = -1; return PT_OK; }
  if (y0 < 0 || y1 > p->H || y0 > y1) return err(PT_ERR_ARG, "pt_pass_set_rows: bad range");
  p->y_begin = y0;
  p->y_end = y1;
  return PT_OK;
}

int pt_pass_set_row_cost(uint32_t pass, void* device_counts) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  Pass* p = pass_of(pass);
  if (!p) return err(PT_ERR_INVALID_HANDLE, "invalid pass");
  p->row_cost = (uint32_t*)device_counts;
  return PT_OK;
}

int pt_pass_set_trace_stats_n(uint32_t pass, void* device_u64, int count) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  Pass* p = pass_of(pass);
  if (!p) return err(PT_ERR_INVALID_HANDLE, "invalid pass");
  if (device_u64 && g.programs[p->program] != PK_PATHTRACE) return err(PT_ERR_ARG, "trace stats need a path-tracing pass");
  if (device_u64 && count <= 0) return err(PT_ERR_ARG, "trace stats buffer of no counters");
  p->stats = (unsigned long long*)device_u64;
  p->stats_n = device_u64 ? std::min(count, (int)kStatCount) : 0;
  return PT_OK;
}

// the entry point as first published took a buffer of 12 counters: it still writes those 12 only
int pt_pass_set_trace_stats(uint32_t pass, void* device_u64) {
  return pt_pass_set_trace_stats_n(pass, device_u64, PT_TRACE_STATS_V1);
}

int pt_trace_stats_count(void) { return kStatCount; }

int pt_pass_set_motion_bound(uint32_t pass, void* device_u32) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  Pass* p = pass_of(pass);
  if (!p) return err(PT_ERR_INVALID_HANDLE, "invalid pass");
  if (device_u32 && g.programs[p->program] != PK_RASTER) return err(PT_ERR_ARG, "motion bound needs a rasterize pass");
  p->motion_max = (uint32_t*)device_u32;
  return PT_OK;
}

int pt_pass_draw(uint32_t pass) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  TRY(ensure_init());
  Pass* p = pass_of(pass);
  if (!p) return err(PT_ERR_INVALID_HANDLE, "invalid pass");
  if (!p->bound) return err(PT_ERR_STATE, "pass drawn before bindData");
  int kind = g.programs[p->program];
  if (g.profiling) {
    if (!p->ev0) { HIPCHK(hipEventCreate(&p->ev0)); HIPCHK(hipEventCreate(&p->ev1)); }
    HIPCHK(hipEventRecord(p->ev0, g.stream));
  }
  int rc;
  if (kind == PK_PATHTRACE) rc = draw_pathtrace(p);
  else if (kind == PK_RASTER) rc = draw_raster(p);
  else rc = draw_svgf(p, kind);
  if (rc != PT_OK) return rc;
  if (g.profiling) {
    HIPCHK(hipEventRecord(p->ev1, g.stream));
    p->timed = true;
  }
  return PT_OK;
}

int pt_pass_draw_batch(const uint32_t* passes, int count) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  TRY(ensure_init());
  if (!passes || count < 1 || count > kMaxBatch) return err(PT_ERR_ARG, "a batch holds 1 to 8 path-tracing passes");
  Pass* ps[kMaxBatch];
  for (int b = 0; b < count; ++b) {
    ps[b] = pass_of(passes[b]);
    if (!ps[b]) return err(PT_ERR_INVALID_HANDLE, "invalid pass");
    if (!ps[b]->bound) return err(PT_ERR_STATE, "pass drawn before bindData");
    if (g.programs[ps[b]->program] != PK_PATHTRACE) return err(PT_ERR_ARG, "a batch holds path-tracing passes only");
    for (int c = 0; c < b; ++c)
      if (ps[c] == ps[b]) return err(PT_ERR_ARG, "a pass appears twice in a batch");
  }
  Pass* h = ps[0];
  if (g.profiling) {  // the batch is timed as the first pass's draw
    if (!h->ev0) { HIPCHK(hipEventCreate(&h->ev0)); HIPCHK(hipEventCreate(&h->ev1)); }
    HIPCHK(hipEventRecord(h->ev0, g.stream));
  }
  TRY(draw_pathtrace_batch(ps, count));
  if (g.profiling) {
    HIPCHK(hipEventRecord(h->ev1, g.stream));
    h->timed = true;
  }
  return PT_OK;
}

int pt_pass_last_ms(uint32_t pass, float* ms) {
  Pass* p = pass_of(pass);
  if (!p || !ms) return err(PT_ERR_INVALID_HANDLE, "invalid pass");
  if (!p->timed) return err(PT_ERR_STATE, "pass has no timed draw (pt_set_profiling(1))");
  HIPCHK(hipEventSynchronize(p->ev1));
  HIPCHK(hipEventElapsedTime(ms, p->ev0, p->ev1));
  return PT_OK;
}

int pt_pass_destroy(uint32_t pass) {
  std::lock_guard<std::recursive_mutex> lk(g_mu);
  auto it = g.passes.find(pass);
  if (it == g.passes.end()) return err(PT_ERR_INVALID_HANDLE, "invalid pass");
  (void)hipStreamSynchronize(g.stream);
  Pass* p = it->second.get();
  if (p->raster.geom) (void)hipFree(p->raster.geom);
  if (p->raster.nrm) (void)hipFree(p->raster.nrm);
  if (p->raster.bvh) (void)hipFree(p->raster.bvh);
  if (p->bins.base) (void)hipFree(p->bins.base);
  if (p->wf.base) (void)hipFree(p->wf.base);
  if (p->wf.spill) (void)hipFree(p->wf.spill);
  if (p->order.cost) (void)hipFree(p->order.cost);
  if (p->order.perm) (void)hipFree(p->order.perm);
  if (p->ev0) (void)hipEventDestroy(p->ev0);
  if (p->ev1) (void)hipEventDestroy(p->ev1);
  g.passes.erase(it);
  return PT_OK;
}

}  // extern "C"

// scene_prep.cpp — host scene preparation (reference layer L1), C ABI in
// include/ptsvgf_scene.h. Runs once at startup on the CPU, exactly as in the
// reference; its output is the data layout the HIP kernels consume.
//
// Bit-compatibility notes (each verified against the reference's own
// known-answer counts, SURVEY.md §8(c): clock 8265 tris / 3010 nodes / 1505
// leaves / depth 15, table 5184 / 2078 / 1039 / 17, table+clock 13449 / 5098):
//  * readObj keeps the max-axis normalisation bug (obj_loader.h:51-52: y/z bounds
//    are taken against maxx/minx) and glm's mat4*vec4 pairwise summation order.
//  * buildBVHwithSAH sorts with std::sort (libstdc++ introsort) on the same
//    comparator keys; std::sort's sequence of moves depends only on comparison
//    outcomes, so sorting an index permutation reproduces the reference's
//    in-place struct sort exactly. Costs use the reference's float/double mix.
//  * all arithmetic is compiled with -ffp-contract=off.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/ptsvgf_scene.h"
#include "glsl_builtins.h"

using glsl::v3;

namespace {

thread_local std::string g_err;
int fail(const std::string& m) {
  g_err = m;
  return -1;
}

struct Tri {
  v3 p1, p2, p3, n1, n2, n3;
  float uv1[2], uv2[2], uv3[2];
  float mat[PTS_MATERIAL_FLOATS];
  int objID;
};

struct Node {
  int left, right, n, index;
  v3 AA, BB;
};

// glm scalar min/max (glm/detail/func_common.inl): min = (y < x) ? y : x, max = (x < y) ? y : x
inline float gmin(float x, float y) { return (y < x) ? y : x; }
inline float gmax(float x, float y) { return (x < y) ? y : x; }

// glm mat4 * vec4 (type_mat4x4.inl): Add0 = m0*v0 + m1*v1; Add1 = m2*v2 + m3*v3; Add0 + Add1
inline v3 xform_point(const float* m, v3 p) {
  float r[3];
  for (int k = 0; k < 3; ++k) {
    float mul0 = m[0 + k] * p.x;
    float mul1 = m[4 + k] * p.y;
    float mul2 = m[8 + k] * p.z;
    float mul3 = m[12 + k] * 1.0f;
    float add0 = mul0 + mul1;
    float add1 = mul2 + mul3;
    r[k] = add0 + add1;
  }
  return glsl::mk(r[0], r[1], r[2]);
}

// glm::normalize = x * inversesqrt(dot(x,x)), inversesqrt = 1/sqrt
inline v3 gnormalize(v3 a) { return glsl::normalize(a); }

}  // namespace

struct pts_scene {
  std::vector<Tri> tris;
  std::vector<float> raster;
  std::vector<Node> nodes;
  bool built = false;
};

// Shared tail of readObj (obj_loader.h:100-161): normals, triangles, raster list.
static void emit_triangles(pts_scene* s, const std::vector<v3>& vertices, const std::vector<int>& indices,
                           const std::vector<int>& tex_indices, const std::vector<float>& texcoords,
                           const float* material, bool smooth, int objIndex) {
  std::vector<v3> normals(vertices.size(), glsl::mk(0, 0, 0));
  for (size_t i = 0; i + 2 < indices.size(); i += 3) {
    v3 p1 = vertices[indices[i]], p2 = vertices[indices[i + 1]], p3 = vertices[indices[i + 2]];
    v3 n = gnormalize(glsl::cross(glsl::sub(p2, p1), glsl::sub(p3, p1)));
    normals[indices[i]] = glsl::add(normals[indices[i]], n);
    normals[indices[i + 1]] = glsl::add(normals[indices[i + 1]], n);
    normals[indices[i + 2]] = glsl::add(normals[indices[i + 2]], n);
  }
  size_t offset = s->tris.size();
  s->tris.resize(offset + indices.size() / 3);
  for (size_t i = 0; i + 2 < indices.size(); i += 3) {
    Tri& t = s->tris[offset + i / 3];
    t.p1 = vertices[indices[i]];
    t.p2 = vertices[indices[i + 1]];
    t.p3 = vertices[indices[i + 2]];
    const int ti[3] = {tex_indices[i], tex_indices[i + 1], tex_indices[i + 2]};
    float* uvs[3] = {t.uv1, t.uv2, t.uv3};
    for (int k = 0; k < 3; ++k) {
      if (ti[k] >= 0 && (size_t)(2 * ti[k] + 1) < texcoords.size()) {
        uvs[k][0] = texcoords[2 * ti[k]];
        uvs[k][1] = texcoords[2 * ti[k] + 1];
      } else {
        uvs[k][0] = uvs[k][1] = 0.0f;
      }
    }
    t.objID = objIndex;
    if (!smooth) {
      v3 n = gnormalize(glsl::cross(glsl::sub(t.p2, t.p1), glsl::sub(t.p3, t.p1)));
      t.n1 = t.n2 = t.n3 = n;
    } else {
      t.n1 = gnormalize(normals[indices[i]]);
      t.n2 = gnormalize(normals[indices[i + 1]]);
      t.n3 = gnormalize(normals[indices[i + 2]]);
    }
    memcpy(t.mat, material, sizeof(t.mat));
    const v3* pv[3] = {&t.p1, &t.p2, &t.p3};
    const v3* nv[3] = {&t.n1, &t.n2, &t.n3};
    for (int k = 0; k < 3; ++k) {
      s->raster.push_back(pv[k]->x);
      s->raster.push_back(pv[k]->y);
      s->raster.push_back(pv[k]->z);
      s->raster.push_back(nv[k]->x);
      s->raster.push_back(nv[k]->y);
      s->raster.push_back(nv[k]->z);
    }
  }
  s->built = false;
}

// ------------------------------------------------------------- BVH (SAH) ---
namespace {

struct Builder {
  std::vector<Tri>& tris;  // permuted in place through `perm`
  std::vector<int> perm;
  std::vector<float> cx, cy, cz;  // comparator keys: (p1+p2+p3)/vec3(3) (BVH.h:25-39)
  std::vector<float> tmin[3], tmax[3];
  std::vector<Node>& nodes;

  Builder(std::vector<Tri>& t, std::vector<Node>& n) : tris(t), nodes(n) {
    size_t N = t.size();
    perm.resize(N);
    cx.resize(N); cy.resize(N); cz.resize(N);
    for (int a = 0; a < 3; ++a) { tmin[a].resize(N); tmax[a].resize(N); }
    for (size_t i = 0; i < N; ++i) {
      perm[i] = (int)i;
      const Tri& q = t[i];
      cx[i] = ((q.p1.x + q.p2.x) + q.p3.x) / 3.0f;
      cy[i] = ((q.p1.y + q.p2.y) + q.p3.y) / 3.0f;
      cz[i] = ((q.p1.z + q.p2.z) + q.p3.z) / 3.0f;
      // glm::min(p1, glm::min(p2, p3)) per axis
      tmin[0][i] = gmin(q.p1.x, gmin(q.p2.x, q.p3.x));
      tmin[1][i] = gmin(q.p1.y, gmin(q.p2.y, q.p3.y));
      tmin[2][i] = gmin(q.p1.z, gmin(q.p2.z, q.p3.z));
      tmax[0][i] = gmax(q.p1.x, gmax(q.p2.x, q.p3.x));
      tmax[1][i] = gmax(q.p1.y, gmax(q.p2.y, q.p3.y));
      tmax[2][i] = gmax(q.p1.z, gmax(q.p2.z, q.p3.z));
    }
  }

  void sort_axis(int l, int r, int axis) {
    const std::vector<float>& key = axis == 0 ? cx : (axis == 1 ? cy : cz);
    std::sort(perm.begin() + l, perm.begin() + r + 1, [&key](int a, int b) { return key[a] < key[b]; });
  }

  int build(int l, int r, int n) {
    if (l > r) return 0;
    const float INFf = (float)114514.0;  // #define INF 114514.0 (BVH.h:8)
    nodes.push_back(Node());
    int id = (int)nodes.size() - 1;
    nodes[id].left = nodes[id].right = nodes[id].n = nodes[id].index = 0;
    nodes[id].AA = glsl::splat((float)1145141919);
    nodes[id].BB = glsl::splat((float)-1145141919);
    for (int i = l; i <= r; ++i) {
      int t = perm[i];
      nodes[id].AA.x = gmin(nodes[id].AA.x, tmin[0][t]);
      nodes[id].AA.y = gmin(nodes[id].AA.y, tmin[1][t]);
      nodes[id].AA.z = gmin(nodes[id].AA.z, tmin[2][t]);
      nodes[id].BB.x = gmax(nodes[id].BB.x, tmax[0][t]);
      nodes[id].BB.y = gmax(nodes[id].BB.y, tmax[1][t]);
      nodes[id].BB.z = gmax(nodes[id].BB.z, tmax[2][t]);
    }
    if ((r - l + 1) <= n) {
      nodes[id].n = r - l + 1;
      nodes[id].index = l;
      return id;
    }
    float Cost = INFf;
    int Axis = 0;
    int Split = (l + r) / 2;
    int len = r - l + 1;
    std::vector<float> lmax[3], lmin[3], rmax[3], rmin[3];
    for (int a = 0; a < 3; ++a) {
      lmax[a].resize(len); lmin[a].resize(len);
      rmax[a].resize(len); rmin[a].resize(len);
    }
    for (int axis = 0; axis < 3; ++axis) {
      sort_axis(l, r, axis);
      for (int i = l; i <= r; ++i) {
        int t = perm[i];
        int bias = (i == l) ? 0 : 1;
        for (int a = 0; a < 3; ++a) {
          // bias == 0 reads the freshly initialised +-INF entry (BVH.h:88-101)
          lmax[a][i - l] = gmax(bias ? lmax[a][i - l - 1] : -INFf, tmax[a][t]);
          lmin[a][i - l] = gmin(bias ? lmin[a][i - l - 1] : INFf, tmin[a][t]);
        }
      }
      for (int i = r; i >= l; --i) {
        int t = perm[i];
        int bias = (i == r) ? 0 : 1;
        for (int a = 0; a < 3; ++a) {
          rmax[a][i - l] = gmax(bias ? rmax[a][i - l + 1] : -INFf, tmax[a][t]);
          rmin[a][i - l] = gmin(bias ? rmin[a][i - l + 1] : INFf, tmin[a][t]);
        }
      }
      float cost = INFf;
      int split = l;
      for (int i = l; i <= r - 1; ++i) {
        float lenx = lmax[0][i - l] - lmin[0][i - l];
        float leny = lmax[1][i - l] - lmin[1][i - l];
        float lenz = lmax[2][i - l] - lmin[2][i - l];
        float leftS = (float)(2.0 * (double)(((lenx * leny) + (lenx * lenz)) + (leny * lenz)));
        float leftCost = leftS * (float)(i - l + 1);
        lenx = rmax[0][i + 1 - l] - rmin[0][i + 1 - l];
        leny = rmax[1][i + 1 - l] - rmin[1][i + 1 - l];
        lenz = rmax[2][i + 1 - l] - rmin[2][i + 1 - l];
        float rightS = (float)(2.0 * (double)(((lenx * leny) + (lenx * lenz)) + (leny * lenz)));
        float rightCost = rightS * (float)(r - i);
        float totalCost = leftCost + rightCost;
        if (totalCost < cost) {
          cost = totalCost;
          split = i;
        }
      }
      if (cost < Cost) {
        Cost = cost;
        Axis = axis;
        Split = split;
      }
    }
    sort_axis(l, r, Axis);
    int left = build(l, Split, n);
    int right = build(Split + 1, r, n);
    nodes[id].left = left;
    nodes[id].right = right;
    return id;
  }
};

void node_stats(const std::vector<Node>& nodes, int id, int depth, int64_t* leaves, int64_t* maxdepth,
                int64_t* maxleaf) {
  const Node& nd = nodes[id];
  if (depth > *maxdepth) *maxdepth = depth;
  if (nd.n > 0) {
    (*leaves)++;
    if (nd.n > *maxleaf) *maxleaf = nd.n;
    return;
  }
  if (nd.left > 0) node_stats(nodes, nd.left, depth + 1, leaves, maxdepth, maxleaf);
  if (nd.right > 0) node_stats(nodes, nd.right, depth + 1, leaves, maxdepth, maxleaf);
}

// ---------------------------------------------------------- OBJ parsing ---
bool parse_obj(const char* path, std::vector<v3>& vertices, std::vector<int>& indices, std::vector<int>& tex_indices,
               std::vector<float>& texcoords, float* maxaxis_out) {
  std::ifstream fin(path);
  if (!fin.is_open()) return false;
  // obj_loader.h:21-26 (double literals narrowed to float)
  float maxx = (float)-11451419.19, maxy = (float)-11451419.19, maxz = (float)-11451419.19;
  float minx = (float)11451419.19, miny = (float)11451419.19, minz = (float)11451419.19;
  std::string line;
  while (std::getline(fin, line)) {
    std::istringstream sin(line);
    std::string type;
    float x = 0, y = 0, z = 0, uvx = 0, uvy = 0;
    int v0 = 0, v1 = 0, v2 = 0, vn0 = 0, vn1 = 0, vn2 = 0, vt0 = 0, vt1 = 0, vt2 = 0;
    char slash;
    int slashCnt = 0;
    for (char c : line)
      if (c == '/') slashCnt++;
    sin >> type;
    if (type == "v") {
      sin >> x >> y >> z;
      vertices.push_back(glsl::mk(x, y, z));
      // the reference's bug: y/z bounds use maxx/minx (obj_loader.h:51-52)
      maxx = gmax(maxx, x); maxy = gmax(maxx, y); maxz = gmax(maxx, z);
      minx = gmin(minx, x); miny = gmin(minx, y); minz = gmin(minx, z);
    }
    if (type == "vt") {
      sin >> uvx >> uvy;
      texcoords.push_back(uvx);
      texcoords.push_back(uvy);
    }
    if (type == "f") {
      if (slashCnt == 6) {
        sin >> v0 >> slash >> vt0 >> slash >> vn0;
        sin >> v1 >> slash >> vt1 >> slash >> vn1;
        sin >> v2 >> slash >> vt2 >> slash >> vn2;
      } else if (slashCnt == 3) {
        sin >> v0 >> slash >> vt0;
        sin >> v1 >> slash >> vt1;
        sin >> v2 >> slash >> vt2;
      } else {
        sin >> v0 >> v1 >> v2;
      }
      indices.push_back(v0 - 1);
      indices.push_back(v1 - 1);
      indices.push_back(v2 - 1);
      tex_indices.push_back(vt0 - 1);
      tex_indices.push_back(vt1 - 1);
      tex_indices.push_back(vt2 - 1);
    }
  }
  float lenx = maxx - minx, leny = maxy - miny, lenz = maxz - minz;
  *maxaxis_out = gmax(lenx, gmax(leny, lenz));
  return true;
}

}  // namespace

// ============================================================== C ABI ===
extern "C" {

const char* pts_last_error(void) { return g_err.c_str(); }

pts_scene* pts_scene_create(void) { return new pts_scene(); }
void pts_scene_destroy(pts_scene* s) { delete s; }

int pts_scene_add_obj(pts_scene* s, const char* path, const float* material18, const float* trans16,
                      int smooth_normal, int obj_index) {
  if (!s || !path || !material18 || !trans16) return fail("pts_scene_add_obj: null argument");
  std::vector<v3> vertices;
  std::vector<int> indices, tex_indices;
  std::vector<float> texcoords;
  float maxaxis = 1.0f;
  if (!parse_obj(path, vertices, indices, tex_indices, texcoords, &maxaxis))
    return fail(std::string("cannot open ") + path);
  for (int i : indices)
    if (i < 0 || (size_t)i >= vertices.size()) return fail("obj face index out of range");
  for (auto& v : vertices) {  // obj_loader.h:87-91
    v.x /= maxaxis;
    v.y /= maxaxis;
    v.z /= maxaxis;
  }
  for (auto& v : vertices) v = xform_point(trans16, v);  // obj_loader.h:94-98
  emit_triangles(s, vertices, indices, tex_indices, texcoords, material18, smooth_normal != 0, obj_index);
  return 0;
}

int pts_scene_add_mesh(pts_scene* s, const float* positions, const float* uvs, int n_verts, const int* indices,
                       int n_tris, const float* material18, const float* trans16, int smooth_normal,
                       int obj_index) {
  if (!s || !positions || !indices || !material18 || !trans16 || n_verts <= 0 || n_tris < 0)
    return fail("pts_scene_add_mesh: bad argument");
  std::vector<v3> vertices(n_verts);
  std::vector<float> texcoords;
  for (int i = 0; i < n_verts; ++i)
    vertices[i] = xform_point(trans16, glsl::mk(positions[3 * i], positions[3 * i + 1], positions[3 * i + 2]));
  if (uvs) texcoords.assign(uvs, uvs + 2 * (size_t)n_verts);
  std::vector<int> idx(indices, indices + 3 * (size_t)n_tris);
  for (int i : idx)
    if (i < 0 || i >= n_verts) return fail("mesh index out of range");
  std::vector<int> tidx = uvs ? idx : std::vector<int>(idx.size(), -1);
  emit_triangles(s, vertices, idx, tidx, texcoords, material18, smooth_normal != 0, obj_index);
  return 0;
}

int pts_scene_add_raw(pts_scene* s, const float* v, int n_tris, const float* material18, int obj_index) {
  if (!s || !v || !material18 || n_tris < 0) return fail("pts_scene_add_raw: bad argument");
  size_t off = s->tris.size();
  s->tris.resize(off + n_tris);
  for (int i = 0; i < n_tris; ++i) {
    const float* q = v + (size_t)i * 18;
    Tri& t = s->tris[off + i];
    t.p1 = glsl::mk(q[0], q[1], q[2]); t.n1 = glsl::mk(q[3], q[4], q[5]);
    t.p2 = glsl::mk(q[6], q[7], q[8]); t.n2 = glsl::mk(q[9], q[10], q[11]);
    t.p3 = glsl::mk(q[12], q[13], q[14]); t.n3 = glsl::mk(q[15], q[16], q[17]);
    t.uv1[0] = t.uv1[1] = t.uv2[0] = t.uv2[1] = t.uv3[0] = t.uv3[1] = 0.0f;
    memcpy(t.mat, material18, sizeof(t.mat));
    t.objID = obj_index < 0 ? i : obj_index;
    s->raster.insert(s->raster.end(), q, q + 18);
  }
  s->built = false;
  return 0;
}

int pts_scene_build_bvh(pts_scene* s, int leaf_n) {
  if (!s || leaf_n < 1) return fail("pts_scene_build_bvh: bad argument");
  if (s->tris.empty()) return fail("pts_scene_build_bvh: empty scene");
  s->nodes.clear();
  // main.cpp:88-94: dummy node 0 so the root is node 1
  Node dummy;
  dummy.left = 255; dummy.right = 128; dummy.n = 30; dummy.index = 0;
  dummy.AA = glsl::mk(1, 1, 0);
  dummy.BB = glsl::mk(0, 1, 0);
  s->nodes.push_back(dummy);
  Builder b(s->tris, s->nodes);
  b.build(0, (int)s->tris.size() - 1, leaf_n);
  std::vector<Tri> sorted(s->tris.size());
  for (size_t i = 0; i < sorted.size(); ++i) sorted[i] = s->tris[b.perm[i]];
  s->tris.swap(sorted);
  s->built = true;
  return 0;
}

int pts_scene_counts(const pts_scene* s, int64_t* out) {
  if (!s || !out) return fail("pts_scene_counts: null argument");
  int64_t leaves = 0, maxdepth = 0, maxleaf = 0;
  if (s->built && s->nodes.size() > 1) node_stats(s->nodes, 1, 0, &leaves, &maxdepth, &maxleaf);
  out[0] = (int64_t)s->tris.size();
  out[1] = (int64_t)s->nodes.size();
  out[2] = leaves;
  out[3] = maxdepth;
  out[4] = maxleaf;
  out[5] = (int64_t)s->raster.size();
  return 0;
}

int pts_scene_root_aabb(const pts_scene* s, float* out6) {
  if (!s || !out6 || !s->built || s->nodes.size() < 2) return fail("pts_scene_root_aabb: BVH not built");
  const Node& r = s->nodes[1];
  out6[0] = r.AA.x; out6[1] = r.AA.y; out6[2] = r.AA.z;
  out6[3] = r.BB.x; out6[4] = r.BB.y; out6[5] = r.BB.z;
  return 0;
}

int pts_scene_encode(const pts_scene* s, float* tri_out, float* node_out, float* raster_out) {
  if (!s) return fail("pts_scene_encode: null scene");
  if ((tri_out || node_out) && !s->built) return fail("pts_scene_encode: BVH not built");
  if (tri_out) {  // main.cpp:101-124
    for (size_t i = 0; i < s->tris.size(); ++i) {
      const Tri& t = s->tris[i];
      const float* m = t.mat;
      float* o = tri_out + i * PTS_TRI_ENCODED_FLOATS;
      const v3* p[6] = {&t.p1, &t.p2, &t.p3, &t.n1, &t.n2, &t.n3};
      for (int k = 0; k < 6; ++k) { o[3 * k] = p[k]->x; o[3 * k + 1] = p[k]->y; o[3 * k + 2] = p[k]->z; }
      o[18] = m[0]; o[19] = m[1]; o[20] = m[2];               // emissive
      o[21] = m[3]; o[22] = m[4]; o[23] = m[5];               // baseColor
      o[24] = m[6]; o[25] = m[7]; o[26] = m[8];               // subsurface, metallic, specular
      o[27] = m[9]; o[28] = m[10]; o[29] = m[11];             // specularTint, roughness, anisotropic
      o[30] = m[12]; o[31] = m[13]; o[32] = m[14];            // sheen, sheenTint, clearcoat
      o[33] = m[15]; o[34] = m[16]; o[35] = m[17];            // clearcoatGloss, IOR, transmission
      o[36] = t.uv1[0]; o[37] = t.uv1[1]; o[38] = t.uv2[0];  // uvPacked1
      o[39] = t.uv2[1]; o[40] = t.uv3[0]; o[41] = t.uv3[1];  // uvPacked2
      o[42] = (float)t.objID; o[43] = 0.0f; o[44] = 0.0f;     // objIndex
    }
  }
  if (node_out) {  // main.cpp:127-133
    for (size_t i = 0; i < s->nodes.size(); ++i) {
      const Node& n = s->nodes[i];
      float* o = node_out + i * PTS_NODE_ENCODED_FLOATS;
      o[0] = (float)n.left; o[1] = (float)n.right; o[2] = 0.0f;
      o[3] = (float)n.n; o[4] = (float)n.index; o[5] = 0.0f;
      o[6] = n.AA.x; o[7] = n.AA.y; o[8] = n.AA.z;
      o[9] = n.BB.x; o[10] = n.BB.y; o[11] = n.BB.z;
    }
  }
  if (raster_out) memcpy(raster_out, s->raster.data(), s->raster.size() * sizeof(float));
  return 0;
}

void pts_transform_matrix(const float* rot3, const float* tr3, const float* sc3, float* out16) {
  // glm::scale / translate / rotate on the identity (obj_loader.h:166-182)
  float I[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
  auto matmul = [](const float* a, const float* b, float* o) {  // o = a*b column-major, glm order
    for (int c = 0; c < 4; ++c)
      for (int r = 0; r < 4; ++r) {
        float m0 = a[0 * 4 + r] * b[c * 4 + 0];
        float m1 = a[1 * 4 + r] * b[c * 4 + 1];
        float m2 = a[2 * 4 + r] * b[c * 4 + 2];
        float m3 = a[3 * 4 + r] * b[c * 4 + 3];
        o[c * 4 + r] = (m0 + m1) + (m2 + m3);
      }
  };
  float S[16], T[16];
  memcpy(S, I, sizeof(I));
  S[0] = sc3[0]; S[5] = sc3[1]; S[10] = sc3[2];
  memcpy(T, I, sizeof(I));
  T[12] = tr3[0]; T[13] = tr3[1]; T[14] = tr3[2];
  float R[16];
  memcpy(R, I, sizeof(I));
  const float axes[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
  for (int k = 0; k < 3; ++k) {
    float a = rot3[k] * (float)0.01745329251994329576923690768489;  // glm::radians
    float c = std::cos(a), s = std::sin(a);
    const float* ax = axes[k];
    float temp[3] = {(1 - c) * ax[0], (1 - c) * ax[1], (1 - c) * ax[2]};
    float Rt[16] = {c + temp[0] * ax[0], temp[0] * ax[1] + s * ax[2], temp[0] * ax[2] - s * ax[1], 0,
                    temp[1] * ax[0] - s * ax[2], c + temp[1] * ax[1], temp[1] * ax[2] + s * ax[0], 0,
                    temp[2] * ax[0] + s * ax[1], temp[2] * ax[1] - s * ax[0], c + temp[2] * ax[2], 0,
                    0, 0, 0, 1};
    float o[16];
    matmul(R, Rt, o);
    memcpy(R, o, sizeof(o));
  }
  float TR[16];
  matmul(T, R, TR);
  matmul(TR, S, out16);
}

int pts_hdr_cache(const float* HDR, int width, int height, float* cache) {
  if (!HDR || !cache || width <= 0 || height <= 0) return fail("pts_hdr_cache: bad argument");
  const size_t W = width, H = height;
  float lumSum = 0.0f;
  std::vector<float> pdf(W * H);  // pdf[i][j] at i*W+j (hdr_compute.h:7-21)
  for (size_t i = 0; i < H; ++i)
    for (size_t j = 0; j < W; ++j) {
      float R = HDR[3 * (i * W + j)], G = HDR[3 * (i * W + j) + 1], B = HDR[3 * (i * W + j) + 2];
      float lum = (float)((0.2 * (double)R + 0.7 * (double)G) + 0.1 * (double)B);
      pdf[i * W + j] = lum;
      lumSum += lum;
    }
  for (size_t k = 0; k < W * H; ++k) pdf[k] /= lumSum;
  std::vector<float> pdf_x_margin(W, 0.0f);
  for (size_t j = 0; j < W; ++j)
    for (size_t i = 0; i < H; ++i) pdf_x_margin[j] += pdf[i * W + j];
  std::vector<float> cdf_x_margin = pdf_x_margin;
  for (size_t i = 1; i < W; ++i) cdf_x_margin[i] += cdf_x_margin[i - 1];
  // conditional cdf, stored column-major: cdf_y[j][i] at j*H+i (hdr_compute.h:40-59)
  std::vector<float> cdf_y(W * H);
  for (size_t j = 0; j < W; ++j) {
    for (size_t i = 0; i < H; ++i) cdf_y[j * H + i] = pdf[i * W + j] / pdf_x_margin[j];
    for (size_t i = 1; i < H; ++i) cdf_y[j * H + i] += cdf_y[j * H + i - 1];
  }
  for (size_t j = 0; j < W; ++j) {
    for (size_t i = 0; i < H; ++i) {
      float xi_1 = float(i) / (float)height;
      float xi_2 = float(j) / (float)width;
      size_t x = std::lower_bound(cdf_x_margin.begin(), cdf_x_margin.end(), xi_1) - cdf_x_margin.begin();
      if (x >= W) x = W - 1;  // the reference would index past the end here (UB); clamp
      const float* col = &cdf_y[x * H];
      size_t y = std::lower_bound(col, col + H, xi_2) - col;
      if (y >= H) y = H - 1;
      cache[3 * (i * W + j)] = float(x) / (float)width;
      cache[3 * (i * W + j) + 1] = float(y) / (float)height;
      cache[3 * (i * W + j) + 2] = pdf[i * W + j];
    }
  }
  return 0;
}

// ------------------------------------------------ synthetic stand-ins ----
namespace {
struct MeshOut {
  std::vector<float> pos;
  std::vector<int> idx;
  int vert(float x, float y, float z) {
    pos.push_back(x); pos.push_back(y); pos.push_back(z);
    return (int)(pos.size() / 3) - 1;
  }
  void tri(int a, int b, int c) { idx.push_back(a); idx.push_back(b); idx.push_back(c); }
  void quad(int a, int b, int c, int d) { tri(a, b, c); tri(a, c, d); }
};
int mesh_result(const MeshOut& m, int* nv, int* nt, float* positions, int* indices) {
  if (nv) *nv = (int)(m.pos.size() / 3);
  if (nt) *nt = (int)(m.idx.size() / 3);
  if (positions) memcpy(positions, m.pos.data(), m.pos.size() * sizeof(float));
  if (indices) memcpy(indices, m.idx.data(), m.idx.size() * sizeof(int));
  return 0;
}
struct Lcg {
  uint32_t s;
  float next() {  // deterministic [0,1)
    s = s * 1664525u + 1013904223u;
    return (float)(s >> 8) * (1.0f / 16777216.0f);
  }
};
// Surface of revolution: profile (r_k, y_k), k = 0..np-1, `seg` segments, outward winding.
// A zero radius is a pole: one vertex and a triangle fan (no zero-area faces).
void lathe(MeshOut& m, const float* r, const float* y, int np, int seg) {
  std::vector<int> start(np);
  for (int k = 0; k < np; ++k) {
    start[k] = (int)(m.pos.size() / 3);
    if (r[k] == 0.0f) {
      m.vert(0.0f, y[k], 0.0f);
      continue;
    }
    for (int s = 0; s < seg; ++s) {
      float a = 2.0f * glsl::kPI * (float)s / (float)seg;
      m.vert(r[k] * glsl::g_cos(a), y[k], r[k] * glsl::g_sin(a));
    }
  }
  for (int k = 0; k + 1 < np; ++k) {
    bool pa = r[k] == 0.0f, pb = r[k + 1] == 0.0f;
    if (pa && pb) continue;
    for (int s = 0; s < seg; ++s) {
      int s1 = (s + 1) % seg;
      if (pa) m.tri(start[k], start[k + 1] + s, start[k + 1] + s1);
      else if (pb) m.tri(start[k] + s, start[k + 1], start[k] + s1);
      else m.quad(start[k] + s, start[k + 1] + s, start[k + 1] + s1, start[k] + s1);
    }
  }
}
// Tube along a polyline (centres c, radius rad), `seg` segments around.
void tube(MeshOut& m, const std::vector<v3>& c, float rad, int seg) {
  int base = (int)(m.pos.size() / 3);
  int n = (int)c.size();
  for (int k = 0; k < n; ++k) {
    v3 t = glsl::normalize(glsl::sub(c[k < n - 1 ? k + 1 : k], c[k > 0 ? k - 1 : k]));
    v3 helper = glsl::f_abs(t.y) < 0.9f ? glsl::mk(0, 1, 0) : glsl::mk(1, 0, 0);
    v3 u = glsl::normalize(glsl::cross(t, helper));
    v3 w = glsl::cross(t, u);
    for (int s = 0; s < seg; ++s) {
      float a = 2.0f * glsl::kPI * (float)s / (float)seg;
      v3 p = glsl::add(c[k], glsl::add(glsl::muls(u, rad * glsl::g_cos(a)), glsl::muls(w, rad * glsl::g_sin(a))));
      m.vert(p.x, p.y, p.z);
    }
  }
  for (int k = 0; k + 1 < n; ++k)
    for (int s = 0; s < seg; ++s) {
      int s1 = (s + 1) % seg;
      m.quad(base + k * seg + s, base + k * seg + s1, base + (k + 1) * seg + s1, base + (k + 1) * seg + s);
    }
}
}  // namespace

int pts_gen_plant(uint32_t seed, int leaves, int* nv, int* nt, float* positions, int* indices) {
  if (leaves < 0) return fail("pts_gen_plant: leaves < 0");
  MeshOut m;
  Lcg rng{seed * 2654435761u + 12345u};
  // pot: tapered cylinder with rim and soil disk (y in [0, 0.35])
  const float pr[] = {0.0f, 0.16f, 0.22f, 0.24f, 0.22f, 0.0f};
  const float py[] = {0.0f, 0.0f, 0.33f, 0.35f, 0.31f, 0.31f};
  lathe(m, pr, py, 6, 48);
  // stems + leaves
  for (int i = 0; i < leaves; ++i) {
    float ang = 2.0f * glsl::kPI * rng.next();
    float h = 0.45f + 0.55f * rng.next();
    float lean = 0.15f + 0.35f * rng.next();
    v3 root = glsl::mk(0.04f * glsl::g_cos(ang), 0.31f, 0.04f * glsl::g_sin(ang));
    v3 dir = glsl::normalize(glsl::mk(lean * glsl::g_cos(ang), 1.0f, lean * glsl::g_sin(ang)));
    std::vector<v3> stem;
    for (int k = 0; k < 5; ++k) {
      float t = (float)k / 4.0f;
      v3 p = glsl::add(root, glsl::muls(dir, h * t));
      p.y -= 0.12f * t * t * lean;  // droop
      stem.push_back(p);
    }
    tube(m, stem, 0.006f, 6);
    // leaf: curved blade from the stem tip, nu x nv grid
    v3 tip = stem.back();
    v3 fwd = glsl::normalize(glsl::mk(glsl::g_cos(ang), 0.25f - 0.5f * rng.next(), glsl::g_sin(ang)));
    v3 side = glsl::normalize(glsl::cross(fwd, glsl::mk(0, 1, 0)));
    float L = 0.18f + 0.14f * rng.next(), Wd = 0.05f + 0.04f * rng.next();
    const int nu = 8, nvv = 4;
    int base = (int)(m.pos.size() / 3);
    for (int a = 0; a <= nu; ++a) {
      float u = (float)a / nu;
      float half = Wd * (0.15f + 0.85f * glsl::g_sin(glsl::kPI * u));  // never zero width: no degenerate faces
      for (int b = 0; b <= nvv; ++b) {
        float v = (float)b / nvv * 2.0f - 1.0f;
        v3 p = glsl::add(tip, glsl::muls(fwd, L * u));
        p = glsl::add(p, glsl::muls(side, half * v));
        p.y += -0.10f * u * u + 0.015f * (1.0f - v * v);
        m.vert(p.x, p.y, p.z);
      }
    }
    for (int a = 0; a < nu; ++a)
      for (int b = 0; b < nvv; ++b) {
        int i0 = base + a * (nvv + 1) + b;
        m.quad(i0, i0 + 1, i0 + nvv + 2, i0 + nvv + 1);
      }
  }
  return mesh_result(m, nv, nt, positions, indices);
}

int pts_gen_teapot(int segments, int* nv, int* nt, float* positions, int* indices) {
  if (segments < 8) return fail("pts_gen_teapot: segments < 8");
  MeshOut m;
  // body + lid profile (radius, height)
  const float r[] = {0.0f, 0.30f, 0.42f, 0.48f, 0.47f, 0.40f, 0.30f, 0.32f, 0.20f, 0.05f, 0.06f, 0.0f};
  const float y[] = {0.0f, 0.0f, 0.06f, 0.22f, 0.38f, 0.52f, 0.58f, 0.60f, 0.66f, 0.70f, 0.76f, 0.78f};
  lathe(m, r, y, 12, segments);
  std::vector<v3> spout, handle;
  for (int k = 0; k <= 10; ++k) {
    float t = (float)k / 10.0f;
    spout.push_back(glsl::mk(0.42f + 0.30f * t, 0.20f + 0.38f * t * t, 0.0f));
  }
  for (int k = 0; k <= 16; ++k) {
    float a = -0.5f * glsl::kPI + glsl::kPI * (float)k / 16.0f;
    handle.push_back(glsl::mk(-0.46f - 0.16f * glsl::g_cos(a), 0.38f + 0.16f * glsl::g_sin(a), 0.0f));
  }
  tube(m, spout, 0.05f, segments / 2);
  tube(m, handle, 0.03f, segments / 2);
  return mesh_result(m, nv, nt, positions, indices);
}

int pts_gen_cornell(int* nv, int* nt, float* positions, int* indices) {
  MeshOut m;
  auto quad = [&m](v3 a, v3 b, v3 c, v3 d) {
    int i0 = m.vert(a.x, a.y, a.z), i1 = m.vert(b.x, b.y, b.z), i2 = m.vert(c.x, c.y, c.z),
        i3 = m.vert(d.x, d.y, d.z);
    m.quad(i0, i1, i2, i3);
  };
  using glsl::mk;
  quad(mk(-1, -1, -1), mk(-1, -1, 1), mk(1, -1, 1), mk(1, -1, -1));  // floor (faces +y)
  quad(mk(-1, 1, -1), mk(1, 1, -1), mk(1, 1, 1), mk(-1, 1, 1));      // ceiling (faces -y)
  quad(mk(-1, -1, -1), mk(1, -1, -1), mk(1, 1, -1), mk(-1, 1, -1));  // back (faces +z)
  quad(mk(-1, -1, -1), mk(-1, 1, -1), mk(-1, 1, 1), mk(-1, -1, 1));  // left (faces +x)
  quad(mk(1, -1, -1), mk(1, -1, 1), mk(1, 1, 1), mk(1, 1, -1));      // right (faces -x)
  return mesh_result(m, nv, nt, positions, indices);
}

// ------------------------------------------------------------- RGBE ---
namespace {
typedef unsigned char Rgbe[4];
// decrunch / oldDecrunch (hdrloader.cpp:118-191) over a byte cursor; false = truncated or malformed
struct Bytes {
  const std::vector<unsigned char>& b;
  size_t i;
  int get() { return i < b.size() ? b[i++] : -1; }
};
bool old_decrunch(Rgbe* scan, int len, Bytes& f, Rgbe* first) {
  int rshift = 0;
  while (len > 0) {
    int c[4];
    for (int k = 0; k < 4; ++k) c[k] = f.get();
    if (c[3] < 0) return false;  // feof
    for (int k = 0; k < 4; ++k) scan[0][k] = (unsigned char)c[k];
    if (scan[0][0] == 1 && scan[0][1] == 1 && scan[0][2] == 1) {  // repeat the previous pixel
      if (scan == first) return false;                            // nothing before it
      for (int i = scan[0][3] << rshift; i > 0; --i) {
        if (len <= 0) return false;
        memcpy(&scan[0][0], &scan[-1][0], 4);
        ++scan;
        --len;
      }
      rshift += 8;
    } else {
      ++scan;
      --len;
      rshift = 0;
    }
  }
  return true;
}
bool decrunch(Rgbe* scan, int len, Bytes& f) {
  if (len < 8 || len > 0x7fff) return old_decrunch(scan, len, f, scan);
  size_t mark = f.i;
  int i = f.get();
  if (i != 2) {
    f.i = mark;  // fseek(file, -1, SEEK_CUR)
    return old_decrunch(scan, len, f, scan);
  }
  int g = f.get(), b = f.get();
  i = f.get();
  if (i < 0) return false;
  scan[0][1] = (unsigned char)g;
  scan[0][2] = (unsigned char)b;
  if (scan[0][1] != 2 || (scan[0][2] & 128)) {
    scan[0][0] = 2;
    scan[0][3] = (unsigned char)i;
    return old_decrunch(scan + 1, len - 1, f, scan);
  }
  for (int c = 0; c < 4; ++c) {
    for (int j = 0; j < len;) {
      int code = f.get();
      if (code < 0) return false;
      if (code > 128) {  // run
        code &= 127;
        int val = f.get();
        if (val < 0 || j + code > len) return false;
        while (code--) scan[j++][c] = (unsigned char)val;
      } else {           // literal
        if (j + code > len) return false;
        while (code--) {
          int v = f.get();
          if (v < 0) return false;
          scan[j++][c] = (unsigned char)v;
        }
      }
    }
  }
  return true;
}
float rgbe_component(int expo, int val) {  // convertComponent (hdrloader.cpp:101-106)
  float v = val / 256.0f;
  float d = (float)pow(2.0, (double)expo);
  return v * d;
}
}  // namespace

int pts_load_hdr(const char* path, int* width, int* height, float* rgb_out) {
  if (!path || !width || !height) return fail("pts_load_hdr: bad argument");
  FILE* fp = fopen(path, "rb");
  if (!fp) return fail(std::string("pts_load_hdr: cannot open ") + path);
  std::vector<unsigned char> buf;
  unsigned char chunk[65536];
  size_t n;
  while ((n = fread(chunk, 1, sizeof(chunk), fp)) > 0) buf.insert(buf.end(), chunk, chunk + n);
  fclose(fp);
  if (buf.size() < 11 || memcmp(buf.data(), "#?RADIANCE", 10)) return fail("pts_load_hdr: not a Radiance file");
  Bytes f{buf, 11};  // magic + one skipped byte (fseek(file, 1, SEEK_CUR))
  int c = 0, oldc;
  for (;;) {  // header up to the empty line
    oldc = c;
    c = f.get();
    if (c < 0) return fail("pts_load_hdr: truncated header");
    if (c == 0xa && oldc == 0xa) break;
  }
  std::string reso;
  for (;;) {
    c = f.get();
    if (c < 0) return fail("pts_load_hdr: truncated resolution line");
    reso.push_back((char)c);
    if (c == 0xa) break;
  }
  long lh = 0, lw = 0;
  if (sscanf(reso.c_str(), "-Y %ld +X %ld", &lh, &lw) != 2 || lh <= 0 || lw <= 0 || lh > 65536 || lw > 65536)
    return fail("pts_load_hdr: unsupported resolution line");
  const int w = (int)lw, h = (int)lh;
  *width = w;
  *height = h;
  if (!rgb_out) return 0;
  std::vector<Rgbe> scan((size_t)w);
  float* cols = rgb_out;
  for (int y = h - 1; y >= 0; --y) {  // scanlines in file order; the reference ignores y for placement
    if (!decrunch(scan.data(), w, f)) return fail("pts_load_hdr: truncated or malformed scanline data");
    for (int x = 0; x < w; ++x) {
      const int expo = scan[x][3] - 128;
      cols[0] = rgbe_component(expo, scan[x][0]);
      cols[1] = rgbe_component(expo, scan[x][1]);
      cols[2] = rgbe_component(expo, scan[x][2]);
      cols += 3;
    }
  }
  return 0;
}

int pts_gen_env_map(int width, int height, float* out) {
  if (width <= 0 || height <= 0 || !out) return fail("pts_gen_env_map: bad argument");
  v3 sun = glsl::normalize(glsl::mk(0.4f, 0.6f, 0.3f));
  for (int i = 0; i < height; ++i) {
    // row i <-> v = (i+0.5)/H, elevation = pi*(0.5 - v) (toSphericalCoord, path_tracing.frag:804-810)
    float v = ((float)i + 0.5f) / (float)height;
    float el = glsl::kPI * (0.5f - v);
    float ce = glsl::g_cos(el), se = glsl::g_sin(el);
    for (int j = 0; j < width; ++j) {
      float u = ((float)j + 0.5f) / (float)width;
      float ph = 2.0f * glsl::kPI * (u - 0.5f);
      v3 d = glsl::mk(ce * glsl::g_cos(ph), se, ce * glsl::g_sin(ph));
      v3 c;
      if (d.y > 0.0f) {
        float t = glsl::f_sqrt(d.y);
        c = glsl::mixv(glsl::mk(1.25f, 1.15f, 1.05f), glsl::mk(0.35f, 0.55f, 1.25f), t);
      } else {
        float t = glsl::f_sqrt(-d.y);
        c = glsl::mixv(glsl::mk(0.45f, 0.40f, 0.35f), glsl::mk(0.18f, 0.15f, 0.12f), t);
      }
      // warm window strip (indoor "room" feel) + sun lobe
      float win = glsl::g_exp(-((ph - 1.2f) * (ph - 1.2f)) / 0.02f) * glsl::g_exp(-((el - 0.25f) * (el - 0.25f)) / 0.03f);
      float cs = glsl::dot(d, sun);
      float lobe = glsl::g_exp((cs - 1.0f) / 0.0015f);
      float* o = out + 3 * ((size_t)i * width + j);
      o[0] = c.x + 6.0f * win + 60.0f * lobe;
      o[1] = c.y + 5.0f * win + 55.0f * lobe;
      o[2] = c.z + 4.0f * win + 45.0f * lobe;
    }
  }
  return 0;
}

}  // extern "C"

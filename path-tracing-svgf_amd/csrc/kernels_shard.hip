// kernels_shard.hip — tile-shard transfers (multi-GPU; no GL counterpart).
//
// Under the tile shard (dist.TileShardRenderer) every rank's path tracer draws the 16 x 16 tiles t = k * stride +
// offset of every frame (PTParams::tile_stride / tile_offset, tiles numbered row-major from row tile_y0), and every
// band owner needs all ranks' pixels of its band's rows (widened by the ghost zone). These kernels move one rank's
// subset pixels of a row range between frame planes and a packed buffer, so that each (source, band) pair travels
// as ONE contiguous RCCL message:
//   packed block of a segment = for each plane j: for each row y in [y0, y1): the subset tiles' 16-pixel runs of
//   that row in x order.
// HBM-bound byte moves (16 B per pixel and plane each way, 256-B runs on the plane side, dense on the packed side);
// one launch covers every segment of a call.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "pt_device.h"

namespace ptk {

// Subset tiles in tile row ty: tiles tx in [0, ntx) with (ty * ntx + tx) % stride == offset.
__host__ __device__ __forceinline__ int shard_row_tiles(int ty, int ntx, int stride, int offset, int* tx0) {
  int r = (int)(((long long)offset - (long long)ty * ntx) % stride);
  if (r < 0) r += stride;
  *tx0 = r;
  return r < ntx ? (ntx - 1 - r) / stride + 1 : 0;
}

// Pixels of the subset in rows [y0, y) per plane (rows grouped by tile row).
__host__ __device__ __forceinline__ long long shard_row_offset(int y0, int y, int tile_y0, int ntx, int stride,
                                                               int offset) {
  long long n = 0;
  int row = y0;
  while (row < y) {
    const int ty = (row - tile_y0) / 16;
    const int end = min(y, tile_y0 + 16 * (ty + 1));
    int tx0;
    n += (long long)(end - row) * 16 * shard_row_tiles(ty, ntx, stride, offset, &tx0);
    row = end;
  }
  return n;
}

__global__ void __launch_bounds__(256) shard_copy_kernel(ShardCopy c) {
  const int s = blockIdx.y, j = blockIdx.z;
  const ShardSeg& sg = c.seg[s];
  const int y = sg.y0 + (int)blockIdx.x;
  if (y >= sg.y1) return;
  const int ntx = c.W / 16, ty = (y - c.tile_y0) / 16;
  int tx0;
  const int cnt = shard_row_tiles(ty, ntx, c.stride, sg.offset, &tx0);
  if (cnt == 0) return;
  const long long per_plane = shard_row_offset(sg.y0, sg.y1, c.tile_y0, ntx, c.stride, sg.offset);
  const long long row_off = shard_row_offset(sg.y0, y, c.tile_y0, ntx, c.stride, sg.offset);
  float4* packed = sg.packed + (size_t)(j * per_plane + row_off);
  float4* plane = c.plane[j] + (size_t)(y - c.row0[j]) * c.W;
  const int n = cnt * 16;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int x = 16 * (tx0 + (i >> 4) * c.stride) + (i & 15);
    if (c.unpack) plane[x] = packed[i];
    else packed[i] = plane[x];
  }
}

// Rows of the frame shard's planes as rgb (RgbRows): a thread moves 4 consecutive texels of one plane, 4 float4 on
// the plane side and 3 float4 (their 12 floats) on the packed side, so both sides move whole 16-B vectors (a texel
// count that is not a multiple of 4 ends in a scalar tail). Unpacking writes alpha 1.0.
__global__ void __launch_bounds__(256) rgb_rows_kernel(RgbRows c) {
  const int j = blockIdx.y;
  const long long n = (long long)(c.y1 - c.y0) * c.W;  // texels per plane
  const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;  // group of 4 texels
  if (4 * q >= n) return;
  float4* plane = c.plane[j] + (size_t)(c.y0 - c.row0[j]) * c.W;
  float* packed = c.packed + (size_t)j * n * 3;
  if (4 * q + 4 <= n && n % 4 == 0) {
    float4* pk = (float4*)packed + 3 * q;  // 16-B aligned: n a multiple of 4, and the buffer is
    if (c.unpack) {
      const float4 a = pk[0], b = pk[1], d = pk[2];
      plane[4 * q + 0] = make_float4(a.x, a.y, a.z, 1.0f);
      plane[4 * q + 1] = make_float4(a.w, b.x, b.y, 1.0f);
      plane[4 * q + 2] = make_float4(b.z, b.w, d.x, 1.0f);
      plane[4 * q + 3] = make_float4(d.y, d.z, d.w, 1.0f);
    } else {
      const float4 t0 = plane[4 * q + 0], t1 = plane[4 * q + 1], t2 = plane[4 * q + 2], t3 = plane[4 * q + 3];
      pk[0] = make_float4(t0.x, t0.y, t0.z, t1.x);
      pk[1] = make_float4(t1.y, t1.z, t2.x, t2.y);
      pk[2] = make_float4(t2.z, t3.x, t3.y, t3.z);
    }
    return;
  }
  for (long long i = 4 * q; i < n && i < 4 * q + 4; ++i) {
    if (c.unpack) plane[i] = make_float4(packed[3 * i], packed[3 * i + 1], packed[3 * i + 2], 1.0f);
    else {
      const float4 t = plane[i];
      packed[3 * i] = t.x;
      packed[3 * i + 1] = t.y;
      packed[3 * i + 2] = t.z;
    }
  }
}

int launch_rgb_rows(const RgbRows& c, hipStream_t s) {
  const long long n = (long long)(c.y1 - c.y0) * c.W;
  if (n <= 0 || c.nplanes <= 0) return 0;
  const long long groups = (n + 3) / 4;
  hipLaunchKernelGGL(rgb_rows_kernel, dim3((unsigned)((groups + 255) / 256), c.nplanes), dim3(256), 0, s, c);
  return (int)hipGetLastError();
}

long long shard_pixels(int W, int tile_y0, int stride, int offset, int y0, int y1) {
  return shard_row_offset(y0, y1, tile_y0, W / 16, stride, offset);
}

int launch_shard_copy(const ShardCopy& c, hipStream_t s) {
  int rows = 0;
  for (int i = 0; i < c.nseg; ++i) rows = max(rows, c.seg[i].y1 - c.seg[i].y0);
  if (rows <= 0 || c.nseg <= 0) return 0;
  hipLaunchKernelGGL(shard_copy_kernel, dim3(rows, c.nseg, c.nplanes), dim3(256), 0, s, c);
  return (int)hipGetLastError();
}

}  // namespace ptk

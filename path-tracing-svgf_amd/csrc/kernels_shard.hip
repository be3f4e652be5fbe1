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

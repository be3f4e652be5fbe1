// kernels_sched.hip — cost-ordered tile dispatch (TileSched, pt_device.h): turns the
// per-tile costs one traversal launch recorded into the tile order of the next one
// (descending cost, 4 buckets per octave; order inside a bucket is arbitrary), and
// clears the costs for that launch to record.
#include <hip/hip_runtime.h>

#include "pt_device.h"

namespace ptk {

constexpr int kSortBuckets = 64;

__device__ __forceinline__ int cost_bucket(uint32_t c) {
  // bucket 0 = most expensive
  if (c == 0) return kSortBuckets - 1;
  const int q = 1 + (int)(__log2f((float)c) * 4.0f);
  return kSortBuckets - 1 - (q < kSortBuckets - 1 ? q : kSortBuckets - 1);
}

__global__ void __launch_bounds__(1024) tile_sort_kernel(uint32_t* __restrict__ cost, int* __restrict__ perm, int n) {
  __shared__ int hist[kSortBuckets];
  if (threadIdx.x < kSortBuckets) hist[threadIdx.x] = 0;
  __syncthreads();
  for (int t = threadIdx.x; t < n; t += blockDim.x) atomicAdd(&hist[cost_bucket(cost[t])], 1);
  __syncthreads();
  if (threadIdx.x == 0) {
    int run = 0;
    for (int b = 0; b < kSortBuckets; ++b) {
      const int h = hist[b];
      hist[b] = run;
      run += h;
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < n; t += blockDim.x) {
    const int pos = atomicAdd(&hist[cost_bucket(cost[t])], 1);
    perm[pos] = t;
    cost[t] = 0;
  }
}

int launch_tile_sort(uint32_t* cost, int* perm, int ntiles, hipStream_t s) {
  if (ntiles <= 0) return 0;
  hipLaunchKernelGGL(tile_sort_kernel, dim3(1), dim3(1024), 0, s, cost, perm, ntiles);
  return (int)hipGetLastError();
}

}  // namespace ptk

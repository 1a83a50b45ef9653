// lzma_kernels.hip -- batch LZMA / LZMA2 decode kernels for gfx950.
//
// Grid mapping: one stream per lane, 64-lane workgroups (one wave each).
// `order` (optional) maps lane -> descriptor so the host planner can group
// streams of similar size and table width into the same wave (a wave runs
// until its slowest lane finishes).  The per-lane work is in lzma_lane.h.
#include <hip/hip_runtime.h>

#include "lzma_gpu_internal.h"

using namespace lzgpu;

__global__ void __launch_bounds__(64) lzgpu_decode_batch_kernel(
    const LzmaGpuStreamDesc* __restrict__ descs, const uint32_t* __restrict__ order, uint32_t n,
    const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint16_t* __restrict__ ws,
    LzmaGpuResult* __restrict__ results) {
  const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= n) return;
  const uint32_t id = order ? order[lane] : lane;
  const LzmaGpuStreamDesc d = descs[id];
  results[id] = lane_decode(d, src, dst, ws);
}

// One DecodeToDic call per lane on a device-resident decoder state.
__global__ void __launch_bounds__(64) lzgpu_session_kernel(LzgpuSession* __restrict__ sess,
                                                           uint32_t n) {
  const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= n) return;
  lane_session(sess[lane]);
}

extern "C" int lzgpu_launch_decode_batch(const LzmaGpuStreamDesc* d_descs, const uint32_t* d_order,
                                         uint32_t n, const uint8_t* d_src, uint8_t* d_dst,
                                         uint16_t* d_ws, LzmaGpuResult* d_results,
                                         hipStream_t stream) {
  if (n == 0) return 0;
  const uint32_t block = 64;
  const uint32_t grid = (n + block - 1) / block;
  hipLaunchKernelGGL(lzgpu_decode_batch_kernel, dim3(grid), dim3(block), 0, stream, d_descs,
                     d_order, n, d_src, d_dst, d_ws, d_results);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int lzgpu_launch_session(LzgpuSession* d_sess, uint32_t n, hipStream_t stream) {
  if (n == 0) return 0;
  const uint32_t block = 64;
  const uint32_t grid = (n + block - 1) / block;
  hipLaunchKernelGGL(lzgpu_session_kernel, dim3(grid), dim3(block), 0, stream, d_sess, n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// crc32_kernels.hip -- batch CRC-32 (7zCrc.c CrcCalc / CrcUpdate) for gfx950.
//
// Two launches per batch (formulation in crc32_device.h):
//   lzgpu_crc_chunk_kernel: one lane per kChunk-byte chunk slot, grid-stride;
//     raw CRC register of the chunk with slice-by-16 tables in LDS.  The loop
//     reads aligned 16-byte blocks, eight in flight per lane; partial blocks at
//     either end of a chunk are loaded whole (an aligned block holding a valid
//     byte never crosses a page) and consumed byte-wise from registers.
//   lzgpu_crc_fold_kernel: one lane per range; folds the chunk registers with
//     the table-driven multiply by x^(8 * kChunk).
// Ranges come from (offset, length) arrays or straight from a decode batch
// (descriptor dst_off + result dest_len), so the CRC of a decoded batch needs
// no host round trip.
#include <hip/hip_runtime.h>

#include "crc32_device.h"
#include "lzma_gpu_internal.h"

using namespace lzgpu;

__constant__ CrcTables kCrcTables = crc_make_tables();

namespace {

struct ArrayRanges {
  const uint64_t* off;
  const uint64_t* len;
  __device__ __forceinline__ uint64_t offset(uint32_t i) const { return off[i]; }
  __device__ __forceinline__ uint64_t length(uint32_t i) const { return len[i]; }
};

struct DecodeRanges {
  const LzmaGpuStreamDesc* descs;
  const LzmaGpuResult* res;
  __device__ __forceinline__ uint64_t offset(uint32_t i) const { return descs[i].dst_off; }
  __device__ __forceinline__ uint64_t length(uint32_t i) const { return res[i].dest_len; }
};

template <class Ranges>
__global__ void __launch_bounds__(256) lzgpu_crc_chunk_kernel(
    Ranges rg, const uint8_t* __restrict__ data, const uint32_t* __restrict__ chunk_base,
    const uint32_t* __restrict__ chunk_range, uint32_t n_chunks, uint32_t init,
    uint32_t* __restrict__ chunk_crc) {
  __shared__ uint32_t tab[16 * 256];
  const uint32_t* src = &kCrcTables.slice[0][0];
  for (uint32_t i = threadIdx.x; i < 16 * 256; i += blockDim.x) tab[i] = src[i];
  __syncthreads();
  const lds_u32t* t = (const lds_u32t*)tab;
  for (uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x; slot < n_chunks;
       slot += gridDim.x * blockDim.x) {
    const uint32_t r = chunk_range[slot];
    uint32_t c;
    if (crc_chunk(t, data + rg.offset(r), rg.length(r), slot - chunk_base[r], init, &c))
      chunk_crc[slot] = c;
  }
}

template <class Ranges>
__global__ void __launch_bounds__(256) lzgpu_crc_fold_kernel(
    Ranges rg, const uint32_t* __restrict__ chunk_base, const uint32_t* __restrict__ chunk_crc,
    uint32_t n, uint32_t init, uint32_t xorout, uint32_t* __restrict__ crc_out) {
  __shared__ uint32_t sh[4 * 256];
  const uint32_t* src = &kCrcTables.shift[0][0];
  for (uint32_t i = threadIdx.x; i < 4 * 256; i += blockDim.x) sh[i] = src[i];
  __syncthreads();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t r = crc_fold((const lds_u32t*)sh, chunk_crc + chunk_base[i], rg.length(i), init);
  crc_out[i] = r ^ xorout;
}

template <class Ranges>
int launch_crc(Ranges rg, const uint8_t* data, const uint32_t* chunk_base,
               const uint32_t* chunk_range, uint32_t n, uint32_t n_chunks, uint32_t init,
               uint32_t xorout, uint32_t* chunk_crc, uint32_t* crc, hipStream_t stream) {
  if (n == 0) return 0;
  if (n_chunks) {
    // grid-stride: up to 8 workgroups of 256 per CU on 256 CUs
    const uint32_t want = (n_chunks + 255) / 256;
    const uint32_t grid = want < 2048 ? want : 2048;
    hipLaunchKernelGGL(lzgpu_crc_chunk_kernel<Ranges>, dim3(grid), dim3(256), 0, stream, rg, data,
                       chunk_base, chunk_range, n_chunks, init, chunk_crc);
    if (hipGetLastError() != hipSuccess) return -1;
  }
  hipLaunchKernelGGL(lzgpu_crc_fold_kernel<Ranges>, dim3((n + 255) / 256), dim3(256), 0, stream,
                     rg, chunk_base, chunk_crc, n, init, xorout, crc);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace

extern "C" int lzgpu_launch_crc_arrays(const uint8_t* d_data, const uint64_t* d_off,
                                       const uint64_t* d_len, uint32_t n,
                                       const uint32_t* d_chunk_base,
                                       const uint32_t* d_chunk_range, uint32_t n_chunks,
                                       uint32_t init, uint32_t xorout, uint32_t* d_chunk_crc,
                                       uint32_t* d_crc, hipStream_t stream) {
  return launch_crc(ArrayRanges{d_off, d_len}, d_data, d_chunk_base, d_chunk_range, n, n_chunks,
                    init, xorout, d_chunk_crc, d_crc, stream);
}

extern "C" int lzgpu_launch_crc_decoded(const LzmaGpuStreamDesc* d_descs,
                                        const LzmaGpuResult* d_results, const uint8_t* d_dst,
                                        uint32_t n, const uint32_t* d_chunk_base,
                                        const uint32_t* d_chunk_range, uint32_t n_chunks,
                                        uint32_t* d_chunk_crc, uint32_t* d_crc,
                                        hipStream_t stream) {
  return launch_crc(DecodeRanges{d_descs, d_results}, d_dst, d_chunk_base, d_chunk_range, n,
                    n_chunks, 0xFFFFFFFFu, 0xFFFFFFFFu, d_chunk_crc, d_crc, stream);
}

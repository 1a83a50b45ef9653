// xz_kernels.hip -- the xz block-batch kernels for gfx950.
//
//   lzgpu_crc64_chunk_kernel / lzgpu_crc64_fold_kernel: CRC-64 (XzCrc64.c) of
//     byte ranges, the crc32_kernels.hip formulation with a 64-bit register
//     (crc64_device.h): one lane per 2 KiB chunk (slice-by-8 tables in LDS,
//     aligned 16-byte loads), then one lane per range folds the chunk
//     registers.
//   lzgpu_bcj_x86_kernel: x86 BCJ (Bra86.c) in place, one lane per range
//     (bcj_device.h); an xz block's filter state starts at 0 and runs over the
//     block's whole output.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "../../include/lzma_gpu.h"
#include "bcj2_device.h"
#include "bcj_device.h"
#include "bra_device.h"
#include "crc64_device.h"

using namespace lzgpu;

__constant__ Crc64Tables kCrc64Tables = crc64_make_tables();

__global__ void __launch_bounds__(256) lzgpu_crc64_chunk_kernel(
    const uint8_t* __restrict__ data, const uint64_t* __restrict__ off,
    const uint64_t* __restrict__ len, const uint32_t* __restrict__ chunk_base,
    const uint32_t* __restrict__ chunk_range, uint32_t n_chunks, uint64_t init,
    uint64_t* __restrict__ chunk_crc) {
  __shared__ uint64_t tab[8 * 256];
  const uint64_t* src = &kCrc64Tables.slice[0][0];
  for (uint32_t i = threadIdx.x; i < 8 * 256; i += blockDim.x) tab[i] = src[i];
  __syncthreads();
  const lds_u64t* t = (const lds_u64t*)tab;
  for (uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x; slot < n_chunks;
       slot += gridDim.x * blockDim.x) {
    const uint32_t r = chunk_range[slot];
    uint64_t c;
    if (crc64_chunk(t, data + off[r], len[r], slot - chunk_base[r], init, &c)) chunk_crc[slot] = c;
  }
}

__global__ void __launch_bounds__(256) lzgpu_crc64_fold_kernel(
    const uint64_t* __restrict__ len, const uint32_t* __restrict__ chunk_base,
    const uint64_t* __restrict__ chunk_crc, uint32_t n, uint64_t init, uint64_t xorout,
    uint64_t* __restrict__ crc_out) {
  __shared__ uint64_t sh[8 * 256];
  const uint64_t* src = &kCrc64Tables.shift[0][0];
  for (uint32_t i = threadIdx.x; i < 8 * 256; i += blockDim.x) sh[i] = src[i];
  __syncthreads();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  crc_out[i] = crc64_fold((const lds_u64t*)sh, chunk_crc + chunk_base[i], len[i], init) ^ xorout;
}

__global__ void __launch_bounds__(64) lzgpu_bcj_x86_kernel(
    uint8_t* __restrict__ data, const uint64_t* __restrict__ off, const uint64_t* __restrict__ len,
    const uint32_t* __restrict__ ip, uint32_t* __restrict__ state, uint64_t* __restrict__ done,
    uint32_t n, int encoding) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t s = state[i];
  done[i] = bcj_x86((bcj_byte*)(data + off[i]), len[i], ip[i], &s, encoding);
  state[i] = s;
}

extern "C" int lzgpu_launch_crc64_arrays(const uint8_t* d_data, const uint64_t* d_off,
                                         const uint64_t* d_len, uint32_t n,
                                         const uint32_t* d_chunk_base,
                                         const uint32_t* d_chunk_range, uint32_t n_chunks,
                                         uint64_t init, uint64_t xorout, uint64_t* d_chunk_crc,
                                         uint64_t* d_crc, hipStream_t stream) {
  if (n == 0) return 0;
  if (n_chunks) {
    const uint32_t want = (n_chunks + 255) / 256;
    const uint32_t grid = want < 2048 ? want : 2048;
    hipLaunchKernelGGL(lzgpu_crc64_chunk_kernel, dim3(grid), dim3(256), 0, stream, d_data, d_off,
                       d_len, d_chunk_base, d_chunk_range, n_chunks, init, d_chunk_crc);
    if (hipGetLastError() != hipSuccess) return -1;
  }
  hipLaunchKernelGGL(lzgpu_crc64_fold_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, d_len,
                     d_chunk_base, d_chunk_crc, n, init, xorout, d_crc);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// x86 BCJ, tiled (bcj_device.h, "tiled form"): one workgroup per range walks
// it in 4 KiB tiles.  Every lane takes 16 bytes of the tile into LDS (plus the
// four bytes behind the tile), finds its E8/E9 positions below size - 4, and
// an LDS scan of the per-lane counts places their (position, operand) records
// in tile order; lane 0 then runs the reference's decisions over the records
// and writes the converted operands.  For text (no E8/E9) a tile costs its
// loads and three barriers; branch-dense code is serial only per hit, not per
// byte.
constexpr uint32_t kBcjTile = 4096;

__global__ void __launch_bounds__(256) lzgpu_bcj_x86_tile_kernel(
    uint8_t* __restrict__ data, const uint64_t* __restrict__ off, const uint64_t* __restrict__ len,
    const uint32_t* __restrict__ ip, uint32_t* __restrict__ state, uint64_t* __restrict__ done,
    uint32_t n, int encoding) {
  __shared__ __attribute__((aligned(16))) uint8_t tile[kBcjTile + 16];
  __shared__ uint16_t rec_pos[kBcjTile];
  __shared__ uint32_t rec_op[kBcjTile];
  __shared__ uint32_t scan[256];
  typedef __attribute__((address_space(1))) uint8_t gb;
  typedef uint64_t u64a1 __attribute__((aligned(1)));
  typedef uint32_t u32a1 __attribute__((aligned(1)));
  const uint32_t t = threadIdx.x;
  for (uint32_t r = blockIdx.x; r < n; r += gridDim.x) {
    const uint64_t size = len[r];
    gb* p = (gb*)(data + off[r]);
    if (size < 5) {  // x86_Convert returns 0, state untouched
      if (t == 0) done[r] = 0;
      continue;
    }
    const uint64_t limit = size - 4;
    BcjRun run;  // lane 0's
    run.resume = 0;
    run.prev_pos = ~uint64_t(0);
    run.mask = state[r] & 7u;
    const uint32_t ip5 = ip[r] + 5;
    for (uint64_t tb = 0; tb < limit; tb += kBcjTile) {
      // the tile's bytes [tb, tb + 4096 + 4) that lie in the range
      const uint64_t a = tb + 16 * uint64_t(t);
      if (a + 16 <= size) {
        const uint64_t lo = *(const __attribute__((address_space(1))) u64a1*)(p + a);
        const uint64_t hi = *(const __attribute__((address_space(1))) u64a1*)(p + a + 8);
        *(uint64_t*)(tile + 16 * t) = lo;
        *(uint64_t*)(tile + 16 * t + 8) = hi;
      } else {
        for (uint32_t k = 0; k < 16; ++k) tile[16 * t + k] = a + k < size ? p[a + k] : 0;
      }
      if (t < 4) {
        const uint64_t q = tb + kBcjTile + t;
        tile[kBcjTile + t] = q < size ? p[q] : 0;
      }
      __syncthreads();
      // this lane's hits: E8 / E9 at positions below limit
      uint32_t hits = 0;  // bit k: byte 16 t + k is a hit
      for (uint32_t k = 0; k < 16; ++k)
        if ((tile[16 * t + k] & 0xFEu) == 0xE8u && a + k < limit) hits |= 1u << k;
      const uint32_t cnt = uint32_t(__builtin_popcount(hits));
      scan[t] = cnt;
      __syncthreads();
      for (uint32_t o = 1; o < 256; o <<= 1) {  // inclusive scan of the counts
        const uint32_t v = t >= o ? scan[t - o] : 0u;
        __syncthreads();
        scan[t] += v;
        __syncthreads();
      }
      uint32_t w = scan[t] - cnt;
      while (hits) {
        const uint32_t k = uint32_t(__builtin_ctz(hits));
        hits &= hits - 1;
        const uint32_t j = 16 * t + k;
        rec_pos[w] = uint16_t(j);
        rec_op[w] = uint32_t(tile[j + 1]) | (uint32_t(tile[j + 2]) << 8) |
                    (uint32_t(tile[j + 3]) << 16) | (uint32_t(tile[j + 4]) << 24);
        ++w;
      }
      const uint32_t total = scan[255];
      __syncthreads();
      if (t == 0) {
        for (uint32_t i = 0; i < total; ++i) {
          const uint64_t h = tb + rec_pos[i];
          if (h < run.resume) continue;
          uint32_t v;
          if (bcj_hit(run, h, rec_op[i], ip5, encoding, &v))
            *(__attribute__((address_space(1))) u32a1*)(p + h + 1) = v;
        }
      }
      __syncthreads();  // the conversions are visible to the next tile's loads
    }
    if (t == 0) {
      uint32_t st;
      done[r] = bcj_finish(run, limit, &st);
      state[r] = st;
    }
  }
}

extern "C" int lzgpu_launch_bcj_x86(uint8_t* d_data, const uint64_t* d_off, const uint64_t* d_len,
                                    const uint32_t* d_ip, uint32_t* d_state, uint64_t* d_done,
                                    uint32_t n, int encoding, hipStream_t stream) {
  if (n == 0) return 0;
  if (getenv("LZGPU_BCJ_SERIAL")) {  // the lane-serial statement (A/B)
    hipLaunchKernelGGL(lzgpu_bcj_x86_kernel, dim3((n + 63) / 64), dim3(64), 0, stream, d_data,
                       d_off, d_len, d_ip, d_state, d_done, n, encoding);
  } else {
    const uint32_t grid = n < 65536 ? n : 65536;
    hipLaunchKernelGGL(lzgpu_bcj_x86_tile_kernel, dim3(grid), dim3(256), 0, stream, d_data, d_off,
                       d_len, d_ip, d_state, d_done, n, encoding);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---- RISC branch converters and delta (bra_device.h; Bra.c, BraIA64.c, Delta.c)

// ARM / PPC / SPARC / IA64: one lane per aligned unit, blockIdx.y walks the ranges
__global__ void __launch_bounds__(256) lzgpu_bra_unit_kernel(
    uint8_t* __restrict__ data, const uint64_t* __restrict__ off, const uint64_t* __restrict__ len,
    const uint32_t* __restrict__ ip, uint64_t* __restrict__ done, uint32_t n, uint32_t kind,
    int encoding) {
  const uint32_t u = bra_unit(kind);
  for (uint32_t r = blockIdx.y; r < n; r += gridDim.y) {
    const uint64_t units = bra_done_units(kind, len[r]);
    bra_byte* base = (bra_byte*)(data + off[r]);
    // ARMT: the candidate test reads only bytes no conversion changes (bra_device.h)
    if (blockIdx.x == 0 && threadIdx.x == 0)
      done[r] = kind == kBraARMT ? bra_armt_done(base, units) : units * u;
    const uint32_t ip0 = ip[r];
    const uint64_t k0 = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint64_t step = uint64_t(gridDim.x) * blockDim.x;
    if (u == 4 && ((uintptr_t)base & 3) == 0) {  // word kinds, aligned range: dword access
      for (uint64_t k = k0; k < units; k += step)
        bra_word_aligned(kind, base + k * 4, ip0 + uint32_t(k * 4), encoding);
    } else {
      for (uint64_t k = k0; k < units; k += step)
        bra_unit_convert(kind, base + k * u, ip0 + uint32_t(k * u), encoding);
    }
  }
}

__global__ void __launch_bounds__(64) lzgpu_bra_armt_kernel(
    uint8_t* __restrict__ data, const uint64_t* __restrict__ off, const uint64_t* __restrict__ len,
    const uint32_t* __restrict__ ip, uint64_t* __restrict__ done, uint32_t n, int encoding) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  done[i] = bra_armt((bra_byte*)(data + off[i]), len[i], ip[i], encoding);
}

// one workgroup per range, lane r < delta runs residue r; state is 256 B per
// range (DELTA_STATE_SIZE), rewritten as the last `delta` bytes seen
__global__ void __launch_bounds__(256) lzgpu_delta_kernel(
    uint8_t* __restrict__ data, const uint64_t* __restrict__ off, const uint64_t* __restrict__ len,
    const uint32_t* __restrict__ delta, uint8_t* __restrict__ state, uint32_t n, int encoding) {
  __shared__ uint8_t st[256], sums[256], last[16];
  __shared__ V16 lanes[256];
  for (uint32_t r = blockIdx.x; r < n; r += gridDim.x) {
    const uint32_t d = delta[r];
    const uint64_t size = len[r];
    const uint32_t t = threadIdx.x;
    // a distance outside 1..256 (Delta.h: DELTA_STATE_SIZE) is not a delta
    // filter: the range is left as it is (uniform over the workgroup, before
    // any barrier -- d = 0 would otherwise never leave the prefix loop)
    if (d == 0 || d > 256) continue;
    if (t < d) st[t] = state[uint64_t(r) * 256 + t];
    __syncthreads();  // every state byte read before any is rewritten
    bra_byte* p = (bra_byte*)(data + off[r]);
    if (encoding) {  // Delta_Encode: one lane per residue
      if (t < d)
        state[uint64_t(r) * 256 + delta_state_slot(size, d, t)] =
            delta_residue(p, size, d, t, st[t], 1);
    } else if (d <= 16 && (d & (d - 1)) == 0) {  // Delta_Decode, d | 16: tile scan
      // head bytes up to a 16-byte aligned address: lane 0, serially
      const uintptr_t a0 = (uintptr_t)p;
      uint64_t h = (16 - (a0 & 15)) & 15;
      if (h > size) h = size;
      if (t == 0) {
        for (uint32_t q = 0; q < d; ++q) last[q] = st[q];
        for (uint64_t q = 0; q < h; ++q) {
          const uint32_t rq = uint32_t(q % d);
          last[rq] = uint8_t(last[rq] + p[q]);
          p[q] = last[rq];
        }
      }
      __syncthreads();
      V16 C{0, 0};  // byte j: last output of residue (h + j) mod d
      for (uint32_t j = 0; j < 16; ++j) {
        const uint64_t b = last[(h + j) % d];
        if (j < 8)
          C.lo |= b << (8 * j);
        else
          C.hi |= b << (8 * (j - 8));
      }
      typedef __attribute__((address_space(1))) uint64_t g64;
      for (uint64_t base = h; base < size; base += 4096) {
        const uint64_t pos = base + 16 * uint64_t(t);
        V16 x{0, 0};
        if (pos + 16 <= size) {
          x.lo = *(g64*)(p + pos);
          x.hi = *(g64*)(p + pos + 8);
        } else {
          for (uint64_t q = pos; q < size; ++q) {
            const uint64_t b = p[q];
            const uint32_t j = uint32_t(q - pos);
            if (j < 8)
              x.lo |= b << (8 * j);
            else
              x.hi |= b << (8 * (j - 8));
          }
        }
        const V16 pre = delta_lane_prefix(x, d);
        lanes[t] = delta_lane_total(pre, d);
        __syncthreads();
        for (uint32_t o = 1; o < 256; o <<= 1) {  // inclusive scan of the lane totals
          V16 v = lanes[t];
          if (t >= o) v = vadd8(v, lanes[t - o]);
          __syncthreads();
          lanes[t] = v;
          __syncthreads();
        }
        const V16 excl = t ? lanes[t - 1] : V16{0, 0};
        const V16 o = vadd8(vadd8(pre, excl), C);
        if (pos + 16 <= size) {
          *(g64*)(p + pos) = o.lo;
          *(g64*)(p + pos + 8) = o.hi;
        } else {
          for (uint64_t q = pos; q < size; ++q) {
            const uint32_t j = uint32_t(q - pos);
            p[q] = uint8_t((j < 8 ? o.lo >> (8 * j) : o.hi >> (8 * (j - 8))));
          }
        }
        C = vadd8(C, lanes[255]);
        __syncthreads();  // lanes[] is rewritten by the next tile
      }
      if (t < d) {  // residue t's last byte sits at C byte (t - h) mod d
        const uint32_t j = uint32_t((t + d - h % d) % d);
        const uint8_t b = uint8_t(j < 8 ? C.lo >> (8 * j) : C.hi >> (8 * (j - 8)));
        state[uint64_t(r) * 256 + delta_state_slot(size, d, t)] = b;
      }
    } else {  // Delta_Decode: segmented scan per residue
      DeltaSeg sg;
      const bool on = delta_seg(size, d, t, &sg);
      if (on) sums[t] = delta_seg_sum(p, d, sg);
      __syncthreads();
      if (on) {
        uint32_t carry = st[sg.r];
        for (uint32_t g = 0; g < sg.g; ++g) carry += sums[sg.r + g * d];
        const uint8_t last = delta_seg_apply(p, d, sg, uint8_t(carry));
        // the residue's last byte: from the segment holding its last position,
        // else (no positions) its state byte, kept by segment 0
        const uint64_t mr = sg.r < size ? (size - 1 - sg.r) / d + 1 : 0;
        if ((mr > 0 && sg.m0 < mr && sg.m1 == mr) || (mr == 0 && sg.g == 0))
          state[uint64_t(r) * 256 + delta_state_slot(size, d, sg.r)] = last;
      }
    }
    __syncthreads();
  }
}

// BCJ2 (Bcj2.c:28-128): one lane per job, the 258 probabilities in the
// lane's LDS slice; the main stream may be the tail of the job's output.
__global__ void __launch_bounds__(64) lzgpu_bcj2_kernel(const Bcj2GpuJob* __restrict__ jobs,
                                                       uint32_t n, int32_t* __restrict__ res) {
  __shared__ uint16_t probs[64 * 258];
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  typedef __attribute__((address_space(3))) uint16_t lds16;
  typedef __attribute__((address_space(1))) uint8_t gb;
  lds16* p = (lds16*)probs + threadIdx.x * 258;
  const Bcj2GpuJob j = jobs[i];
  res[i] = bcj2_decode((const gb*)j.buf0, j.size0, (const gb*)j.buf1, j.size1, (const gb*)j.buf2,
                       j.size2, (const gb*)j.buf3, j.size3, (gb*)j.out, j.out_size, p);
}

extern "C" int lzgpu_launch_bcj2(const Bcj2GpuJob* d_jobs, uint32_t n, int32_t* d_res,
                                 hipStream_t stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(lzgpu_bcj2_kernel, dim3((n + 63) / 64), dim3(64), 0, stream, d_jobs, n,
                     d_res);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int lzgpu_launch_bra(uint32_t kind, uint8_t* d_data, const uint64_t* d_off,
                                const uint64_t* d_len, const uint32_t* d_ip, uint64_t* d_done,
                                uint32_t n, int encoding, hipStream_t stream) {
  if (n == 0) return 0;
  if (kind == kBraARMT && getenv("LZGPU_ARMT_SERIAL")) {  // the lane-serial statement (A/B)
    hipLaunchKernelGGL(lzgpu_bra_armt_kernel, dim3((n + 63) / 64), dim3(64), 0, stream, d_data,
                       d_off, d_len, d_ip, d_done, n, encoding);
  } else {
    // a few workgroups per range; enough ranges in y to fill 256 CUs
    const uint32_t gy = n < 65535 ? n : 65535;
    const uint32_t gx = n >= 2048 ? 2 : (n >= 256 ? 8 : 64);
    hipLaunchKernelGGL(lzgpu_bra_unit_kernel, dim3(gx, gy), dim3(256), 0, stream, d_data, d_off,
                       d_len, d_ip, d_done, n, kind, encoding);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int lzgpu_launch_delta(uint8_t* d_data, const uint64_t* d_off, const uint64_t* d_len,
                                  const uint32_t* d_delta, uint8_t* d_state, uint32_t n,
                                  int encoding, hipStream_t stream) {
  if (n == 0) return 0;
  const uint32_t grid = n < 65536 ? n : 65536;
  hipLaunchKernelGGL(lzgpu_delta_kernel, dim3(grid), dim3(256), 0, stream, d_data, d_off, d_len,
                     d_delta, d_state, n, encoding);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// crc32_device.h -- CRC-32 of decoded output on the GPU.
//
// The reference's check after decode is CrcCalc (7zCrc.c:49-52: CrcUpdate
// from CRC_INIT_VAL 0xFFFFFFFF, result ^ 0xFFFFFFFF; reflected polynomial
// kCrcPoly 0xEDB88320, 7zCrc.c:7; byte step CRC_UPDATE_BYTE, 7zCrc.h:18;
// slice tables T[k][v] = T[0][T[k-1][v] & 0xFF] ^ (T[k-1][v] >> 8),
// 7zCrc.c:70-74).  Callers: 7zIn.c:1186, 1380, 1397 (folder and file CRCs).
//
// GPU formulation (own design): a range of L bytes is cut into chunks of
// kCrcChunk bytes aligned to its END, so only chunk 0 is short.  One lane per
// chunk computes the raw CRC register of its bytes (chunk 0 from the init
// value, the others from 0) with slice-by-16 tables in LDS and aligned 16-byte
// loads; a second pass folds the chunk registers of each range:
//     r = shift(r) ^ c_j,   shift(x) = x * x^(8 * kCrcChunk) mod P,
// which is exact because the CRC register is linear over GF(2)
// (R(A||B, init) = shift_|B|(R(A, init)) ^ R(B, 0)).  shift() is a
// table-driven multiply by a constant (4 lookups).
#pragma once

#include <stdint.h>

#ifdef LZGPU_HOST_EMU
#ifndef __device__
#define __device__
#define __host__
#define __forceinline__ inline
#endif
#else
#include <hip/hip_runtime.h>
#endif

namespace lzgpu {

constexpr uint32_t kCrcPoly = 0xEDB88320u;
#ifndef LZGPU_CRC_CHUNK
#define LZGPU_CRC_CHUNK 2048
#endif
#ifndef LZGPU_CRC_UNROLL
#define LZGPU_CRC_UNROLL 8
#endif
constexpr uint32_t kCrcChunk = LZGPU_CRC_CHUNK;  // bytes per chunk lane (multiple of 16)

struct CrcTables {
  uint32_t slice[16][256];  // slice[k][v]: register after byte v then k zero bytes
  uint32_t shift[4][256];   // shift[b][v] = (v << 8b) * x^(8 * kCrcChunk) mod P
};

// a * b mod P in the reflected representation (bit 31 = x^0)
__host__ __device__ constexpr uint32_t crc_mulmod(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (uint32_t m = 1u << 31; m != 0; m >>= 1) {
    if (a & m) p ^= b;
    b = (b & 1u) ? ((b >> 1) ^ kCrcPoly) : (b >> 1);
  }
  return p;
}

// x^(8 * nbytes) mod P
__host__ __device__ constexpr uint32_t crc_x8n(uint64_t nbytes) {
  uint32_t result = 1u << 31;  // x^0
  uint32_t sq = 1u << 23;      // x^8
  while (nbytes != 0) {
    if (nbytes & 1u) result = crc_mulmod(result, sq);
    sq = crc_mulmod(sq, sq);
    nbytes >>= 1;
  }
  return result;
}

__host__ __device__ constexpr CrcTables crc_make_tables() {
  CrcTables t{};
  for (uint32_t v = 0; v < 256; ++v) {
    uint32_t r = v;
    for (int j = 0; j < 8; ++j) r = (r >> 1) ^ ((r & 1u) ? kCrcPoly : 0u);
    t.slice[0][v] = r;
  }
  for (int k = 1; k < 16; ++k)
    for (uint32_t v = 0; v < 256; ++v) {
      const uint32_t r = t.slice[k - 1][v];
      t.slice[k][v] = t.slice[0][r & 0xFFu] ^ (r >> 8);
    }
  const uint32_t K = crc_x8n(kCrcChunk);
  for (int b = 0; b < 4; ++b)
    for (uint32_t v = 0; v < 256; ++v) t.shift[b][v] = crc_mulmod(K, v << (8 * b));
  return t;
}

// ---------------------------------------------------------------- per-lane code
#ifdef LZGPU_HOST_EMU
struct u32x4 {
  uint32_t x, y, z, w;
};
typedef const uint32_t lds_u32t;
__device__ __forceinline__ u32x4 load16(uintptr_t a) {
  const uint32_t* p = (const uint32_t*)a;
  return u32x4{p[0], p[1], p[2], p[3]};
}
#else
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const uint32_t lds_u32t;
__device__ __forceinline__ u32x4 load16(uintptr_t a) {
  return *(__attribute__((address_space(1))) const u32x4*)a;
}
#endif

__device__ __forceinline__ uint32_t crc_byte(uint32_t crc, uint32_t b, const lds_u32t* t0) {
  return t0[(crc ^ b) & 0xFFu] ^ (crc >> 8);
}

// bytes [k0, k1) of a 16-byte block, one at a time
__device__ __forceinline__ uint32_t crc_block_bytes(uint32_t crc, u32x4 v, uint32_t k0,
                                                    uint32_t k1, const lds_u32t* t0) {
  const uint64_t lo = uint64_t(v.x) | (uint64_t(v.y) << 32);
  const uint64_t hi = uint64_t(v.z) | (uint64_t(v.w) << 32);
  for (uint32_t k = k0; k < k1; ++k) {
    const uint32_t b = uint32_t((k < 8 ? lo >> (8 * k) : hi >> (8 * (k - 8)))) & 0xFFu;
    crc = crc_byte(crc, b, t0);
  }
  return crc;
}

// 16 bytes at once: slice[15 - i] for byte i (7zCrc.c's T8 scheme widened to 16)
__device__ __forceinline__ uint32_t crc_block16(uint32_t crc, u32x4 v, const lds_u32t* t) {
  const uint32_t x = v.x ^ crc;
  return t[15 * 256 + (x & 0xFFu)] ^ t[14 * 256 + ((x >> 8) & 0xFFu)] ^
         t[13 * 256 + ((x >> 16) & 0xFFu)] ^ t[12 * 256 + (x >> 24)] ^
         t[11 * 256 + (v.y & 0xFFu)] ^ t[10 * 256 + ((v.y >> 8) & 0xFFu)] ^
         t[9 * 256 + ((v.y >> 16) & 0xFFu)] ^ t[8 * 256 + (v.y >> 24)] ^
         t[7 * 256 + (v.z & 0xFFu)] ^ t[6 * 256 + ((v.z >> 8) & 0xFFu)] ^
         t[5 * 256 + ((v.z >> 16) & 0xFFu)] ^ t[4 * 256 + (v.z >> 24)] ^
         t[3 * 256 + (v.w & 0xFFu)] ^ t[2 * 256 + ((v.w >> 8) & 0xFFu)] ^
         t[1 * 256 + ((v.w >> 16) & 0xFFu)] ^ t[0 * 256 + (v.w >> 24)];
}

// raw CRC register over [p, e) starting from crc
__device__ __forceinline__ uint32_t crc_span(uint32_t crc, uintptr_t p, uintptr_t e,
                                             const lds_u32t* t) {
  if (p >= e) return crc;
  uintptr_t a = p & ~uintptr_t(15);
  if (a != p || e - a < 16) {
    const uint32_t k1 = e - a < 16 ? uint32_t(e - a) : 16u;
    crc = crc_block_bytes(crc, load16(a), uint32_t(p - a), k1, t);
    a += 16;
  }
  // LZGPU_CRC_UNROLL aligned 16-byte loads in flight per lane
  constexpr uint32_t U = LZGPU_CRC_UNROLL;
  while (a + 16 * U <= e) {
    u32x4 v[U];
#pragma unroll
    for (uint32_t k = 0; k < U; ++k) v[k] = load16(a + 16 * k);
#pragma unroll
    for (uint32_t k = 0; k < U; ++k) crc = crc_block16(crc, v[k], t);
    a += 16 * U;
  }
  while (a + 16 <= e) {
    crc = crc_block16(crc, load16(a), t);
    a += 16;
  }
  if (a < e) crc = crc_block_bytes(crc, load16(a), 0, uint32_t(e - a), t);
  return crc;
}

// Chunk j of a range of `len` bytes at `base` (chunks end-aligned, chunk 0
// short): its raw register, from `init` for chunk 0 and from 0 otherwise.
// Returns false for a slot beyond the range's chunk count.
__device__ __forceinline__ bool crc_chunk(const lds_u32t* t, const uint8_t* base, uint64_t len,
                                          uint32_t j, uint32_t init, uint32_t* out) {
  const uint64_t nch = (len + kCrcChunk - 1) / kCrcChunk;
  if (j >= nch) return false;
  const uint64_t hi = len - (nch - 1 - j) * kCrcChunk;
  const uint64_t lo = j == 0 ? 0 : hi - kCrcChunk;
  const uintptr_t b = (uintptr_t)base;
  *out = crc_span(j == 0 ? init : 0u, b + lo, b + hi, t);
  return true;
}

// Register after the whole range: fold of its chunk registers c[0..nch)
// (sh = CrcTables::shift flattened); `init` for an empty range.
__device__ __forceinline__ uint32_t crc_fold(const lds_u32t* sh, const uint32_t* c, uint64_t len,
                                             uint32_t init) {
  const uint32_t nch = uint32_t((len + kCrcChunk - 1) / kCrcChunk);
  if (nch == 0) return init;
  uint32_t r = c[0];
  for (uint32_t j = 1; j < nch; ++j)
    r = sh[r & 0xFFu] ^ sh[256 + ((r >> 8) & 0xFFu)] ^ sh[512 + ((r >> 16) & 0xFFu)] ^
        sh[768 + (r >> 24)] ^ c[j];
  return r;
}

}  // namespace lzgpu

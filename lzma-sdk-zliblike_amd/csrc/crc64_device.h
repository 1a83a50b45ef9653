// crc64_device.h -- CRC-64 of decoded xz blocks on the GPU (SURVEY.md 8(f)
// row 3: the xz block check XZ_CHECK_CRC64).
//
// The reference check is Crc64Calc (XzCrc64.c:30: Crc64Update from
// CRC64_INIT_VAL ~0, result ^ ~0; reflected polynomial kCrc64Poly
// 0xC96C5795D7870F42, XzCrc64.c:6; byte step CRC64_UPDATE_BYTE,
// XzCrc64.h:16), used by XzCheck_Update / XzCheck_Final (Xz.c:55-85).
//
// Same GPU formulation as crc32_device.h with a 64-bit register: a range is
// cut into kCrc64Chunk-byte chunks aligned to its end, one lane per chunk
// computes the raw register with slice-by-8 tables in LDS (two 8-byte steps
// per aligned 16-byte load), and a fold pass combines the chunk registers
//     r = shift(r) ^ c_j,   shift(x) = x * x^(8 * kCrc64Chunk) mod P
// (exact: the register is linear over GF(2)), shift() by 8 table lookups.
#pragma once

#include <stdint.h>

#include "crc32_device.h"  // u32x4, load16, host-emulation macros

namespace lzgpu {

constexpr uint64_t kCrc64Poly = 0xC96C5795D7870F42ull;
constexpr uint32_t kCrc64Chunk = 2048;  // bytes per chunk lane (multiple of 16)
#ifndef LZGPU_CRC64_UNROLL
#define LZGPU_CRC64_UNROLL 8
#endif

struct Crc64Tables {
  uint64_t slice[8][256];  // slice[k][v]: register after byte v then k zero bytes
  uint64_t shift[8][256];  // shift[b][v] = (v << 8b) * x^(8 * kCrc64Chunk) mod P
};

// a * b mod P in the reflected representation (bit 63 = x^0)
__host__ __device__ constexpr uint64_t crc64_mulmod(uint64_t a, uint64_t b) {
  uint64_t p = 0;
  for (uint64_t m = 1ull << 63; m != 0; m >>= 1) {
    if (a & m) p ^= b;
    b = (b & 1u) ? ((b >> 1) ^ kCrc64Poly) : (b >> 1);
  }
  return p;
}

// x^(8 * nbytes) mod P
__host__ __device__ constexpr uint64_t crc64_x8n(uint64_t nbytes) {
  uint64_t result = 1ull << 63;  // x^0
  uint64_t sq = 1ull << 55;      // x^8
  while (nbytes != 0) {
    if (nbytes & 1u) result = crc64_mulmod(result, sq);
    sq = crc64_mulmod(sq, sq);
    nbytes >>= 1;
  }
  return result;
}

__host__ __device__ constexpr Crc64Tables crc64_make_tables() {
  Crc64Tables t{};
  for (uint32_t v = 0; v < 256; ++v) {
    uint64_t r = v;
    for (int j = 0; j < 8; ++j) r = (r >> 1) ^ ((r & 1u) ? kCrc64Poly : 0ull);
    t.slice[0][v] = r;
  }
  for (int k = 1; k < 8; ++k)
    for (uint32_t v = 0; v < 256; ++v) {
      const uint64_t r = t.slice[k - 1][v];
      t.slice[k][v] = t.slice[0][r & 0xFFu] ^ (r >> 8);
    }
  const uint64_t K = crc64_x8n(kCrc64Chunk);
  for (int b = 0; b < 8; ++b)
    for (uint32_t v = 0; v < 256; ++v) t.shift[b][v] = crc64_mulmod(K, uint64_t(v) << (8 * b));
  return t;
}

#ifdef LZGPU_HOST_EMU
typedef const uint64_t lds_u64t;
#else
typedef __attribute__((address_space(3))) const uint64_t lds_u64t;
#endif

__device__ __forceinline__ uint64_t crc64_byte(uint64_t crc, uint32_t b, const lds_u64t* t0) {
  return t0[(crc ^ b) & 0xFFu] ^ (crc >> 8);
}

// 8 bytes (little-endian word w) at once: slice[7 - i] for byte i
__device__ __forceinline__ uint64_t crc64_word(uint64_t crc, uint64_t w, const lds_u64t* t) {
  const uint64_t x = w ^ crc;
  return t[7 * 256 + (x & 0xFFu)] ^ t[6 * 256 + ((x >> 8) & 0xFFu)] ^
         t[5 * 256 + ((x >> 16) & 0xFFu)] ^ t[4 * 256 + ((x >> 24) & 0xFFu)] ^
         t[3 * 256 + ((x >> 32) & 0xFFu)] ^ t[2 * 256 + ((x >> 40) & 0xFFu)] ^
         t[1 * 256 + ((x >> 48) & 0xFFu)] ^ t[0 * 256 + (x >> 56)];
}

__device__ __forceinline__ uint64_t crc64_block16(uint64_t crc, u32x4 v, const lds_u64t* t) {
  crc = crc64_word(crc, uint64_t(v.x) | (uint64_t(v.y) << 32), t);
  return crc64_word(crc, uint64_t(v.z) | (uint64_t(v.w) << 32), t);
}

// bytes [k0, k1) of a 16-byte block, one at a time
__device__ __forceinline__ uint64_t crc64_block_bytes(uint64_t crc, u32x4 v, uint32_t k0,
                                                      uint32_t k1, const lds_u64t* t0) {
  const uint64_t lo = uint64_t(v.x) | (uint64_t(v.y) << 32);
  const uint64_t hi = uint64_t(v.z) | (uint64_t(v.w) << 32);
  for (uint32_t k = k0; k < k1; ++k) {
    const uint32_t b = uint32_t((k < 8 ? lo >> (8 * k) : hi >> (8 * (k - 8)))) & 0xFFu;
    crc = crc64_byte(crc, b, t0);
  }
  return crc;
}

// raw CRC-64 register over [p, e) starting from crc (aligned 16-byte loads;
// an aligned block holding a valid byte never crosses a page)
__device__ __forceinline__ uint64_t crc64_span(uint64_t crc, uintptr_t p, uintptr_t e,
                                               const lds_u64t* t) {
  if (p >= e) return crc;
  uintptr_t a = p & ~uintptr_t(15);
  if (a != p || e - a < 16) {
    const uint32_t k1 = e - a < 16 ? uint32_t(e - a) : 16u;
    crc = crc64_block_bytes(crc, load16(a), uint32_t(p - a), k1, t);
    a += 16;
  }
  // LZGPU_CRC64_UNROLL aligned 16-byte loads in flight per lane
  constexpr uint32_t U = LZGPU_CRC64_UNROLL;
  while (a + 16 * U <= e) {
    u32x4 v[U];
#pragma unroll
    for (uint32_t k = 0; k < U; ++k) v[k] = load16(a + 16 * k);
#pragma unroll
    for (uint32_t k = 0; k < U; ++k) crc = crc64_block16(crc, v[k], t);
    a += 16 * U;
  }
  while (a + 16 <= e) {
    crc = crc64_block16(crc, load16(a), t);
    a += 16;
  }
  if (a < e) crc = crc64_block_bytes(crc, load16(a), 0, uint32_t(e - a), t);
  return crc;
}

// chunk j of a range of `len` bytes at `base` (end-aligned chunks, chunk 0 short)
__device__ __forceinline__ bool crc64_chunk(const lds_u64t* t, const uint8_t* base, uint64_t len,
                                            uint32_t j, uint64_t init, uint64_t* out) {
  const uint64_t nch = (len + kCrc64Chunk - 1) / kCrc64Chunk;
  if (j >= nch) return false;
  const uint64_t hi = len - (nch - 1 - j) * kCrc64Chunk;
  const uint64_t lo = j == 0 ? 0 : hi - kCrc64Chunk;
  const uintptr_t b = (uintptr_t)base;
  *out = crc64_span(j == 0 ? init : 0ull, b + lo, b + hi, t);
  return true;
}

// register after the whole range: fold of its chunk registers (sh = shift
// tables flattened); `init` for an empty range
__device__ __forceinline__ uint64_t crc64_fold(const lds_u64t* sh, const uint64_t* c,
                                               uint64_t len, uint64_t init) {
  const uint32_t nch = uint32_t((len + kCrc64Chunk - 1) / kCrc64Chunk);
  if (nch == 0) return init;
  uint64_t r = c[0];
  for (uint32_t j = 1; j < nch; ++j) {
    uint64_t s = 0;
#pragma unroll
    for (int b = 0; b < 8; ++b) s ^= sh[b * 256 + ((r >> (8 * b)) & 0xFFu)];
    r = s ^ c[j];
  }
  return r;
}

}  // namespace lzgpu

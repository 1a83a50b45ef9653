// bra_device.h -- the RISC branch converters and the delta filter for the GPU
// (beyond x86).
//
// Restates Bra.c (ARM_Convert :6-31, ARMT_Convert :33-66, PPC_Convert :68-97,
// SPARC_Convert :99-133), BraIA64.c (IA64_Convert :14-67) and Delta.c
// (Delta_Decode :42-62, Delta_Encode :20-40).  The kind numbers are the xz
// filter IDs (Xz.h: PPC 5, IA64 6, ARM 7, ARMT 8, SPARC 9).
//
// ARM, PPC, SPARC (one 32-bit word) and IA64 (one 16-byte bundle) convert
// every aligned unit on its own: the unit at offset i depends only on its own
// bytes and ip + i, so the batch kernel gives each unit its own lane.  ARMT
// looks serial (a converted pair skips the next halfword, Bra.c:63) but is not:
// a candidate at even i needs byte i+1 = 11110xxx and byte i+3 = 11111xxx, so
// the candidates at i-2 and i+2 are impossible next to one at i (they need the
// other pattern in the same byte), the skip never skips a candidate, and a
// conversion rewrites only the even bytes and the low 3 bits of the odd ones,
// which no other candidate reads or tests.  So every even position is its own
// lane too (bra_armt_at), and the serial bra_armt below is kept as its
// statement.  Delta is a running sum per residue class modulo `delta`: one lane
// per (range, residue).
#pragma once

#include <stdint.h>

#include "crc32_device.h"  // host-emulation macros

namespace lzgpu {

enum : uint32_t { kBraPPC = 5, kBraIA64 = 6, kBraARM = 7, kBraARMT = 8, kBraSPARC = 9 };

#ifdef LZGPU_HOST_EMU
typedef uint8_t bra_byte;
#else
typedef __attribute__((address_space(1))) uint8_t bra_byte;
#endif

// unit size and the bytes Convert returns for a buffer of `size` bytes
// (the last unit that fits entirely; nothing when size < one unit)
// (ARMT: `units` candidate positions 2 bytes apart, each reading 4 bytes)
__host__ __device__ inline uint32_t bra_unit(uint32_t kind) {
  return kind == kBraIA64 ? 16u : (kind == kBraARMT ? 2u : 4u);
}
__host__ __device__ inline uint64_t bra_done_units(uint32_t kind, uint64_t size) {
  const uint64_t u = bra_unit(kind), need = kind == kBraARMT ? 4 : u;
  return size < need ? 0 : (size - need) / u + 1;
}

// ARM BL (Bra.c:15-29): byte 3 == 0xEB, 24-bit word offset, ip + 8
template <typename B>
__device__ __forceinline__ void bra_arm_word(B* p, uint32_t pos, int encoding) {
  if (p[3] != 0xEB) return;
  const uint32_t src = ((uint32_t(p[2]) << 16) | (uint32_t(p[1]) << 8) | p[0]) << 2;
  uint32_t dest = encoding ? pos + 8 + src : src - (pos + 8);
  dest >>= 2;
  p[2] = uint8_t(dest >> 16);
  p[1] = uint8_t(dest >> 8);
  p[0] = uint8_t(dest);
}

// PPC "bl" (Bra.c:76-95): opcode 18 with AA=0, LK=1, big-endian word
template <typename B>
__device__ __forceinline__ void bra_ppc_word(B* p, uint32_t pos, int encoding) {
  const uint32_t b0 = p[0], b3 = p[3];
  if ((b0 >> 2) != 0x12 || (b3 & 3) != 1) return;
  const uint32_t src = ((b0 & 3) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | (b3 & ~3u);
  const uint32_t dest = encoding ? pos + src : src - pos;
  p[0] = uint8_t(0x48 | ((dest >> 24) & 0x3));
  p[1] = uint8_t(dest >> 16);
  p[2] = uint8_t(dest >> 8);
  p[3] = uint8_t((b3 & 0x3) | (dest & 0xFF));
}

// SPARC "call" (Bra.c:107-130): 0x40 / 0x7F prefixes with a sign-consistent byte 1
template <typename B>
__device__ __forceinline__ void bra_sparc_word(B* p, uint32_t pos, int encoding) {
  const uint32_t b0 = p[0], b1 = p[1];
  if (!((b0 == 0x40 && (b1 & 0xC0) == 0x00) || (b0 == 0x7F && (b1 & 0xC0) == 0xC0))) return;
  const uint32_t src = ((b0 << 24) | (b1 << 16) | (uint32_t(p[2]) << 8) | p[3]) << 2;
  uint32_t dest = encoding ? pos + src : src - pos;
  dest >>= 2;
  dest = (((0u - ((dest >> 22) & 1u)) << 22) & 0x3FFFFFFFu) | (dest & 0x3FFFFFu) | 0x40000000u;
  p[0] = uint8_t(dest >> 24);
  p[1] = uint8_t(dest >> 16);
  p[2] = uint8_t(dest >> 8);
  p[3] = uint8_t(dest);
}

// IA64 bundle (BraIA64.c:23-64): the template picks the slots that may hold a
// branch (kBranchTable, :6-12, packed as one nibble per template)
__device__ __forceinline__ void bra_ia64_bundle(bra_byte* p, uint32_t pos, int encoding) {
  // kBranchTable[16..31] = 4,4,6,6,0,0,7,7,4,4,0,0,4,4,0,0; entries 0..15 are 0
  const uint32_t t = p[0] & 0x1Fu;
  const uint64_t kHi = 0x0044004477006644ull;  // nibble (t - 16) = kBranchTable[t]
  const uint32_t mask = t < 16 ? 0u : uint32_t(kHi >> (4 * (t - 16))) & 0xFu;
  uint32_t bit_pos = 5;
  for (int slot = 0; slot < 3; ++slot, bit_pos += 41) {
    if (((mask >> slot) & 1u) == 0) continue;
    const uint32_t byte_pos = bit_pos >> 3, bit_res = bit_pos & 7u;
    uint64_t instruction = 0;
    for (int j = 0; j < 6; ++j) instruction |= uint64_t(p[byte_pos + j]) << (8 * j);
    uint64_t norm = instruction >> bit_res;
    if (((norm >> 37) & 0xF) != 0x5 || ((norm >> 9) & 0x7) != 0) continue;
    uint32_t src = uint32_t((norm >> 13) & 0xFFFFF);
    src |= (uint32_t(norm >> 36) & 1u) << 20;
    src <<= 4;
    uint32_t dest = encoding ? pos + src : src - pos;
    dest >>= 4;
    norm &= ~(uint64_t(0x8FFFFF) << 13);
    norm |= uint64_t(dest & 0xFFFFF) << 13;
    norm |= uint64_t(dest & 0x100000) << (36 - 20);
    instruction &= (uint64_t(1) << bit_res) - 1;
    instruction |= norm << bit_res;
    for (int j = 0; j < 6; ++j) p[byte_pos + j] = uint8_t(instruction >> (8 * j));
  }
}

__device__ __forceinline__ bool bra_armt_candidate(const bra_byte* p) {
  return (p[1] & 0xF8) == 0xF0 && (p[3] & 0xF8) == 0xF8;
}

// ARMT BL pair at even offset i (pos = ip + i): Bra.c:42-62 for one position
__device__ __forceinline__ void bra_armt_at(bra_byte* p, uint32_t pos, int encoding) {
  if (!bra_armt_candidate(p)) return;
  uint32_t src = ((uint32_t(p[1]) & 7u) << 19) | (uint32_t(p[0]) << 11) |
                 ((uint32_t(p[3]) & 7u) << 8) | p[2];
  src <<= 1;
  uint32_t dest = encoding ? pos + 4 + src : src - (pos + 4);
  dest >>= 1;
  p[1] = uint8_t(0xF0 | ((dest >> 19) & 0x7));
  p[0] = uint8_t(dest >> 11);
  p[3] = uint8_t(0xF8 | ((dest >> 8) & 0x7));
  p[2] = uint8_t(dest);
}

// what ARMT_Convert returns: one past the last position tested, + 2 when that
// position converted (its skip); `units` = bra_done_units(kBraARMT, size)
__device__ __forceinline__ uint64_t bra_armt_done(const bra_byte* data, uint64_t units) {
  if (units == 0) return 0;
  const uint64_t last = 2 * (units - 1);
  return last + 2 + (bra_armt_candidate(data + last) ? 2 : 0);
}

// ARM / PPC / SPARC on a word held in a register (one 32-bit load, a store
// only when the word changed): `p` 4-byte aligned
__device__ __forceinline__ void bra_word_aligned(uint32_t kind, bra_byte* p, uint32_t pos,
                                                 int encoding) {
#ifdef LZGPU_HOST_EMU
  uint32_t w;
  __builtin_memcpy(&w, p, 4);
#else
  const uint32_t w = *(const __attribute__((address_space(1))) uint32_t*)p;
#endif
  uint8_t b[4] = {uint8_t(w), uint8_t(w >> 8), uint8_t(w >> 16), uint8_t(w >> 24)};
  if (kind == kBraARM)
    bra_arm_word(b, pos, encoding);
  else if (kind == kBraPPC)
    bra_ppc_word(b, pos, encoding);
  else
    bra_sparc_word(b, pos, encoding);
  const uint32_t o = uint32_t(b[0]) | (uint32_t(b[1]) << 8) | (uint32_t(b[2]) << 16) |
                     (uint32_t(b[3]) << 24);
  if (o == w) return;
#ifdef LZGPU_HOST_EMU
  __builtin_memcpy(p, &o, 4);
#else
  *(__attribute__((address_space(1))) uint32_t*)p = o;
#endif
}

// one unit of a word-parallel kind at byte offset i of a range starting at ip
__device__ __forceinline__ void bra_unit_convert(uint32_t kind, bra_byte* p, uint32_t pos,
                                                 int encoding) {
  switch (kind) {
    case kBraARM: bra_arm_word(p, pos, encoding); break;
    case kBraPPC: bra_ppc_word(p, pos, encoding); break;
    case kBraSPARC: bra_sparc_word(p, pos, encoding); break;
    case kBraARMT: bra_armt_at(p, pos, encoding); break;
    default: bra_ia64_bundle(p, pos, encoding); break;
  }
}

// ARMT_Convert (Bra.c:33-66) over one range: BL pairs of Thumb halfwords; a
// converted pair is skipped, so the scan is serial.  Returns the bytes done.
__device__ inline uint64_t bra_armt(bra_byte* data, uint64_t size, uint32_t ip, int encoding) {
  if (size < 4) return 0;
  const uint64_t last = size - 4;
  ip += 4;
  uint64_t i = 0;
  for (; i <= last; i += 2) {
    if ((data[i + 1] & 0xF8) != 0xF0 || (data[i + 3] & 0xF8) != 0xF8) continue;
    uint32_t src = ((uint32_t(data[i + 1]) & 7u) << 19) | (uint32_t(data[i + 0]) << 11) |
                   ((uint32_t(data[i + 3]) & 7u) << 8) | data[i + 2];
    src <<= 1;
    uint32_t dest = encoding ? ip + uint32_t(i) + src : src - (ip + uint32_t(i));
    dest >>= 1;
    data[i + 1] = uint8_t(0xF0 | ((dest >> 19) & 0x7));
    data[i + 0] = uint8_t(dest >> 11);
    data[i + 3] = uint8_t(0xF8 | ((dest >> 8) & 0x7));
    data[i + 2] = uint8_t(dest);
    i += 2;
  }
  return i;
}

// Delta_Decode / Delta_Encode (Delta.c:20-62) for residue r of a range:
// positions r, r + delta, ... start from state[r] (the byte `delta` before
// position 0).  Decode: out = in + prev; encode: out = in - prev(in).  Returns
// the residue's last state byte (decoded byte for decode, input for encode).
__device__ inline uint8_t delta_residue(bra_byte* data, uint64_t size, uint32_t delta, uint32_t r,
                                     uint8_t prev, int encoding) {
  for (uint64_t i = r; i < size; i += delta) {
    const uint8_t b = data[i];
    if (encoding) {
      data[i] = uint8_t(b - prev);
      prev = b;
    } else {
      prev = uint8_t(prev + b);
      data[i] = prev;
    }
  }
  return prev;
}

// Delta_Decode as a segmented scan: lane t of a workgroup takes residue
// r = t % delta and segment g = t / delta of that residue's positions
// (G = floor(256 / delta) segments of `chunk` positions each).  Pass 1 sums a
// segment (mod 256); the carry into it is the residue's state byte plus the
// sums of the earlier segments; pass 2 rewrites the segment as a running sum.
struct DeltaSeg {
  uint32_t r, g, G;
  uint64_t m0, m1;  // positions r + m * delta, m in [m0, m1)
};
__host__ __device__ inline bool delta_seg(uint64_t size, uint32_t delta, uint32_t t, DeltaSeg* s) {
  const uint32_t G = 256u / delta;
  if (t >= delta * G) return false;
  s->r = t % delta;
  s->g = t / delta;
  s->G = G;
  const uint64_t mmax = (size + delta - 1) / delta;
  const uint64_t chunk = (mmax + G - 1) / G;
  const uint64_t mr = s->r < size ? (size - 1 - s->r) / delta + 1 : 0;
  s->m0 = uint64_t(s->g) * chunk;
  s->m1 = s->m0 + chunk < mr ? s->m0 + chunk : mr;
  if (s->m0 > s->m1) s->m0 = s->m1;
  return true;
}
__device__ inline uint8_t delta_seg_sum(const bra_byte* data, uint32_t delta, const DeltaSeg& s) {
  uint32_t acc = 0;
  for (uint64_t m = s.m0; m < s.m1; ++m) acc += data[s.r + m * delta];
  return uint8_t(acc);
}
__device__ inline uint8_t delta_seg_apply(bra_byte* data, uint32_t delta, const DeltaSeg& s,
                                          uint8_t carry) {
  for (uint64_t m = s.m0; m < s.m1; ++m) {
    carry = uint8_t(carry + data[s.r + m * delta]);
    data[s.r + m * delta] = carry;
  }
  return carry;
}

// Delta_Decode for d | 16 as a tile scan over 16-byte lane vectors (two u64
// halves, little-endian byte order = position order).  Byte-wise adds are SWAR
// (no carry between bytes); a lane's inclusive prefix at distance d is log-step
// x += x << 8d; its contribution to later lanes is its top d bytes repeated
// with period d (d | 16 keeps every lane's byte j on residue (start + j) mod d).
struct V16 {
  uint64_t lo, hi;
};
__host__ __device__ inline uint64_t add8(uint64_t a, uint64_t b) {
  const uint64_t H = 0x8080808080808080ull;
  return ((a & ~H) + (b & ~H)) ^ ((a ^ b) & H);
}
__host__ __device__ inline V16 vadd8(V16 a, V16 b) { return V16{add8(a.lo, b.lo), add8(a.hi, b.hi)}; }
__host__ __device__ inline V16 vshl_bytes(V16 a, uint32_t n) {  // toward higher positions, n < 16
  if (n == 0) return a;
  if (n >= 8) return V16{0, a.lo << (8 * (n - 8))};
  return V16{a.lo << (8 * n), (a.hi << (8 * n)) | (a.lo >> (64 - 8 * n))};
}
__host__ __device__ inline V16 delta_lane_prefix(V16 x, uint32_t d) {
  for (uint32_t s = d; s < 16; s <<= 1) x = vadd8(x, vshl_bytes(x, s));
  return x;
}
// top d bytes of a lane prefix repeated with period d (bytes 16-d .. 15)
__host__ __device__ inline V16 delta_lane_total(V16 pre, uint32_t d) {
  uint8_t b[16], t[16];
  for (int j = 0; j < 8; ++j) {
    b[j] = uint8_t(pre.lo >> (8 * j));
    b[8 + j] = uint8_t(pre.hi >> (8 * j));
  }
  for (uint32_t j = 0; j < 16; ++j) t[j] = b[16 - d + (j % d)];
  V16 o{0, 0};
  for (int j = 0; j < 8; ++j) {
    o.lo |= uint64_t(t[j]) << (8 * j);
    o.hi |= uint64_t(t[8 + j]) << (8 * j);
  }
  return o;
}

// where residue r's returned byte goes in the new state: its last position q
// in [size - delta, size) of (old state ++ data), i.e. state[q + delta - size]
__host__ __device__ inline uint32_t delta_state_slot(uint64_t size, uint32_t delta, uint32_t r) {
  const int64_t q = uint64_t(r) < size ? int64_t(r + delta * ((size - 1 - r) / delta))
                                       : int64_t(r) - int64_t(delta);
  return uint32_t(q + int64_t(delta) - int64_t(size));
}

}  // namespace lzgpu

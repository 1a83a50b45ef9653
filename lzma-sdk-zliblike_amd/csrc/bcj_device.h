// bcj_device.h -- x86 BCJ branch converter for one lane.
//
// Restates x86_Convert (Bra86.c:11-85): E8 (call) / E9 (jmp) rel32 operands
// whose top byte is 0x00 or 0xFF are turned between relative and absolute
// form (decode: dest = src - (ip + pos + 5)); `state` carries the positions
// of the last three E8/E9 bytes (prevMask) across calls; the last four bytes
// of a buffer are never converted (an instruction needs five), so the caller
// feeds them again with the next piece.  kMaskToAllowedStatus /
// kMaskToBitNumber are the reference's tables (Bra86.c:8-9).
//
// Memory access: the scan reads a 32-byte register window refilled from
// aligned 16-byte loads and tests eight bytes per step for E8/E9 (SWAR); the
// operand bytes it looks ahead at (<= 4) are always inside the window; a
// conversion rewrites four bytes with one unaligned 32-bit store.  Bytes a
// conversion rewrites are behind the scan afterwards, so the stale window
// copies are never read again.
#pragma once

#include <stdint.h>

#include "crc32_device.h"  // u32x4, load16, host-emulation macros

namespace lzgpu {

#ifdef LZGPU_HOST_EMU
typedef uint8_t bcj_byte;
#else
typedef __attribute__((address_space(1))) uint8_t bcj_byte;
#endif

struct BcjWindow {
  uintptr_t base;  // 16-byte aligned address of w[0]
  uintptr_t end;   // one past the buffer
  uint64_t w[4];   // 32 bytes from base
  __device__ __forceinline__ void fill(uint32_t half, uintptr_t a) {
    // a whole aligned block beyond the buffer is never loaded
    u32x4 v;
    if (a < end) {
      v = load16(a);
    } else {
      v.x = v.y = v.z = v.w = 0;
    }
    w[2 * half] = uint64_t(v.x) | (uint64_t(v.y) << 32);
    w[2 * half + 1] = uint64_t(v.z) | (uint64_t(v.w) << 32);
  }
  __device__ __forceinline__ void init(uintptr_t p, uintptr_t e) {
    base = p & ~uintptr_t(15);
    end = e;
    fill(0, base);
    fill(1, base + 16);
  }
  // byte at address a (base <= a < base + 32 after slide(a))
  __device__ __forceinline__ uint32_t at(uintptr_t a) const {
    const uint32_t o = uint32_t(a - base);
    const uint64_t q = (o & 16) ? ((o & 8) ? w[3] : w[2]) : ((o & 8) ? w[1] : w[0]);
    return uint32_t(q >> (8 * (o & 7))) & 0xFFu;
  }
  // bytes [a, a + 8) as a little-endian word (after slide(a))
  __device__ __forceinline__ uint64_t word(uintptr_t a) const {
    const uint32_t o = uint32_t(a - base), i = o >> 3, sh = 8 * (o & 7);
    const uint64_t lo = (i & 2) ? ((i & 1) ? w[3] : w[2]) : ((i & 1) ? w[1] : w[0]);
    const uint64_t hi = (i & 2) ? w[3] : ((i & 1) ? w[2] : w[1]);
    return sh ? ((lo >> sh) | (hi << (64 - sh))) : lo;
  }
  // make [a, a + 8) readable
  __device__ __forceinline__ void slide(uintptr_t a) {
    while (a + 8 > base + 32) {
      w[0] = w[2];
      w[1] = w[3];
      base += 16;
      fill(1, base + 16);
    }
  }
};

__device__ __forceinline__ bool bcj_test_ms(uint32_t b) { return b == 0 || b == 0xFF; }

// x86_Convert over data[0, size): returns the bytes processed, state in/out.
__device__ inline uint64_t bcj_x86(bcj_byte* data, uint64_t size, uint32_t ip, uint32_t* state,
                                   int encoding) {
  // kMaskToAllowedStatus = {1,1,1,0,1,0,0,0}, kMaskToBitNumber = {0,1,2,2,3,3,3,3}
  constexpr uint32_t kAllowed = 0x17u;  // bit m set = kMaskToAllowedStatus[m]
  auto bitnum = [](uint32_t m) -> uint32_t {  // kMaskToBitNumber[m]
    return m == 0 ? 0u : (m == 1 ? 1u : (m < 4 ? 2u : 3u));
  };
  uint32_t prev_mask = *state & 7u;
  if (size < 5) return 0;
  ip += 5;
  const uintptr_t d0 = (uintptr_t)data;
  BcjWindow win;
  win.init(d0, d0 + size);
  uint64_t pos = 0, prev_pos = ~uint64_t(0);
  const uint64_t limit = size - 4;
  for (;;) {
    // scan for E8 / E9 eight bytes at a time: x has a zero byte exactly where
    // the byte is E8 or E9, and the lowest set bit of the has-zero mask marks
    // the first of them (higher bits may be borrow artefacts, never lower)
    const uint64_t scan0 = pos;
    while (pos < limit) {
      win.slide(d0 + pos);
      const uint64_t x = (win.word(d0 + pos) & 0xFEFEFEFEFEFEFEFEull) ^ 0xE8E8E8E8E8E8E8E8ull;
      const uint64_t z = (x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull;
      if (z != 0) {
        pos += uint64_t(__builtin_ctzll(z) >> 3);
        break;
      }
      pos += 8;
    }
    if (pos >= limit) {
      // the byte-wise scan stops at limit; a conversion may have left pos beyond it
      pos = scan0 < limit ? limit : scan0;
      break;
    }
    win.slide(d0 + pos);  // the operand bytes pos + 1 .. pos + 4
    uint64_t gap = pos - prev_pos;
    if (gap > 3) {
      prev_mask = 0;
    } else {
      prev_mask = (prev_mask << (uint32_t(gap) - 1)) & 7u;
      if (prev_mask != 0) {
        const uint32_t b = win.at(d0 + pos + 4 - bitnum(prev_mask));
        if (!((kAllowed >> prev_mask) & 1u) || bcj_test_ms(b)) {
          prev_pos = pos;
          prev_mask = ((prev_mask << 1) & 7u) | 1u;
          ++pos;
          continue;
        }
      }
    }
    prev_pos = pos;
    const uint32_t b4 = win.at(d0 + pos + 4);
    if (bcj_test_ms(b4)) {
      uint32_t src = (b4 << 24) | (win.at(d0 + pos + 3) << 16) | (win.at(d0 + pos + 2) << 8) |
                     win.at(d0 + pos + 1);
      uint32_t dest;
      for (;;) {
        if (encoding)
          dest = (ip + uint32_t(pos)) + src;
        else
          dest = src - (ip + uint32_t(pos));
        if (prev_mask == 0) break;
        const uint32_t index = bitnum(prev_mask) * 8;
        const uint32_t b = (dest >> (24 - index)) & 0xFFu;
        if (!bcj_test_ms(b)) break;
        src = dest ^ ((1u << (32 - index)) - 1u);
      }
      const uint32_t out = (dest & 0x00FFFFFFu) | ((~(((dest >> 24) & 1u) - 1u)) << 24);
#ifdef LZGPU_HOST_EMU
      __builtin_memcpy(data + pos + 1, &out, 4);
#else
      typedef uint32_t u32a1 __attribute__((aligned(1)));
      *(__attribute__((address_space(1))) u32a1*)(data + pos + 1) = out;
#endif
      pos += 5;
    } else {
      prev_mask = ((prev_mask << 1) & 7u) | 1u;
      ++pos;
    }
  }
  const uint64_t gap = pos - prev_pos;
  *state = (gap > 3) ? 0u : ((prev_mask << (uint32_t(gap) - 1)) & 7u);
  return pos;
}

// ------------------------------------------------------------------ tiled form
//
// x86_Convert reads a byte only at or after the position it scans next, and
// writes a converted operand (positions h+1..h+4) only behind that position
// (the scan resumes at h+5): every byte it reads is still the original.  So
// the E8/E9 positions of a range and their four operand bytes can be found
// for a whole tile at once by every lane of a workgroup (lzgpu_bcj_x86_tile
// _kernel), and the reference's decisions then run hit by hit over that list
// -- bcj_hit below, one lane, with the state of x86_Convert's loop carried:
// the position the scan resumes at, the last hit and prevMask.  Hits the list
// holds before the resume position (inside a converted operand, or bytes an
// earlier tile's conversion rewrote) are skipped, as the byte scan skips them.
struct BcjRun {
  uint64_t resume;    // bufferPos at the top of the reference's loop
  uint64_t prev_pos;  // prevPosT (~0 before the first hit)
  uint32_t mask;      // prevMask
};

// One E8/E9 at h (< size - 4) with operand bytes op = h+1 .. h+4 (byte h+1 in
// bits 0-7): the reference's loop body (Bra86.c:33-84).  Returns true and the
// new operand in *out when the hit converts.
__device__ __forceinline__ bool bcj_hit(BcjRun& r, uint64_t h, uint32_t op, uint32_t ip,
                                        int encoding, uint32_t* out) {
  constexpr uint32_t kAllowed = 0x17u;  // kMaskToAllowedStatus as bits
  auto bitnum = [](uint32_t m) -> uint32_t {
    return m == 0 ? 0u : (m == 1 ? 1u : (m < 4 ? 2u : 3u));
  };
  const uint64_t gap = h - r.prev_pos;
  if (gap > 3) {
    r.mask = 0;
  } else {
    r.mask = (r.mask << (uint32_t(gap) - 1)) & 7u;
    if (r.mask != 0) {
      const uint32_t b = (op >> (8 * (3 - bitnum(r.mask)))) & 0xFFu;  // p[4 - bitnum]
      if (!((kAllowed >> r.mask) & 1u) || bcj_test_ms(b)) {
        r.prev_pos = h;
        r.mask = ((r.mask << 1) & 7u) | 1u;
        r.resume = h + 1;
        return false;
      }
    }
  }
  r.prev_pos = h;
  const uint32_t b4 = op >> 24;
  if (!bcj_test_ms(b4)) {
    r.mask = ((r.mask << 1) & 7u) | 1u;
    r.resume = h + 1;
    return false;
  }
  uint32_t src = op, dest;
  const uint32_t at = ip + uint32_t(h);  // ip already + 5
  for (;;) {
    dest = encoding ? at + src : src - at;
    if (r.mask == 0) break;
    const uint32_t index = bitnum(r.mask) * 8;
    const uint32_t b = (dest >> (24 - index)) & 0xFFu;
    if (!bcj_test_ms(b)) break;
    src = dest ^ ((1u << (32 - index)) - 1u);
  }
  *out = (dest & 0x00FFFFFFu) | ((~(((dest >> 24) & 1u) - 1u)) << 24);
  r.resume = h + 5;
  return true;
}

// The loop's end (Bra86.c:85-89): bytes processed and the state carried out.
__device__ __forceinline__ uint64_t bcj_finish(const BcjRun& r, uint64_t limit, uint32_t* state) {
  const uint64_t pos = r.resume > limit ? r.resume : limit;
  const uint64_t gap = pos - r.prev_pos;
  *state = (gap > 3) ? 0u : ((r.mask << (uint32_t(gap) - 1)) & 7u);
  return pos;
}

}  // namespace lzgpu

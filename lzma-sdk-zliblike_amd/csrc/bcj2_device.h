// bcj2_device.h -- BCJ2 x86 branch decoder for one lane.
//
// Restates Bcj2_Decode (Bcj2.c:28-128): four input streams --
//   buf0  the main stream (every byte that is not a converted operand),
//   buf1  the CALL (E8) operands, buf2 the JMP (E9) / Jcc (0F 8x) operands,
//         4-byte big-endian absolute targets,
//   buf3  a range-coded bit per branch opcode saying whether its operand was
//         moved out (the 9.20 coder: 5 init bytes, post-decision NORMALIZE
//         with an end-of-buffer check that fails the call with SZ_ERROR_DATA;
//         probabilities p[prevByte] for E8, p[256] for E9, p[257] for Jcc)
// -- merged into out[0, outSize).  A converted operand is written back as
// dest - (outPos + 4), little-endian, clipped at outSize.  The result is
// SZ_OK iff exactly outSize bytes came out.
//
// buf0 may lie inside out (7zDec.c:367-372 decodes the main stream into the
// tail of the folder's output): reads of buf0 stay ahead of the writes there.
// The copy between branch opcodes moves eight bytes per step while no byte of
// the step is a branch opcode (exact SWAR zero-byte tests on E8/E9 and on
// 0F-followed-by-8x, the previous byte carried in), and only while the
// distance from the write position to the read position is >= 16, so a wide
// store never lands on main-stream bytes not yet read; everywhere else the
// reference's byte loop runs as written.
#pragma once

#include <stdint.h>

#ifdef LZGPU_HOST_EMU
#ifndef __device__
#define __device__
#define __forceinline__ inline
#endif
#endif

namespace lzgpu {

constexpr int kBcj2Ok = 0, kBcj2ErrData = 1;

// 0x80 in every byte of v that is zero, exactly (no borrow between bytes)
__device__ __forceinline__ uint64_t bcj2_zero_bytes(uint64_t v) {
  const uint64_t m = 0x7F7F7F7F7F7F7F7Full;
  return ~(((v & m) + m) | v | m);
}

// branch opcodes in the eight bytes x (byte k = position k), prev = the byte
// before x[0]: E8/E9 anywhere, or 8x after 0F (IsJ, Bcj2.c:5-6)
__device__ __forceinline__ uint64_t bcj2_branch_mask(uint64_t x, uint32_t prev) {
  const uint64_t e8 = bcj2_zero_bytes((x & 0xFEFEFEFEFEFEFEFEull) ^ 0xE8E8E8E8E8E8E8E8ull);
  const uint64_t shifted = (x << 8) | uint64_t(prev & 0xFFu);
  const uint64_t jcc = bcj2_zero_bytes(shifted ^ 0x0F0F0F0F0F0F0F0Full) &
                       bcj2_zero_bytes((x & 0xF0F0F0F0F0F0F0F0ull) ^ 0x8080808080808080ull);
  return e8 | jcc;
}

__device__ __forceinline__ bool bcj2_is_j(uint32_t b0, uint32_t b1) {
  return (b1 & 0xFEu) == 0xE8u || (b0 == 0x0Fu && (b1 & 0xF0u) == 0x80u);
}

template <class B>
__device__ __forceinline__ uint64_t bcj2_ld64(const B* p) {
  uint64_t v = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) v |= uint64_t(p[k]) << (8 * k);
  return v;
}

template <class B>
__device__ __forceinline__ void bcj2_st64(B* p, uint64_t v) {
#pragma unroll
  for (int k = 0; k < 8; ++k) p[k] = uint8_t(v >> (8 * k));
}
#ifndef LZGPU_HOST_EMU
// global memory runs in unaligned mode: one dwordx2 per eight bytes
typedef __attribute__((address_space(1))) uint8_t bcj2_gbyte;
typedef uint64_t bcj2_u64a1 __attribute__((aligned(1)));
template <>
__device__ __forceinline__ uint64_t bcj2_ld64(const bcj2_gbyte* p) {
  return *(const __attribute__((address_space(1))) bcj2_u64a1*)p;
}
template <>
__device__ __forceinline__ void bcj2_st64(bcj2_gbyte* p, uint64_t v) {
  *(__attribute__((address_space(1))) bcj2_u64a1*)p = v;
}
#endif

// One Bcj2_Decode call.  `prob` points at 258 cells of lane-private storage
// (LDS on the device).  B = the byte type of the global buffers.
template <class B, class P>
__device__ int bcj2_decode(const B* buf0, uint64_t size0, const B* buf1, uint64_t size1,
                           const B* buf2, uint64_t size2, const B* buf3, uint64_t size3,
                           B* out, uint64_t out_size, P prob) {
  for (int i = 0; i < 258; ++i) prob[i] = uint16_t(1024);  // kBitModelTotal >> 1
  uint64_t in_pos = 0, out_pos = 0, rc_pos = 0;
  uint32_t prev = 0;
  // RC_INIT2 (Bcj2.c:12-13): five bytes, each behind RC_TEST
  uint32_t code = 0, range = 0xFFFFFFFFu;
  for (int i = 0; i < 5; ++i) {
    if (rc_pos == size3) return kBcj2ErrData;
    code = (code << 8) | uint32_t(buf3[rc_pos++]);
  }
  if (out_size == 0) return kBcj2Ok;
  // where buf0 sits inside out (if it does): reads of buf0[in_pos] are at
  // out index in_base + in_pos
  const uintptr_t ob = reinterpret_cast<uintptr_t>(out), ib = reinterpret_cast<uintptr_t>(buf0);
  const bool inside = ib >= ob && ib < ob + out_size;
  const uint64_t in_base = inside ? uint64_t(ib - ob) : 0;
  for (;;) {
    uint64_t limit = size0 - in_pos;
    if (out_size - out_pos < limit) limit = out_size - out_pos;
    bool hit = false;
    // eight bytes per step while none is a branch opcode and the write
    // position trails the main-stream read position by >= 16 bytes
    while (limit >= 8 && (!inside || in_base + in_pos >= out_pos + 16)) {
      const uint64_t x = bcj2_ld64(buf0 + in_pos);
      const uint64_t m = bcj2_branch_mask(x, prev);
      if (m != 0) break;
      bcj2_st64(out + out_pos, x);
      out_pos += 8;
      in_pos += 8;
      limit -= 8;
      prev = uint32_t(x >> 56);
    }
    // the reference's copy loop (Bcj2.c:58-68)
    while (limit != 0) {
      const uint32_t b = buf0[in_pos];
      out[out_pos++] = uint8_t(b);
      if (bcj2_is_j(prev, b)) {
        hit = true;
        break;
      }
      in_pos++;
      prev = b;
      limit--;
    }
    if (!hit || out_pos == out_size) break;
    const uint32_t b = buf0[in_pos++];
    const uint32_t pi = b == 0xE8u ? prev : (b == 0xE9u ? 256u : 257u);
    const uint32_t ttt = prob[pi];
    const uint32_t bound = (range >> 11) * ttt;
    bool bit1;
    if (code < bound) {
      range = bound;
      prob[pi] = uint16_t(ttt + ((2048u - ttt) >> 5));
      bit1 = false;
    } else {
      range -= bound;
      code -= bound;
      prob[pi] = uint16_t(ttt - (ttt >> 5));
      bit1 = true;
    }
    if (range < (1u << 24)) {  // NORMALIZE with RC_TEST (Bcj2.c:15)
      if (rc_pos == size3) return kBcj2ErrData;
      range <<= 8;
      code = (code << 8) | uint32_t(buf3[rc_pos++]);
    }
    if (!bit1) {
      prev = b;
      continue;
    }
    const B* v;
    if (b == 0xE8u) {
      if (size1 < 4) return kBcj2ErrData;
      v = buf1;
      buf1 += 4;
      size1 -= 4;
    } else {
      if (size2 < 4) return kBcj2ErrData;
      v = buf2;
      buf2 += 4;
      size2 -= 4;
    }
    const uint32_t dest = ((uint32_t(v[0]) << 24) | (uint32_t(v[1]) << 16) |
                           (uint32_t(v[2]) << 8) | uint32_t(v[3])) -
                          uint32_t(out_pos + 4);
    out[out_pos++] = uint8_t(dest);
    if (out_pos == out_size) break;
    out[out_pos++] = uint8_t(dest >> 8);
    if (out_pos == out_size) break;
    out[out_pos++] = uint8_t(dest >> 16);
    if (out_pos == out_size) break;
    out[out_pos++] = uint8_t(dest >> 24);
    prev = dest >> 24;
  }
  return out_pos == out_size ? kBcj2Ok : kBcj2ErrData;
}

}  // namespace lzgpu

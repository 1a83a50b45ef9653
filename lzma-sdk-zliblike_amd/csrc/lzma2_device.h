// lzma2_device.h -- per-lane LZMA2 chunk walker (Lzma2Dec.c:98-289).
//
// A lane owns one LZMA2 byte range (for config 4: one dictionary-reset block
// found by the host splitter) and decodes it into a flat output window that
// is also its dictionary.  Control bytes, chunk sizes, property bytes, stored
// chunks and the per-chunk range-coder re-initialisation follow the reference
// state machine exactly, so error codes and {destLen, srcLen} match it.
#pragma once

#include "lzma_device.h"

namespace lzgpu {

enum : int {
  C2_CONTROL, C2_UNPACK0, C2_UNPACK1, C2_PACK0, C2_PACK1, C2_PROP, C2_DATA, C2_DATA_CONT,
  C2_FINISHED, C2_ERROR
};

template <class Lo>
struct Lz2StateT {
  LzStateT<Lo> dec;
  uint32_t pack_left, unpack_left;
  int phase;
  uint32_t control;
  uint32_t need_dic_reset, need_state_reset, need_props;
};

__device__ __forceinline__ bool c2_is_copy(uint32_t c) { return (c & 0x80u) == 0; }
__device__ __forceinline__ uint32_t c2_mode(uint32_t c) { return (c >> 5) & 3u; }

template <class Lo>
__device__ inline int lz2_header_byte(Lz2StateT<Lo>& p, uint32_t b) {
  switch (p.phase) {
    case C2_CONTROL:
      p.control = b;
      if (b == 0) return C2_FINISHED;
      if (c2_is_copy(b)) {
        if ((b & 0x7Fu) > 2) return C2_ERROR;
        p.unpack_left = 0;
      } else {
        p.unpack_left = (b & 0x1Fu) << 16;
      }
      return C2_UNPACK0;
    case C2_UNPACK0:
      p.unpack_left |= b << 8;
      return C2_UNPACK1;
    case C2_UNPACK1:
      p.unpack_left |= b;
      p.unpack_left++;
      return c2_is_copy(p.control) ? C2_DATA : C2_PACK0;
    case C2_PACK0:
      p.pack_left = b << 8;
      return C2_PACK1;
    case C2_PACK1:
      p.pack_left |= b;
      p.pack_left++;
      if (c2_mode(p.control) >= 2) return C2_PROP;
      return p.need_props ? C2_ERROR : C2_DATA;
    case C2_PROP: {
      if (b >= 225) return C2_ERROR;
      uint32_t lc = b % 9;
      b /= 9;
      uint32_t pb = b / 5, lp = b % 5;
      if (lc + lp > 4) return C2_ERROR;
      p.dec.lc = lc;
      p.dec.lp = lp;
      p.dec.pb = pb;
      p.need_props = 0;
      return C2_DATA;
    }
  }
  return C2_ERROR;
}

// Lzma2Dec_DecodeToDic for one lane (src in global memory); M = table placement.
template <uint32_t M, class Lo>
__device__ __forceinline__ int lz2_decode_to_dic(Lz2StateT<Lo>& p, uint64_t dic_limit,
                                                 const gbyte* src, uint64_t& src_len, int fin,
                                                 int& status) {
  const uint64_t in_size = src_len;
  src_len = 0;
  status = kStNone;
  while (p.phase != C2_FINISHED) {
    const uint64_t pos0 = p.dec.pos;
    if (p.phase == C2_ERROR) return kErrData;
    if (pos0 == dic_limit && fin == kFinAny) { status = kStNotDone; return kOk; }
    if (p.phase != C2_DATA && p.phase != C2_DATA_CONT) {
      if (src_len == in_size) { status = kStMoreInput; return kOk; }
      src_len++;
      p.phase = lz2_header_byte(p, *src++);
      continue;
    }
    uint64_t out_cur = dic_limit - pos0;
    uint64_t in_cur = in_size - src_len;
    int cur_fin = kFinAny;
    if (p.unpack_left <= out_cur) {
      out_cur = p.unpack_left;
      cur_fin = kFinEnd;
    }
    if (c2_is_copy(p.control)) {
      if (src_len == in_size) { status = kStMoreInput; return kOk; }
      if (p.phase == C2_DATA) {
        const bool reset = (p.control == 1);
        if (reset)
          p.need_props = p.need_state_reset = 1;
        else if (p.need_dic_reset)
          return kErrData;
        p.need_dic_reset = 0;
        lz_init_dic_state(p.dec, reset, false);
      }
      if (in_cur > out_cur) in_cur = out_cur;
      if (in_cur == 0) return kErrData;
      // stored chunk (LzmaDec_UpdateWithUncompressed, Lzma2Dec.c:159-166)
      for (uint64_t i = 0; i < in_cur; ++i) {
        p.dec.dic[p.dec.pos + i] = src[i];
        if constexpr (win_on<M>()) win_put(p.dec.win, src[i]);
      }
      p.dec.pos += in_cur;
      if (p.dec.full == 0 && p.dec.dict_size - p.dec.total <= in_cur)
        p.dec.full = p.dec.dict_size;
      p.dec.total += uint32_t(in_cur);
      src += in_cur;
      src_len += in_cur;
      p.unpack_left -= uint32_t(in_cur);
      p.phase = (p.unpack_left == 0) ? C2_CONTROL : C2_DATA_CONT;
    } else {
      if (p.phase == C2_DATA) {
        const uint32_t mode = c2_mode(p.control);
        const bool init_dic = (mode == 3), init_state = (mode > 0);
        if ((!init_dic && p.need_dic_reset) || (!init_state && p.need_state_reset))
          return kErrData;
        lz_init_dic_state(p.dec, init_dic, init_state);
        p.need_dic_reset = 0;
        p.need_state_reset = 0;
        p.phase = C2_DATA_CONT;
      }
      if (in_cur > p.pack_left) in_cur = p.pack_left;
      // each chunk is one DecodeToDic call over all of its bytes: the
      // tempBuf continuation path is never taken (as in a one-call decode)
      int res = lz_decode_to_dic<false, M>(p.dec, pos0 + out_cur, src, in_cur, cur_fin, status);
      src += in_cur;
      src_len += in_cur;
      p.pack_left -= uint32_t(in_cur);
      const uint64_t produced = p.dec.pos - pos0;
      p.unpack_left -= uint32_t(produced);
      if (res != kOk) return res;
      if (status == kStMoreInput) return res;
      if (in_cur == 0 && produced == 0) {
        if (status != kStMaybeDone || p.unpack_left != 0 || p.pack_left != 0) return kErrData;
        p.phase = C2_CONTROL;
      }
      if (status == kStMaybeDone) status = kStNotDone;
    }
  }
  status = kStDoneMark;
  return kOk;
}

// Lzma2Dec_Init (Lzma2Dec.c:90-97) after Lzma2Dec_AllocateProbs(prop):
// lc = 4, lp = 0, pb = 0 for the allocation; dictionary size from the prop.
// The tables must hold table_cells(4, 0, 4) cells in total (the largest an
// LZMA2 chunk's props can ask for).
template <class Lo>
__device__ __forceinline__ int lz2_init(Lz2StateT<Lo>& p, uint32_t prop, Lo lo, gu16* gl,
                                        gbyte* dic, uint64_t cap) {
  if (prop > 40) return kErrUnsupported;
  uint32_t dict = (prop == 40) ? 0xFFFFFFFFu : ((2u | (prop & 1u)) << (prop / 2 + 11));
  p.dec.lc = 4;
  p.dec.lp = 0;
  p.dec.pb = 0;
  p.dec.dict_size = dict < 4096 ? 4096 : dict;
  p.dec.lo = lo;
  p.dec.gl = gl;
  p.dec.dic = dic;
  p.dec.cap = cap;
  p.dec.pos = 0;
  p.phase = C2_CONTROL;
  p.control = 0;
  p.pack_left = p.unpack_left = 0;
  p.need_dic_reset = p.need_state_reset = p.need_props = 1;
  p.dec.need_state_init = 0;
  p.dec.rep0 = p.dec.rep1 = p.dec.rep2 = p.dec.rep3 = 1;
  p.dec.st = 0;
  p.dec.range = p.dec.code = 0;
  lz_init_dic_state(p.dec, true, true);
  return kOk;
}

}  // namespace lzgpu

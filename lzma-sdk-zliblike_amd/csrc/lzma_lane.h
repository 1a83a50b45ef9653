// lzma_lane.h -- the per-lane work items the kernels run (shared with the
// test-only host emulation build, tests/emu).
//
//   lane_decode   one LzmaDecode (LzmaDec.c:972-1002), or for KIND_LZMA2 one
//                 LZMA2 range over a flat dictionary (Lzma2Dec.c:90-289 as
//                 driven by 7zDec.c:181-202)
//   lane_session  one LzmaDec_DecodeToDic call on a device-resident decoder
//                 state (the dictionary / buffer interfaces)
#pragma once

#include "../../include/lzma_gpu.h"
#include "lzma2_device.h"
#include "lzma_device.h"

// Device-resident decoder state for one DecodeToDic call (the CLzmaDec
// fields of LzmaDec.h:50-69 plus the call's arguments and results).
struct LzgpuSession {
  uint32_t lc, lp, pb, dict_size;
  uint16_t* probs;
  uint8_t* dic;
  const uint8_t* in;
  uint64_t cap, pos, dic_limit, in_len, in_used;
  uint32_t range, code, total, full, st;
  uint32_t rep[4];
  uint32_t pending, need_rc_init, need_state_init, tmp_n;
  int32_t finish_mode, res, status, _pad;
  uint8_t tmp[20];
  uint8_t _pad2[4];
};

namespace lzgpu {

// One batch item with the whole probability table in global memory (the
// generic kernel: any lc/lp/pb, LZMA or LZMA2).  The item's workspace slice
// holds table_cells() cells: lo first, hi behind it.
__device__ __forceinline__ LzmaGpuResult lane_decode(const LzmaGpuStreamDesc& d,
                                                     const uint8_t* __restrict__ src,
                                                     uint8_t* __restrict__ dst,
                                                     uint16_t* __restrict__ ws) {
  LzmaGpuResult r;
  r.status = -1;
  r.dest_len = 0;
  r.src_len = 0;
  if (d.kind == LZMA_GPU_KIND_LZMA2) {
    if (d.probs_off == LZMA_GPU_NO_WORKSPACE) {
      r.res = (d.props[0] > 40) ? kErrUnsupported : kErrMem;
      return r;
    }
    Lz2StateT<gu16*> p;
    gu16* gl = (gu16*)(ws + d.probs_off);
    r.res = lz2_init(p, d.props[0], gl, gl, (gbyte*)(dst + d.dst_off), d.dst_cap);
    if (r.res != kOk) return r;
    uint64_t sl = d.src_len;
    int status = kStNone;
    // the batch contract for an LZMA2 range is Lzma2Dec_DecodeToDic's own
    // result (NEEDS_MORE_INPUT stays SZ_OK); Lzma2Decode maps it to INPUT_EOF
    int res = lz2_decode_to_dic<0u>(p, d.dst_cap, (const gbyte*)(src + d.src_off), sl,
                                    d.finish_mode, status);
    r.res = res;
    r.status = status;
    r.dest_len = p.dec.pos;
    r.src_len = sl;
    return r;
  }
  if (d.src_len < 5) {
    r.res = kErrInputEof;
    return r;
  }
  LzStateT<gu16*> s;
  r.res = lz_props_parse(d.props, d.props_size, s.lc, s.lp, s.pb, s.dict_size);
  if (r.res != kOk) return r;
  if (d.probs_off == LZMA_GPU_NO_WORKSPACE) {
    r.res = kErrMem;
    return r;
  }
  s.gl = (gu16*)(ws + d.probs_off);
  s.lo = s.gl;
  s.dic = (gbyte*)(dst + d.dst_off);
  s.cap = d.dst_cap;
  s.pos = 0;
  s.range = s.code = 0;
  s.st = 0;
  s.rep0 = s.rep1 = s.rep2 = s.rep3 = 1;
  s.need_state_init = 0;
  lz_init_dic_state(s, true, true);
  uint64_t sl = d.src_len;
  int status = kStNone;
  int res = lz_decode_to_dic<false, 0u>(s, d.dst_cap, (const gbyte*)(src + d.src_off), sl,
                                    d.finish_mode, status);
  if (res == kOk && status == kStMoreInput) res = kErrInputEof;
  r.res = res;
  r.status = status;
  r.dest_len = s.pos;
  r.src_len = sl;
  return r;
}

// LDS cells an LZMA2 range needs under placement M: its chunks may carry any
// lc + lp <= 4 (Lzma2Dec.c:148) and pb <= 4.
__host__ __device__ __forceinline__ uint32_t lzma2_lds_cells(uint32_t m) {
  return make_layout(4, 0, 4, m).lds_cells;
}

// One LZMA (or LZMA2) batch item with the LDS-placed sections (LZGPU_LDS_MASK)
// in the lane's LDS slice (lo_cap cells) and the others in its global
// workspace slice.  The planner only routes items here whose LDS part fits.
__device__ __forceinline__ LzmaGpuResult lane_decode_lds(const LzmaGpuStreamDesc& d,
                                                         const uint8_t* __restrict__ src,
                                                         uint8_t* __restrict__ dst,
                                                         uint16_t* __restrict__ ws, lds_u16* lo,
                                                         uint32_t lo_cap) {
  LzmaGpuResult r;
  r.status = -1;
  r.dest_len = 0;
  r.src_len = 0;
  if (d.kind == LZMA_GPU_KIND_LZMA2) {
    // chunks may switch lc/lp/pb (lc + lp <= 4): the slice holds the widest layout
    if (d.probs_off == LZMA_GPU_NO_WORKSPACE || lzma2_lds_cells(LZGPU_LDS_MASK) > lo_cap) {
      r.res = (d.props[0] > 40) ? kErrUnsupported : kErrMem;
      return r;
    }
    Lz2StateT<lds_u16*> p;
    r.res = lz2_init(p, d.props[0], lo, (gu16*)(ws + d.probs_off), (gbyte*)(dst + d.dst_off),
                     d.dst_cap);
    if (r.res != kOk) return r;
    uint64_t sl = d.src_len;
    int status = kStNone;
    r.res = lz2_decode_to_dic<LZGPU_LDS_MASK>(p, d.dst_cap, (const gbyte*)(src + d.src_off), sl,
                                              d.finish_mode, status);
    r.status = status;
    r.dest_len = p.dec.pos;
    r.src_len = sl;
    return r;
  }
  if (d.src_len < 5) {
    r.res = kErrInputEof;
    return r;
  }
  LzStateT<lds_u16*> s;
  r.res = lz_props_parse(d.props, d.props_size, s.lc, s.lp, s.pb, s.dict_size);
  if (r.res != kOk) return r;
  if (d.probs_off == LZMA_GPU_NO_WORKSPACE ||
      make_layout(s.lc, s.lp, s.pb, LZGPU_LDS_MASK).lds_cells > lo_cap) {
    r.res = kErrMem;
    return r;
  }
  s.lo = lo;
  s.gl = (gu16*)(ws + d.probs_off);
  s.dic = (gbyte*)(dst + d.dst_off);
  s.cap = d.dst_cap;
  s.pos = 0;
  s.range = s.code = 0;
  s.st = 0;
  s.rep0 = s.rep1 = s.rep2 = s.rep3 = 1;
  s.need_state_init = 0;
  lz_init_dic_state(s, true, true);
  uint64_t sl = d.src_len;
  int status = kStNone;
  int res = lz_decode_to_dic<false, LZGPU_LDS_MASK>(s, d.dst_cap, (const gbyte*)(src + d.src_off), sl,
                                    d.finish_mode, status);
  if (res == kOk && status == kStMoreInput) res = kErrInputEof;
  r.res = res;
  r.status = status;
  r.dest_len = s.pos;
  r.src_len = sl;
  return r;
}

// One LzmaDec_DecodeToDic call on a device-resident decoder (compact layout,
// all sections in q.probs, for the current lc/lp/pb).
__device__ __forceinline__ void lane_session(LzgpuSession& q) {
  LzStateT<gu16*> s;
  s.lc = q.lc;
  s.lp = q.lp;
  s.pb = q.pb;
  s.dict_size = q.dict_size;
  s.gl = (gu16*)q.probs;
  s.lo = s.gl;
  s.dic = (gbyte*)q.dic;
  s.cap = q.cap;
  s.pos = q.pos;
  s.range = q.range;
  s.code = q.code;
  s.total = q.total;
  s.full = q.full;
  s.st = q.st;
  s.rep0 = q.rep[0];
  s.rep1 = q.rep[1];
  s.rep2 = q.rep[2];
  s.rep3 = q.rep[3];
  s.pending = q.pending;
  s.need_rc_init = q.need_rc_init;
  s.need_state_init = q.need_state_init;
  s.tmp_n = q.tmp_n;
  for (int i = 0; i < int(kLookahead); ++i) s.tmp[i] = q.tmp[i];
  uint64_t sl = q.in_len;
  int status = kStNone;
  int res = lz_decode_to_dic<true, 0u>(s, q.dic_limit, (const gbyte*)q.in, sl, q.finish_mode, status);
  q.pos = s.pos;
  q.range = s.range;
  q.code = s.code;
  q.total = s.total;
  q.full = s.full;
  q.st = s.st;
  q.rep[0] = s.rep0;
  q.rep[1] = s.rep1;
  q.rep[2] = s.rep2;
  q.rep[3] = s.rep3;
  q.pending = s.pending;
  q.need_rc_init = s.need_rc_init;
  q.need_state_init = s.need_state_init;
  q.tmp_n = s.tmp_n;
  for (int i = 0; i < int(kLookahead); ++i) q.tmp[i] = s.tmp[i];
  q.res = res;
  q.status = status;
  q.in_used = sl;
}

}  // namespace lzgpu

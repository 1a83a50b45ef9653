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

// Device-resident decoder state for one DecodeToDic / DecodeToBuf call: the
// public LzmaGpuSession of include/lzma_gpu.h.
typedef LzmaGpuSession LzgpuSession;

namespace lzgpu {

#if LZGPU_PROF && !defined(LZGPU_HOST_EMU)
// per-region cycle sums over lanes (profiling builds only); [24, 24 + W_N):
// the wait attribution of LZGPU_PROF=3
__device__ unsigned long long g_lz_prof[40];
#endif

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
// Under kWinBit (wave-cooperative kernels) `win` is the LDS history window of
// `win_bytes` (a power of two, >= 1024) for this item, empty at its start.
template <uint32_t M = LZGPU_LDS_MASK, bool K2 = true>
__device__ __forceinline__ LzmaGpuResult lane_decode_lds(const LzmaGpuStreamDesc& d,
                                                         const uint8_t* __restrict__ src,
                                                         uint8_t* __restrict__ dst,
                                                         uint16_t* __restrict__ ws, lds_u16* lo,
                                                         uint32_t lo_cap, gu16* gcol = nullptr,
                                                         lds_u8* win = nullptr,
                                                         uint32_t win_bytes = 0) {
  const LzWin w0 = win_make(win, win_bytes, d.dst_cap);
  // global sections: the stream's own workspace slice, or under kIlvBit the
  // lane's column of its group's interleaved slot rows
  auto gtab = [&]() -> gu16* {
    if constexpr ((M & kIlvBit) != 0u)
      return gcol;
    else
      return (gu16*)(ws + d.probs_off);
  };
  LzmaGpuResult r;
  r.status = -1;
  r.dest_len = 0;
  r.src_len = 0;
  if (d.kind == LZMA_GPU_KIND_LZMA2) {
    if constexpr (!K2) {
      // an LZMA2 item in a class the plan marked LZMA-only: a caller-built plan
      r.res = kErrParam;
      return r;
    } else {
    // chunks may switch lc/lp/pb (lc + lp <= 4): the slice holds the widest layout
    if (d.probs_off == LZMA_GPU_NO_WORKSPACE || lzma2_lds_cells(M) > lo_cap) {
      r.res = (d.props[0] > 40) ? kErrUnsupported : kErrMem;
      return r;
    }
    Lz2StateT<lds_u16*> p;
    r.res = lz2_init(p, d.props[0], lo, gtab(), (gbyte*)(dst + d.dst_off),
                     d.dst_cap);
    if (r.res != kOk) return r;
    p.dec.win = w0;
    uint64_t sl = d.src_len;
    int status = kStNone;
#if LZGPU_PROF && !defined(LZGPU_HOST_EMU)
    for (int k = 0; k < 21; ++k) p.dec.prof[k] = 0;
#if LZGPU_PROF == 3
    for (uint32_t k = 0; k < W_N; ++k) p.dec.wprof[k] = 0;
#endif
    const uint64_t t0 = lz_clock();
#endif
    r.res = lz2_decode_to_dic<M>(p, d.dst_cap, (const gbyte*)(src + d.src_off), sl,
                                              d.finish_mode, status);
#if LZGPU_PROF && !defined(LZGPU_HOST_EMU)
    p.dec.prof[3] = lz_clock() - t0;
    p.dec.prof[12] = p.dec.total;
    for (int k = 0; k < 21; ++k) atomicAdd(&g_lz_prof[k], (unsigned long long)p.dec.prof[k]);
#if LZGPU_PROF == 3
    for (uint32_t k = 0; k < W_N; ++k) atomicAdd(&g_lz_prof[24 + k], (unsigned long long)p.dec.wprof[k]);
#endif
    atomicAdd(&g_lz_prof[23], 1ull);
#endif
    r.status = status;
    r.dest_len = p.dec.pos;
    r.src_len = sl;
    return r;
    }
  }
  if (d.src_len < 5) {
    r.res = kErrInputEof;
    return r;
  }
  LzStateT<lds_u16*> s;
  r.res = lz_props_parse(d.props, d.props_size, s.lc, s.lp, s.pb, s.dict_size);
  if (r.res != kOk) return r;
  if (d.probs_off == LZMA_GPU_NO_WORKSPACE ||
      make_layout(s.lc, s.lp, s.pb, M).lds_cells > lo_cap) {
    r.res = kErrMem;
    return r;
  }
  auto start = [&]() {
    s.lo = lo;
    s.gl = gtab();
    s.win = w0;
    s.dic = (gbyte*)(dst + d.dst_off);
    s.cap = d.dst_cap;
    s.pos = 0;
    s.range = s.code = 0;
    s.st = 0;
    s.rep0 = s.rep1 = s.rep2 = s.rep3 = 1;
    s.need_state_init = 0;
    lz_init_dic_state(s, true, true);
  };
  start();
  uint64_t sl = d.src_len;
  int status = kStNone;
#if LZGPU_PROF && !defined(LZGPU_HOST_EMU)
  for (int k = 0; k < 21; ++k) s.prof[k] = 0;
#if LZGPU_PROF == 3
  for (uint32_t k = 0; k < W_N; ++k) s.wprof[k] = 0;
#endif
  const uint64_t t0 = lz_clock();
#endif
  // the fast tail first; a truncated or corrupt end (kRetryExact) again, with
  // the reference's probe on every symbol of the tail (one instantiation of the
  // decoder for both passes)
  bool fast = LZGPU_FAST_TAIL != 0;
  int res;
  for (;;) {
    res = lz_decode_to_dic<false, M>(s, d.dst_cap, (const gbyte*)(src + d.src_off), sl,
                                     d.finish_mode, status, fast);
    if (res != kRetryExact) break;
    fast = false;
    start();
    sl = d.src_len;
    status = kStNone;
  }
#if LZGPU_PROF && !defined(LZGPU_HOST_EMU)
  s.prof[3] = lz_clock() - t0;
  s.prof[12] = s.total;  // literals + match bytes: decoded bytes
  for (int k = 0; k < 21; ++k) atomicAdd(&g_lz_prof[k], (unsigned long long)s.prof[k]);
#if LZGPU_PROF == 3
  for (uint32_t k = 0; k < W_N; ++k) atomicAdd(&g_lz_prof[24 + k], (unsigned long long)s.wprof[k]);
#endif
  atomicAdd(&g_lz_prof[23], 1ull);
#endif
  if (res == kOk && status == kStMoreInput) res = kErrInputEof;
  r.res = res;
  r.status = status;
  r.dest_len = s.pos;
  r.src_len = sl;
  return r;
}

// One LzmaDec_DecodeToDic call (LzmaDec.c:719-838) on a device-resident
// decoder (compact layout, all sections in q.probs, for the current lc/lp/pb).
// M = 0: the table is used in place (lo = gl = q.probs); M = every section in
// LDS | kCoopBit: the cooperative session kernel staged q.probs into `lo` (the
// offsets of placement 0x7FF equal those of the all-global layout).
template <uint32_t M = 0u, class Lo = gu16*>
__device__ __forceinline__ int session_to_dic(LzgpuSession& q, uint64_t dic_limit,
                                              const gbyte* in, uint64_t& in_len, int fin,
                                              int& status, Lo lo = Lo(), LzWin* w = nullptr) {
  LzStateT<Lo> s;
  if constexpr (win_on<M>()) s.win = *w;
  s.lc = q.lc;
  s.lp = q.lp;
  s.pb = q.pb;
  s.dict_size = q.dict_size;
  s.gl = (gu16*)q.probs;
  if constexpr (M == 0u)
    s.lo = s.gl;
  else
    s.lo = lo;
  s.dic = (gbyte*)q.dic;
  s.cap = q.dic_buf_size;
  s.pos = q.dic_pos;
  s.range = q.range;
  s.code = q.code;
  s.total = q.processed_pos;
  s.full = q.check_dic_size;
  s.st = q.state;
  s.rep0 = q.reps[0];
  s.rep1 = q.reps[1];
  s.rep2 = q.reps[2];
  s.rep3 = q.reps[3];
  s.pending = q.remain_len;
  s.need_rc_init = q.need_flush;
  s.need_state_init = q.need_init_state;
  s.tmp_n = q.temp_buf_size;
  for (uint32_t i = 0; i < kLookahead; ++i) s.tmp.set(i, q.temp_buf[i]);
  const int res = lz_decode_to_dic<true, M>(s, dic_limit, in, in_len, fin, status);
  if constexpr (win_on<M>()) *w = s.win;
  q.dic_pos = s.pos;
  q.range = s.range;
  q.code = s.code;
  q.processed_pos = s.total;
  q.check_dic_size = s.full;
  q.state = s.st;
  q.reps[0] = s.rep0;
  q.reps[1] = s.rep1;
  q.reps[2] = s.rep2;
  q.reps[3] = s.rep3;
  q.remain_len = s.pending;
  q.need_flush = s.need_rc_init;
  q.need_init_state = s.need_state_init;
  q.temp_buf_size = s.tmp_n;
  for (uint32_t i = 0; i < kLookahead; ++i) q.temp_buf[i] = uint8_t(s.tmp.get(i));
  return res;
}

// One call on a session: mode 0 = LzmaDec_DecodeToDic(dic_limit), mode 1 =
// LzmaDec_DecodeToBuf (LzmaDec.c:840-878: the dictionary is a ring of
// dic_buf_size bytes; each pass decodes up to the ring end or the caller's
// remaining room, copies the new bytes to `out`, and stops on an error, on a
// pass that produced nothing, or when `out` is full).
// Under the cooperative placement every lane of the wave runs the call, and the
// produced bytes are copied out lane-strided with no barrier: lane i reads
// bytes other lanes of its wave stored (lz_copy_coop gives byte j of a match
// to lane j % 32).  What makes that correct is the wave's in-order memory
// pipeline -- its global stores and later loads to the same address are seen
// in issue order (one vector L1 per CU) -- the same property lz_copy_coop
// relies on when a match reads bytes the wave just wrote.
// kWinBit: `win` (win_bytes) is the call's LDS history window, preloaded here
// with the last bytes of the session's dictionary that a match can reach --
// the bytes written since its last dictionary init (processedPos), or the
// whole ring once it has been filled (checkDicSize) -- by the wave's lanes.
template <uint32_t M = 0u, class Lo = gu16*>
__device__ __forceinline__ void lane_session(LzgpuSession& q, Lo lo = Lo(), lds_u8* win = nullptr,
                                             uint32_t win_bytes = 0) {
  int status = kStNone;
  LzWin w = win_make(win, win_bytes, q.dic_buf_size);
  if constexpr (win_on<M>()) {
    uint64_t hv = q.check_dic_size != 0 ? q.dic_buf_size : q.processed_pos;
    if (hv > q.dic_buf_size) hv = q.dic_buf_size;
    if (hv > win_bytes) hv = win_bytes;
    const gbyte* dic = (const gbyte*)q.dic;
#ifdef LZGPU_HOST_EMU
    const uint32_t l0 = 0, step = 1;
#else
    const uint32_t l0 = threadIdx.x, step = blockDim.x;
#endif
    // window slot i holds the byte at distance hv - i
    for (uint32_t i = l0; i < uint32_t(hv); i += step)
      win[i] = dic[ring_back(q.dic_pos, uint32_t(hv) - i, q.dic_buf_size)];
    w.t = uint32_t(hv);
    w.av = uint32_t(hv);
  }
  if (q.mode != 1) {
    uint64_t sl = q.in_len;
    q.res = session_to_dic<M>(q, q.dic_limit, (const gbyte*)q.in, sl, q.finish_mode, status, lo,
                              &w);
    q.status = status;
    q.in_used = sl;
    return;
  }
  uint64_t out_left = q.out_len, in_left = q.in_len, in_done = 0, out_done = 0;
  const gbyte* in = (const gbyte*)q.in;
  gbyte* out = (gbyte*)q.out;
  int res = kOk;
  for (;;) {
    if (q.dic_pos == q.dic_buf_size) q.dic_pos = 0;
    const uint64_t start = q.dic_pos;
    uint64_t lim;
    int fin;
    if (out_left > q.dic_buf_size - start) {
      lim = q.dic_buf_size;
      fin = kFinAny;
    } else {
      lim = start + out_left;
      fin = q.finish_mode;
    }
    uint64_t in_cur = in_left;
    res = session_to_dic<M>(q, lim, in + in_done, in_cur, fin, status, lo, &w);
    in_done += in_cur;
    in_left -= in_cur;
    const uint64_t produced = q.dic_pos - start;
    const gbyte* from = (const gbyte*)q.dic + start;
#ifndef LZGPU_HOST_EMU
    if constexpr ((M & kCoopBit) != 0u) {
      for (uint64_t i = threadIdx.x; i < produced; i += blockDim.x) out[out_done + i] = from[i];
    } else
#endif
    {
      for (uint64_t i = 0; i < produced; ++i) out[out_done + i] = from[i];
    }
    out_done += produced;
    out_left -= produced;
    if (res != kOk || produced == 0 || out_left == 0) break;
  }
  q.res = res;
  q.status = status;
  q.in_used = in_done;
  q.out_len = out_done;
}

}  // namespace lzgpu

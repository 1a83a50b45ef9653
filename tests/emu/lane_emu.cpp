// lane_emu.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Host build (-DLZGPU_HOST_EMU) of the exact per-lane code the HIP kernels run
// (lzma-sdk-zliblike_amd/csrc/lzma_lane.h), so the CPU test-suite can check the
// kernel logic against the golden vectors before any GPU run.  Not linked into
// the product library; the product has no CPU decode path.
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../lzma-sdk-zliblike_amd/csrc/lzma_lane.h"
#include "../../lzma-sdk-zliblike_amd/csrc/crc32_device.h"
#include "../../lzma-sdk-zliblike_amd/csrc/crc64_device.h"
#include "../../lzma-sdk-zliblike_amd/csrc/bcj_device.h"
#include "../../lzma-sdk-zliblike_amd/csrc/bcj2_device.h"
#include "../../lzma-sdk-zliblike_amd/csrc/bra_device.h"

using namespace lzgpu;

extern "C" {

// Batch: the kernel body applied lane by lane (descs already planned).
void emu_decode_batch(const LzmaGpuStreamDesc* descs, size_t n, const uint8_t* src, uint8_t* dst,
                      uint16_t* ws, LzmaGpuResult* results) {
  for (size_t i = 0; i < n; ++i) results[i] = lane_decode(descs[i], src, dst, ws);
}

#ifndef EMU_WIN_BYTES
#define EMU_WIN_BYTES 4096
#endif

// LDS-variant kernel body: each lane gets a private "LDS" slice of stride cells.
void emu_decode_batch_lds(const LzmaGpuStreamDesc* descs, size_t n, const uint8_t* src,
                          uint8_t* dst, uint16_t* ws, LzmaGpuResult* results, uint32_t stride) {
  uint16_t* slab = (uint16_t*)malloc(size_t(stride) * 2 + 16);
#if defined(EMU_ILV)
  // lane-interleaved global sections: 32 lane columns of the widest LZMA2
  // layout's global rows; stream i runs in column i % 32, its neighbours'
  // cells left as garbage (columns are reused stream after stream)
  // (rows for the widest table the planner puts on an LDS class: lc + lp <= 6
  // with pb 4 -- LZMA2's lc + lp <= 4 fits inside -- as LzmaGpu_PlanBatchEx
  // sizes slot_cells by the widest stream of the class)
  const size_t rows = (make_layout(6, 0, 4, LZGPU_LDS_MASK).glb_cells + 1) & ~size_t(1);
  std::vector<uint16_t> slots(rows * kIlv, 0x5A5A);
#endif
  for (size_t i = 0; i < n; ++i) {
    memset(slab, 0xA5, size_t(stride) * 2);  // LDS is not zeroed between workgroups
#if defined(EMU_ILV)
    results[i] = lane_decode_lds<LZGPU_LDS_MASK | kIlvBit>(descs[i], src, dst, ws, slab, stride,
                                                          slots.data() + (i % kIlv) * kIlvLaneCells);
#elif defined(EMU_COOP_ALL_WIN)
    // ... with the LDS history window (EMU_WIN_BYTES: 4 KiB exercises the
    // dictionary fallback for longer distances and the slot wrap)
    {
      static std::vector<uint8_t> win(EMU_WIN_BYTES);
      memset(win.data(), 0x5C, win.size());  // stale LDS contents
      results[i] = lane_decode_lds<LZGPU_LDS_MASK_ALL | kCoopBit | kWinBit>(
          descs[i], src, dst, ws, slab, stride, nullptr, win.data(), EMU_WIN_BYTES);
    }
#elif defined(EMU_COOP_ALL)
    // the wave-cooperative kernel with every section in LDS (its default
    // placement where the whole table fits)
    results[i] = lane_decode_lds<LZGPU_LDS_MASK_ALL | kCoopBit>(descs[i], src, dst, ws, slab,
                                                                stride);
#elif defined(EMU_COOP)
    // the wave-cooperative kernel's instantiation on the latency placement
    results[i] = lane_decode_lds<LZGPU_LDS_MASK_LAT | kCoopBit>(descs[i], src, dst, ws, slab,
                                                                stride);
#elif defined(EMU_DUP)
    // the one-stream 32-lane kernel's instantiation (latency placement)
    results[i] = lane_decode_lds<LZGPU_LDS_MASK_LAT | kDupBit>(descs[i], src, dst, ws, slab, stride);
#elif defined(EMU_LAT_MASK)
    // the latency-placement instantiation (the kernels' second LDS variant)
    results[i] = lane_decode_lds<LZGPU_LDS_MASK_LAT>(descs[i], src, dst, ws, slab, stride);
#else
    results[i] = lane_decode_lds(descs[i], src, dst, ws, slab, stride);
#endif
  }
  free(slab);
}

// zlib-like DecodeToBuf loop driven through lane_session (the session
// kernel's body), same contract as orc_lzma_stream_decode.  buf_mode 1: each
// DecodeToBuf call is one session call in mode 1 (the device ring loop);
// buf_mode 0: the ring loop runs here over mode-0 (DecodeToDic) calls.
// One session call: lane_session on the session's table in place, or under
// EMU_SESS_COOP_WIN the cooperative session kernel's body -- the table staged
// into an "LDS" copy and back, and the LDS history window preloaded per call.
static void run_session(LzgpuSession& q) {
#if defined(EMU_SESS_COOP_WIN)
  const uint32_t cells = table_cells(q.lc, q.lp, q.pb);
  std::vector<uint16_t> lo(cells + 8);
  memcpy(lo.data(), q.probs, size_t(cells) * 2);
  static std::vector<uint8_t> win(EMU_WIN_BYTES);
  memset(win.data(), 0x5C, win.size());
  lane_session<LZGPU_LDS_MASK_ALL | kCoopBit | kWinBit>(q, lo.data(), win.data(), EMU_WIN_BYTES);
  memcpy((void*)q.probs, lo.data(), size_t(cells) * 2);
#else
  lane_session(q);
#endif
}

static int stream_decode(const uint8_t* props, const uint8_t* src, size_t src_total, uint8_t* out,
                         size_t out_total, size_t in_chunk, size_t out_chunk, int finish_mode,
                         long long* trace, int max_calls, size_t* out_len, size_t* in_used,
                         int buf_mode) {
  uint32_t lc, lp, pb, dict;
  int r = lz_props_parse(props, 5, lc, lp, pb, dict);
  if (r != kOk) { *out_len = 0; *in_used = 0; return -r; }
  LzgpuSession q;
  memset(&q, 0, sizeof q);
  q.lc = lc; q.lp = lp; q.pb = pb; q.dict_size = dict;
  q.probs = (uint16_t*)malloc(size_t(num_probs(lc, lp)) * 2);
  q.dic = (uint8_t*)malloc(dict);
  q.dic_buf_size = dict;
  q.dic_pos = 0;
  q.need_flush = 1; q.need_init_state = 1; q.remain_len = 0; q.temp_buf_size = 0;
  size_t in_pos = 0, out_pos = 0;
  int calls = 0;
  while (calls < max_calls) {
    size_t sl = src_total - in_pos, dl = out_total - out_pos;
    if (sl > in_chunk) sl = in_chunk;
    if (dl > out_chunk) dl = out_chunk;
    size_t got_in = 0, got_out = 0;
    int res = 0, st = -1;
    if (buf_mode) {
      q.mode = 1;
      q.in = src + in_pos; q.in_len = sl; q.out = out + out_pos; q.out_len = dl;
      q.finish_mode = finish_mode;
      run_session(q);
      res = q.res; st = q.status; got_in = q.in_used; got_out = q.out_len;
    } else {
      // ---- LzmaDec_DecodeToBuf (LzmaDec.c:840-878) over mode-0 calls
      size_t out_left = dl, in_left = sl;
      const uint8_t* s = src + in_pos;
      uint8_t* d = out + out_pos;
      q.mode = 0;
      for (;;) {
        if (q.dic_pos == q.dic_buf_size) q.dic_pos = 0;
        uint64_t start = q.dic_pos, lim;
        int fin;
        if (out_left > q.dic_buf_size - start) { lim = q.dic_buf_size; fin = 0; }
        else { lim = start + out_left; fin = finish_mode; }
        q.in = s; q.in_len = in_left; q.dic_limit = lim; q.finish_mode = fin;
        run_session(q);
        res = q.res; st = q.status;
        s += q.in_used; in_left -= q.in_used; got_in += q.in_used;
        size_t produced = q.dic_pos - start;
        memcpy(d, q.dic + start, produced);
        d += produced; out_left -= produced; got_out += produced;
        if (res != 0) break;
        if (produced == 0 || out_left == 0) break;
      }
    }
    trace[4 * calls + 0] = res;
    trace[4 * calls + 1] = st;
    trace[4 * calls + 2] = (long long)got_in;
    trace[4 * calls + 3] = (long long)got_out;
    calls++;
    in_pos += got_in;
    out_pos += got_out;
    if (res != 0 || st == 1 || out_pos == out_total || (got_in == 0 && got_out == 0)) break;
  }
  free(q.probs);
  free(q.dic);
  *out_len = out_pos;
  *in_used = in_pos;
  return calls;
}

int emu_stream_decode(const uint8_t* props, const uint8_t* src, size_t src_total, uint8_t* out,
                      size_t out_total, size_t in_chunk, size_t out_chunk, int finish_mode,
                      long long* trace, int max_calls, size_t* out_len, size_t* in_used) {
  return stream_decode(props, src, src_total, out, out_total, in_chunk, out_chunk, finish_mode,
                       trace, max_calls, out_len, in_used, 1);
}

int emu_stream_decode_dic(const uint8_t* props, const uint8_t* src, size_t src_total,
                          uint8_t* out, size_t out_total, size_t in_chunk, size_t out_chunk,
                          int finish_mode, long long* trace, int max_calls, size_t* out_len,
                          size_t* in_used) {
  return stream_decode(props, src, src_total, out, out_total, in_chunk, out_chunk, finish_mode,
                       trace, max_calls, out_len, in_used, 0);
}

// CRC-32 kernels' per-lane code (crc_chunk per chunk slot, then crc_fold),
// range by range.  The blocks read may extend up to 15 bytes either side of a
// range (aligned 16-byte loads): callers pad their buffers.
void emu_crc_ranges(const uint8_t* data, const uint64_t* off, const uint64_t* len, size_t n,
                    uint32_t init, uint32_t xorout, uint32_t* out) {
  static const CrcTables T = crc_make_tables();
  for (size_t i = 0; i < n; ++i) {
    const uint64_t nch = (len[i] + kCrcChunk - 1) / kCrcChunk;
    std::vector<uint32_t> c(nch + 1);
    for (uint64_t j = 0; j < nch; ++j)
      crc_chunk(&T.slice[0][0], data + off[i], len[i], uint32_t(j), init, &c[j]);
    out[i] = crc_fold(&T.shift[0][0], c.data(), len[i], init) ^ xorout;
  }
}

// CRC-64 kernels' per-lane code (crc64_chunk per chunk slot, then crc64_fold).
void emu_crc64_ranges(const uint8_t* data, const uint64_t* off, const uint64_t* len, size_t n,
                      uint64_t init, uint64_t xorout, uint64_t* out) {
  static const Crc64Tables T = crc64_make_tables();
  for (size_t i = 0; i < n; ++i) {
    const uint64_t nch = (len[i] + kCrc64Chunk - 1) / kCrc64Chunk;
    std::vector<uint64_t> c(nch + 1);
    for (uint64_t j = 0; j < nch; ++j)
      crc64_chunk(&T.slice[0][0], data + off[i], len[i], uint32_t(j), init, &c[j]);
    out[i] = crc64_fold(&T.shift[0][0], c.data(), len[i], init) ^ xorout;
  }
}

// The x86 BCJ kernel's per-lane code (bcj_x86) on one buffer.  The window
// loads aligned 16-byte blocks holding a valid byte: callers pad buffers.
uint64_t emu_bcj_x86(uint8_t* data, uint64_t size, uint32_t ip, uint32_t* state, int encoding) {
  return bcj_x86(data, size, ip, state, encoding);
}

// lzgpu_bcj_x86_tile_kernel on one range, its phases run in order on the host:
// per 4 KiB tile, the records of every E8/E9 below size - 4 (position and the
// four bytes behind it, read after the previous tile's conversions), then the
// reference's decisions over them (bcj_hit) writing the conversions.
uint64_t emu_bcj_x86_tiled(uint8_t* data, uint64_t size, uint32_t ip, uint32_t* state,
                           int encoding) {
  if (size < 5) return 0;
  const uint64_t limit = size - 4;
  BcjRun run;
  run.resume = 0;
  run.prev_pos = ~uint64_t(0);
  run.mask = *state & 7u;
  std::vector<uint64_t> pos;
  std::vector<uint32_t> op;
  for (uint64_t tb = 0; tb < limit; tb += 4096) {
    uint8_t tile[4096 + 4];
    for (uint64_t k = 0; k < 4096 + 4; ++k) tile[k] = tb + k < size ? data[tb + k] : 0;
    pos.clear();
    op.clear();
    for (uint64_t k = 0; k < 4096 && tb + k < limit; ++k)
      if ((tile[k] & 0xFEu) == 0xE8u) {
        pos.push_back(tb + k);
        op.push_back(uint32_t(tile[k + 1]) | (uint32_t(tile[k + 2]) << 8) |
                     (uint32_t(tile[k + 3]) << 16) | (uint32_t(tile[k + 4]) << 24));
      }
    for (size_t i = 0; i < pos.size(); ++i) {
      if (pos[i] < run.resume) continue;
      uint32_t v;
      if (bcj_hit(run, pos[i], op[i], ip + 5, encoding, &v)) memcpy(data + pos[i] + 1, &v, 4);
    }
  }
  return bcj_finish(run, limit, state);
}

// lzgpu_bcj2_kernel's lane (bcj2_decode) on host buffers; probabilities in a
// lane-private array as the kernel's LDS slice.
int emu_bcj2(const uint8_t* b0, uint64_t s0, const uint8_t* b1, uint64_t s1, const uint8_t* b2,
             uint64_t s2, const uint8_t* b3, uint64_t s3, uint8_t* out, uint64_t out_size) {
  uint16_t probs[258];
  return bcj2_decode(b0, s0, b1, s1, b2, s2, b3, s3, out, out_size, probs);
}

// The branch-converter kernels' code on one buffer, unit by unit in lane
// order (lzgpu_bra_unit_kernel / lzgpu_bra_armt_kernel).
uint64_t emu_bra(uint32_t kind, uint8_t* data, uint64_t size, uint32_t ip, int encoding) {
  if (kind == 0x108) return bra_armt(data, size, ip, encoding);  // the serial statement
  const uint32_t u = bra_unit(kind);
  const uint64_t units = bra_done_units(kind, size);
  const uint64_t done = kind == kBraARMT ? bra_armt_done(data, units) : units * u;
  const bool words = u == 4 && ((uintptr_t)data & 3) == 0;  // the kernel's aligned path
  for (uint64_t k = 0; k < units; ++k) {
    if (words)
      bra_word_aligned(kind, data + k * u, ip + uint32_t(k * u), encoding);
    else
      bra_unit_convert(kind, data + k * u, ip + uint32_t(k * u), encoding);
  }
  return done;
}

// lzgpu_delta_kernel's lanes for one range: read all state bytes, run the residues, rewrite state.
void emu_delta(uint8_t* state, uint32_t delta, uint8_t* data, uint64_t size, int encoding) {
  uint8_t st[256], sums[256];
  for (uint32_t t = 0; t < delta; ++t) st[t] = state[t];
  if (encoding) {
    for (uint32_t t = 0; t < delta; ++t)
      state[delta_state_slot(size, delta, t)] = delta_residue(data, size, delta, t, st[t], 1);
    return;
  }
  if (delta <= 16 && (delta & (delta - 1)) == 0) {  // lzgpu_delta_kernel's tile scan
    const uint32_t d = delta;
    uint64_t h = (16 - ((uintptr_t)data & 15)) & 15;
    if (h > size) h = size;
    uint8_t last[16];
    for (uint32_t q = 0; q < d; ++q) last[q] = st[q];
    for (uint64_t q = 0; q < h; ++q) {
      last[q % d] = uint8_t(last[q % d] + data[q]);
      data[q] = last[q % d];
    }
    V16 C{0, 0};
    for (uint32_t j = 0; j < 16; ++j) {
      const uint64_t b = last[(h + j) % d];
      if (j < 8) C.lo |= b << (8 * j); else C.hi |= b << (8 * (j - 8));
    }
    for (uint64_t base = h; base < size; base += 4096) {
      V16 pre[256], incl[256];
      for (uint32_t t = 0; t < 256; ++t) {
        const uint64_t pos = base + 16 * uint64_t(t);
        V16 x{0, 0};
        for (uint64_t q = pos; q < size && q < pos + 16; ++q) {
          const uint32_t j = uint32_t(q - pos);
          if (j < 8) x.lo |= uint64_t(data[q]) << (8 * j); else x.hi |= uint64_t(data[q]) << (8 * (j - 8));
        }
        pre[t] = delta_lane_prefix(x, d);
        const V16 tot = delta_lane_total(pre[t], d);
        incl[t] = t ? vadd8(incl[t - 1], tot) : tot;
      }
      for (uint32_t t = 0; t < 256; ++t) {
        const uint64_t pos = base + 16 * uint64_t(t);
        const V16 o = vadd8(vadd8(pre[t], t ? incl[t - 1] : V16{0, 0}), C);
        for (uint64_t q = pos; q < size && q < pos + 16; ++q) {
          const uint32_t j = uint32_t(q - pos);
          data[q] = uint8_t(j < 8 ? o.lo >> (8 * j) : o.hi >> (8 * (j - 8)));
        }
      }
      C = vadd8(C, incl[255]);
    }
    for (uint32_t t = 0; t < d; ++t) {
      const uint32_t j = uint32_t((t + d - h % d) % d);
      state[delta_state_slot(size, d, t)] = uint8_t(j < 8 ? C.lo >> (8 * j) : C.hi >> (8 * (j - 8)));
    }
    return;
  }
  DeltaSeg sg[256];
  bool on[256];
  for (uint32_t t = 0; t < 256; ++t) {
    on[t] = delta_seg(size, delta, t, &sg[t]);
    if (on[t]) sums[t] = delta_seg_sum(data, delta, sg[t]);
  }
  for (uint32_t t = 0; t < 256; ++t) {
    if (!on[t]) continue;
    uint32_t carry = st[sg[t].r];
    for (uint32_t g = 0; g < sg[t].g; ++g) carry += sums[sg[t].r + g * delta];
    const uint8_t last = delta_seg_apply(data, delta, sg[t], uint8_t(carry));
    const uint64_t mr = sg[t].r < size ? (size - 1 - sg[t].r) / delta + 1 : 0;
    if ((mr > 0 && sg[t].m0 < mr && sg[t].m1 == mr) || (mr == 0 && sg[t].g == 0))
      state[delta_state_slot(size, delta, sg[t].r)] = last;
  }
}

}  // extern "C"

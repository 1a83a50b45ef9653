// sliced.hip -- time-sliced batch decoding (second half):
// a batch of LZMA streams advanced in rounds of at most `slice` output bytes
// per stream, each stream's CLzmaDec state (LzmaDec.h:50-69) spilled to an
// LzmaGpuSession in the workspace between rounds.  One round = one launch of a
// persistent grid that pulls the round's unfinished streams from a list and
// appends those still unfinished to the next round's list, so no host round
// trip is needed between rounds and every round re-deals the survivors over
// all CUs.
//
// A stream's calls are exactly the reference's streaming contract:
// LzmaDec_DecodeToDic(dicLimit = dicPos + slice, LZMA_FINISH_ANY), and on the
// call whose limit is dst_cap the stream's own finish mode (LzmaDec.c:719-838,
// the loop 7zDec.c:133-171 / LzmaDecode LzmaDec.c:972-1002 reduce to); the
// final state maps to LzmaDecode's result as lane_decode does.
//
// Streams fall in two classes: those whose staged sections fit the LDS
// kernel's slot (class 0: the lane or cooperative kernel) and those decoded in
// place on their spilled table (class 1: the global kernel -- tables over
// 64 KiB, or every stream when the plan says GLOBAL); each round launches the
// class-0 kernel and, if the plan has class-1 streams, the global kernel.
//
// Workspace (LzmaGpu_PlanSliced): [sessions: n x 192 B][tables: per stream,
// at descs[i].probs_off cells][lists: class c, parity b at (2c + b) n u32]
// [counters: class c at c (2R + 2): per round r, [2r] = streams entering
// round r, [2r + 1] = round r's queue].

#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "lzma_gpu_internal.h"

using namespace lzgpu;
using lzgpu_host::ensure_device;
using lzgpu_host::hip_ok;
using lzgpu_host::set_error;

namespace {

struct SlicedRound {
  LzgpuSession* sess;
  LzmaGpuResult* results;
  const uint32_t* list_in;
  uint32_t* list_out;
  const uint32_t* cnt_in;
  uint32_t* queue;
  uint32_t* cnt_out;
  uint64_t slice;
  uint32_t lds_words;  // the staged slot's 32-bit words (a flag word follows it)
};

constexpr int32_t kSlicedDone = -1;  // LzgpuSession.mode of a stream finished at init

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lds_v4;
typedef __attribute__((address_space(1))) u32x4 glb_v4;

// table cells rounded to whole 16-byte vectors (the workspace slots are)
__host__ __device__ __forceinline__ uint32_t sliced_vec(uint32_t cells) { return (cells + 7u) / 8u; }

}  // namespace

// Placements of the LDS kernels: the whole table in LDS (the cooperative
// kernel; the lane kernel for narrow tables), or the latency kernel's
// sections (0x1BF: all but SpecPos, the matched-literal trees and LenHigh)
// staged while the others stay in place in the spilled table (kSessHybBit) --
// 5.2 KB instead of 14.6 KB per lc3 stream, so 16 streams per CU fit as in the
// one-shot latency kernel.
constexpr uint32_t kSlicedAll = LZGPU_LDS_MASK_ALL;
constexpr uint32_t kSlicedHyb = LZGPU_LDS_MASK_LAT | kSessHybBit;

namespace {

// LDS cells a stream's staged sections take under placement mask m
__host__ __device__ __forceinline__ uint32_t staged_cells(uint32_t m, uint32_t lc, uint32_t lp,
                                                          uint32_t pb) {
  return m == kSlicedAll ? sliced_vec(table_cells(lc, lp, pb)) * 8u
                         : make_layout(lc, lp, pb, m).lds_cells;
}

// LzmaDec_Init on a bound session (LzmaDec.c:685-705 via LzmaDec_InitDicAndState)
__device__ __forceinline__ void sliced_reset(LzgpuSession& q) {
  q.dic_pos = 0;
  q.in_used = 0;  // consumed so far (cumulative over rounds)
  q.range = q.code = 0;
  q.processed_pos = q.check_dic_size = 0;
  q.state = 0;
  q.reps[0] = q.reps[1] = q.reps[2] = q.reps[3] = 1;
  q.remain_len = 0;
  q.need_flush = 1;       // range coder init pending
  q.need_init_state = 1;  // probabilities initialised by the first call
  q.temp_buf_size = 0;
}

}  // namespace

// Per stream: the initial decoder (LzmaDec_Allocate + LzmaDec_Init,
// LzmaDec.c:950-970, 685-705) spilled to its session and the stream entered in
// its class's round-0 list, or -- for the failures LzmaDecode reports before
// decoding (LzmaDec.c:980-990) -- its final result.
__global__ void __launch_bounds__(256) lzgpu_sliced_init_kernel(
    const LzmaGpuStreamDesc* __restrict__ descs, const uint32_t* __restrict__ order, uint32_t n,
    const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint16_t* __restrict__ ws,
    LzgpuSession* __restrict__ sess, LzmaGpuResult* __restrict__ results,
    uint32_t* __restrict__ lists, uint32_t* __restrict__ ctr, uint32_t ctr_stride,
    uint32_t lds_cells, uint32_t lds_mask) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint32_t i = order ? order[k] : k;
  const LzmaGpuStreamDesc d = descs[i];
  LzgpuSession q = {};
  q.mode = 0;
  LzmaGpuResult r;
  r.res = kOk;
  r.status = -1;
  r.dest_len = 0;
  r.src_len = 0;
  if (d.kind != LZMA_GPU_KIND_LZMA) {
    r.res = kErrParam;
  } else if (d.src_len < 5) {
    r.res = kErrInputEof;
  } else {
    r.res = lz_props_parse(d.props, d.props_size, q.lc, q.lp, q.pb, q.dict_size);
    if (r.res == kOk && d.probs_off == LZMA_GPU_NO_WORKSPACE) r.res = kErrMem;
  }
  if (r.res != kOk) {
    q.mode = kSlicedDone;
    results[i] = r;
    sess[i] = q;
    return;
  }
  q.probs = ws + d.probs_off;
  q.dic = dst + d.dst_off;
  q.in = src + d.src_off;
  q.dic_buf_size = d.dst_cap;
  q.in_len = d.src_len;
  sliced_reset(q);
  q.finish_mode = d.finish_mode;
  sess[i] = q;
  const uint32_t c = staged_cells(lds_mask, q.lc, q.lp, q.pb) > lds_cells ? 1u : 0u;
  lists[size_t(2 * c) * n + atomicAdd(ctr + size_t(c) * ctr_stride, 1u)] = i;
}

namespace {

// One round's call on one stream; true when the stream is finished (its
// LzmaGpuResult in r).  The call is LzmaDec_DecodeToDic(dicLimit = dicPos +
// slice, LZMA_FINISH_ANY), or with the stream's finish mode once the limit is
// dst_cap.
template <uint32_t M, class Lo>
__device__ __forceinline__ bool sliced_step(LzgpuSession& q, uint64_t slice, Lo lo,
                                            LzmaGpuResult& r) {
  const uint64_t cap = q.dic_buf_size;
  uint64_t lim = (cap - q.dic_pos > slice) ? q.dic_pos + slice : cap;
  int res, st;
  for (int pass = 0;; ++pass) {
    const int fin = lim == cap ? q.finish_mode : int(kFinAny);
    uint64_t used = q.in_len - q.in_used;
    st = kStNone;
    res = session_to_dic<M>(q, lim, (const gbyte*)(q.in + q.in_used), used, fin, st, lo);
    q.in_used += used;
    if (res != kErrData || pass != 0) break;
    // The reference reports a data error with the state of the DecodeReal /
    // DecodeReal2 call it happened in rolled back (LzmaDec.c:797, 826: locals
    // not written back), so destLen / srcLen name that call's start, and a
    // round's call boundaries are starts a one-call LzmaDecode does not have.
    // A corrupt stream is decoded again from its start as that one call, whose
    // result is LzmaDecode's (once per corrupt stream; other streams' rounds
    // stay bounded).
    sliced_reset(q);
    lim = cap;
  }
  const bool done = res != kOk || st == kStDoneMark || st == kStMoreInput || lim == cap;
  if (done) {
    r.res = (res == kOk && st == kStMoreInput) ? int(kErrInputEof) : res;
    r.status = st;
    r.dest_len = q.dic_pos;
    r.src_len = q.in_used;
  }
  return done;
}

__device__ __forceinline__ void sliced_finish(const SlicedRound& a, uint32_t i,
                                              const LzgpuSession& q, bool done,
                                              const LzmaGpuResult& r) {
  a.sess[i] = q;
  if (done)
    a.results[i] = r;
  else
    a.list_out[atomicAdd(a.cnt_out, 1u)] = i;
}

// copy the staged sections between the spilled table (whole-table offsets)
// and LDS (packed), all lanes of the workgroup
template <uint32_t M>
__device__ __forceinline__ void stage(lds_u16* lo, gu16* gp, uint32_t lc, uint32_t lp, uint32_t pb,
                                      bool in) {
  if constexpr ((M & ~kCoopBit) == kSlicedAll) {
    const uint32_t nv = sliced_vec(table_cells(lc, lp, pb));
    glb_v4* g = (glb_v4*)gp;
    lds_v4* l = (lds_v4*)lo;
    for (uint32_t j = threadIdx.x; j < nv; j += blockDim.x) {
      if (in)
        l[j] = g[j];
      else
        g[j] = l[j];
    }
  } else {
    const Layout L = make_layout(lc, lp, pb, M);
    const Layout F = make_layout(lc, lp, pb, 0u);
    for (uint32_t k = 0; k < S_NSEC; ++k) {
      if (!((M >> k) & 1u)) continue;
      const uint32_t n = sec_cells(k, lc, lp, pb);
      for (uint32_t j = threadIdx.x; j < n; j += blockDim.x) {
        if (in)
          lo[L.o[k] + j] = gp[F.o[k] + j];
        else
          gp[F.o[k] + j] = lo[L.o[k] + j];
      }
    }
  }
}

// next list entry for the workgroup (lane 0 takes it, the wave shares it)
__device__ __forceinline__ uint32_t next_entry(const SlicedRound& a) {
  uint32_t k = 0;
  if (threadIdx.x == 0) k = atomicAdd(a.queue, 1u);
  return uint32_t(__builtin_amdgcn_readfirstlane(int(k)));
}

}  // namespace

// Class 0, one stream per workgroup of one wave: the 64 lanes stage the
// stream's sections of placement M into LDS, lane 0 makes the call (the
// per-byte-checked reader of the one-lane kernels), the lanes write them back
// if the stream goes on.  W = register budget (waves per SIMD).
constexpr uint32_t kSlicedDup = 32;
template <int W, uint32_t M>
__global__ void __launch_bounds__(64, W) lzgpu_sliced_lane_kernel(SlicedRound a) {
  extern __shared__ uint32_t lz_smem[];
  lds_u16* lo = (lds_u16*)((uint16_t*)lz_smem);
  uint32_t& s_done = lz_smem[a.lds_words];
  const uint32_t n = *a.cnt_in;
  for (uint32_t k = next_entry(a); k < n; k = next_entry(a)) {
    const uint32_t i = a.list_in[k];
    LzgpuSession* qp = a.sess + i;
    const uint32_t lc = qp->lc, lp = qp->lp, pb = qp->pb;
    gu16* gp = (gu16*)qp->probs;
    if (!qp->need_init_state) stage<M>(lo, gp, lc, lp, pb, true);
    __syncthreads();
    if (threadIdx.x < kSlicedDup) {
      // the first wave's kSlicedDup lanes all decode the stream (identical
      // state, identical stores; lane 0 records the outcome): a wave with
      // >= 16 lanes in EXEC issues ~1.4-3x faster than a one-lane wave
      // (round 5, lzma_kernels.hip lzgpu_decode_dup_kernel)
      LzgpuSession q = *qp;
      const uint32_t z = lz_vzero();  // keep the shared state in vector registers
      q.in = (const uint8_t*)q.in + z;
      q.dic = (uint8_t*)q.dic + z;
      LzmaGpuResult r;
      const bool done = sliced_step<M>(q, a.slice, lo, r);
      if (threadIdx.x == 0) {
        sliced_finish(a, i, q, done, r);
        s_done = done ? 1u : 0u;
      }
    }
    __syncthreads();
    if (!s_done) stage<M>(lo, gp, lc, lp, pb, false);
    __syncthreads();
  }
}

// Class 0, one stream per 32-lane wave, every lane holding its state: the
// cooperative decoder on the whole table
// staged in LDS.
constexpr uint32_t kSlicedCoopMask = kSlicedAll | kCoopBit;
template <int W>
__global__ void __launch_bounds__(32, W) lzgpu_sliced_coop_kernel(SlicedRound a) {
  extern __shared__ uint32_t lz_smem[];
  lds_u16* lo = (lds_u16*)((uint16_t*)lz_smem);
  const uint32_t n = *a.cnt_in;
  for (uint32_t k = next_entry(a); k < n; k = next_entry(a)) {
    const uint32_t i = a.list_in[k];
    LzgpuSession q = a.sess[i];
    gu16* gp = (gu16*)q.probs;
    if (!q.need_init_state) stage<kSlicedCoopMask>(lo, gp, q.lc, q.lp, q.pb, true);
    __syncthreads();
    LzmaGpuResult r;
    const bool done = sliced_step<kSlicedCoopMask>(q, a.slice, lo, r);
    __syncthreads();
    if (!done) stage<kSlicedCoopMask>(lo, gp, q.lc, q.lp, q.pb, false);
    if (threadIdx.x == 0) sliced_finish(a, i, q, done, r);
    __syncthreads();
  }
}

// Class 1, one stream per lane, its table used in place in the workspace.
__global__ void __launch_bounds__(64) lzgpu_sliced_global_kernel(SlicedRound a) {
  const uint32_t n = *a.cnt_in;
  for (;;) {
    const uint32_t k = atomicAdd(a.queue, 1u);
    if (k >= n) break;
    const uint32_t i = a.list_in[k];
    LzgpuSession q = a.sess[i];
    LzmaGpuResult r;
    const bool done = sliced_step<0u>(q, a.slice, (gu16*)q.probs, r);
    sliced_finish(a, i, q, done, r);
  }
}

namespace {

// largest slot the LDS kernels stage (64 KiB, as the cooperative session kernel)
constexpr uint32_t kSlicedMaxLdsCells = kSessCoopMaxCells;

size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// workgroups of `cells` staged cells (+ the lane kernel's flag word) per CU, <= 16
uint32_t lds_fit(uint32_t cells) {
  return std::min<uint32_t>(16, lzgpu_host::lds_groups_fit(size_t(cells) * 2 + 16));
}

SRes plan_sliced(LzmaGpuStreamDesc* descs, size_t n, uint64_t slice, unsigned kernel,
                 uint32_t* order, LzmaGpuSlicedPlan* p) {
  if (!p) return SZ_ERROR_PARAM;
  *p = LzmaGpuSlicedPlan{};
  if (slice == 0 || kernel > LZMA_GPU_SLICED_GLOBAL || n > 0x7FFFFFFFu) return SZ_ERROR_PARAM;
  p->n = n;
  p->slice_bytes = slice;
  // per stream: its own table slot (16-byte aligned); a stream whose props do
  // not parse gets none (it finishes at init, as LzmaDecode's props check)
  uint64_t cells_total = 0, max_cap = 0;
  // widest staged size (<= kSlicedMaxLdsCells) under either placement
  uint32_t max_all = 0, max_hyb = 0;
  std::vector<uint64_t> work(n);
  std::vector<uint8_t> lcs(n, 0xFF), lps(n), pbs(n);
  for (size_t i = 0; i < n; ++i) {
    LzmaGpuStreamDesc& d = descs[i];
    if (d.kind != LZMA_GPU_KIND_LZMA) return SZ_ERROR_PARAM;
    uint32_t lc, lp, pb, dict;
    if (d.src_len >= 5 && lz_props_parse(d.props, d.props_size, lc, lp, pb, dict) == kOk) {
      d.probs_off = cells_total;
      cells_total += sliced_vec(table_cells(lc, lp, pb)) * 8u;
      const uint32_t a = staged_cells(kSlicedAll, lc, lp, pb);
      const uint32_t h = staged_cells(kSlicedHyb, lc, lp, pb);
      if (a <= kSlicedMaxLdsCells) max_all = std::max(max_all, a);
      if (h <= kSlicedMaxLdsCells) max_hyb = std::max(max_hyb, h);
      lcs[i] = uint8_t(lc);
      lps[i] = uint8_t(lp);
      pbs[i] = uint8_t(pb);
    } else {
      d.probs_off = LZMA_GPU_NO_WORKSPACE;
    }
    max_cap = std::max<uint64_t>(max_cap, d.dst_cap);
    work[i] = 24 * d.src_len + d.dst_cap;
  }
  const uint64_t rounds = max_cap == 0 ? 1 : (max_cap + slice - 1) / slice;
  if (rounds > (1u << 24)) return SZ_ERROR_PARAM;
  p->rounds = uint32_t(rounds);
  if (order) {
    for (size_t i = 0; i < n; ++i) order[i] = uint32_t(i);
    std::stable_sort(order, order + n, [&](uint32_t a, uint32_t b) { return work[a] > work[b]; });
  }
  const uint32_t cus = lzgpu_host::device_cus();
  const uint64_t per_cu = (n + cus - 1) / std::max<uint32_t>(cus, 1);
  if (kernel == LZMA_GPU_SLICED_AUTO) {
    if (max_all == 0 && max_hyb == 0)
      kernel = LZMA_GPU_SLICED_GLOBAL;  // nothing to stage
    else
      kernel = per_cu <= 8 ? LZMA_GPU_SLICED_COOP : LZMA_GPU_SLICED_LANE;
  }
  p->kernel = kernel;
  p->lds_mask = kSlicedAll;
  p->table_cells = max_all;
  if (kernel == LZMA_GPU_SLICED_LANE) {
    p->groups_per_cu = std::max<uint32_t>(1, lds_fit(max_all));
    if (max_hyb && lds_fit(max_hyb) > lds_fit(max_all)) {
      // more resident streams with only the latency sections staged
      p->lds_mask = kSlicedHyb;
      p->table_cells = max_hyb;
      p->groups_per_cu = lds_fit(max_hyb);
    }
  } else if (kernel == LZMA_GPU_SLICED_COOP) {
    // one 32-lane wave per SIMD at most: the cooperative decoder is issue-bound
    p->groups_per_cu = std::max<uint32_t>(
        1, std::min<uint32_t>(std::min<uint32_t>(lds_fit(max_all), 8),
                              uint32_t(std::max<uint64_t>(per_cu, 1))));
  } else {
    p->table_cells = 0;      // every stream in place
    p->groups_per_cu = 16;   // 64-lane workgroups, one stream per lane
  }
  p->max_groups = p->groups_per_cu * cus;
  // class 1: streams whose slot is wider than the staged size
  for (size_t i = 0; i < n; ++i)
    if (lcs[i] != 0xFF && staged_cells(p->lds_mask, lcs[i], lps[i], pbs[i]) > p->table_cells)
      p->n_inplace++;
  size_t off = align_up(size_t(n) * sizeof(LzgpuSession), 256);
  p->sess_off = 0;
  // tables follow the sessions: probs_off counts cells from the workspace start
  const uint64_t tab0 = off / 2;
  for (size_t i = 0; i < n; ++i)
    if (descs[i].probs_off != LZMA_GPU_NO_WORKSPACE) descs[i].probs_off += tab0;
  off = align_up(off + size_t(cells_total) * 2, 256);
  p->list_off = off;
  off = align_up(off + 4 * size_t(std::max<size_t>(n, 1)) * sizeof(uint32_t), 256);
  p->ctr_off = off;
  off += 2 * (2 * size_t(p->rounds) + 2) * sizeof(uint32_t);
  p->workspace_bytes = align_up(off, 256);
  return SZ_OK;
}

template <int W, uint32_t M>
hipError_t launch_lane(const SlicedRound& a, uint32_t grid, size_t lds, hipStream_t st) {
  if (lzgpu_allow_full_lds(reinterpret_cast<const void*>(lzgpu_sliced_lane_kernel<W, M>)) != 0)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL((lzgpu_sliced_lane_kernel<W, M>), dim3(grid), dim3(64), lds, st, a);
  return hipGetLastError();
}

template <int W>
hipError_t launch_coop(const SlicedRound& a, uint32_t grid, size_t lds, hipStream_t st) {
  if (lzgpu_allow_full_lds(reinterpret_cast<const void*>(lzgpu_sliced_coop_kernel<W>)) != 0)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(lzgpu_sliced_coop_kernel<W>, dim3(grid), dim3(32), lds, st, a);
  return hipGetLastError();
}

SRes decode_sliced(const LzmaGpuSlicedPlan* p, const LzmaGpuStreamDesc* d_descs,
                   const uint32_t* d_order, const Byte* d_src, Byte* d_dst, void* d_ws,
                   LzmaGpuResult* d_results, unsigned first, unsigned count, hipStream_t st) {
  if (!p || p->slice_bytes == 0 || p->kernel == LZMA_GPU_SLICED_AUTO ||
      p->kernel > LZMA_GPU_SLICED_GLOBAL || first > p->rounds ||
      p->table_cells > kSlicedMaxLdsCells ||
      (p->kernel == LZMA_GPU_SLICED_LANE && p->lds_mask != kSlicedAll &&
       p->lds_mask != kSlicedHyb) ||
      (p->kernel != LZMA_GPU_SLICED_LANE && p->lds_mask != kSlicedAll))
    return SZ_ERROR_PARAM;
  if (!ensure_device()) return SZ_ERROR_FAIL;
  if (p->n == 0) return SZ_OK;
  if (!d_ws || !d_descs || !d_results) return SZ_ERROR_PARAM;
  uint8_t* ws = static_cast<uint8_t*>(d_ws);
  LzgpuSession* sess = reinterpret_cast<LzgpuSession*>(ws + p->sess_off);
  uint32_t* lists = reinterpret_cast<uint32_t*>(ws + p->list_off);
  uint32_t* ctr = reinterpret_cast<uint32_t*>(ws + p->ctr_off);
  const uint32_t n = uint32_t(p->n);
  const uint32_t cs = 2 * p->rounds + 2;  // counters per class
  const bool global_only = p->kernel == LZMA_GPU_SLICED_GLOBAL;
  const uint32_t stage_cells = global_only ? 0u : p->table_cells;
  if (first == 0) {
    if (!hip_ok(hipMemsetAsync(ctr, 0, 2 * size_t(cs) * sizeof(uint32_t), st),
                "sliced: reset counters"))
      return SZ_ERROR_FAIL;
    hipLaunchKernelGGL(lzgpu_sliced_init_kernel, dim3((n + 255) / 256), dim3(256), 0, st, d_descs,
                       d_order, n, d_src, d_dst, reinterpret_cast<uint16_t*>(ws), sess, d_results,
                       lists, ctr, cs, stage_cells, p->lds_mask);
    if (!hip_ok(hipGetLastError(), "sliced: init launch")) return SZ_ERROR_FAIL;
  }
  const unsigned last = count == 0 ? p->rounds : std::min<unsigned>(p->rounds, first + count);
  const uint32_t lds_words = sliced_vec(stage_cells) * 4u;
  const size_t lds = size_t(lds_words) * 4 + 16;
  // pad every workgroup's LDS so that exactly groups_per_cu fit on a CU
  const size_t lds_pad = std::max(lds, lzgpu_host::lds_share(std::max<uint32_t>(p->groups_per_cu, 1)));
  auto round_args = [&](unsigned r, uint32_t c) {
    SlicedRound a;
    a.sess = sess;
    a.results = d_results;
    a.list_in = lists + size_t(2 * c + (r & 1u)) * n;
    a.list_out = lists + size_t(2 * c + ((r + 1) & 1u)) * n;
    uint32_t* cc = ctr + size_t(c) * cs;
    a.cnt_in = cc + 2 * size_t(r);
    a.queue = cc + 2 * size_t(r) + 1;
    a.cnt_out = cc + 2 * size_t(r) + 2;
    a.slice = p->slice_bytes;
    a.lds_words = lds_words;
    return a;
  };
  for (unsigned r = first; r < last; ++r) {
    hipError_t e = hipSuccess;
    const bool w4 = p->groups_per_cu > 8;
    if (p->kernel == LZMA_GPU_SLICED_LANE) {
      const SlicedRound a = round_args(r, 0);
      if (p->lds_mask == kSlicedHyb)
        e = w4 ? launch_lane<4, kSlicedHyb>(a, p->max_groups, lds_pad, st)
               : launch_lane<2, kSlicedHyb>(a, p->max_groups, lds_pad, st);
      else
        e = w4 ? launch_lane<4, kSlicedAll>(a, p->max_groups, lds_pad, st)
               : launch_lane<2, kSlicedAll>(a, p->max_groups, lds_pad, st);
    } else if (p->kernel == LZMA_GPU_SLICED_COOP) {
      const SlicedRound a = round_args(r, 0);
      e = w4 ? launch_coop<4>(a, p->max_groups, lds_pad, st)
             : launch_coop<2>(a, p->max_groups, lds_pad, st);
    }
    if (e == hipSuccess && (global_only || p->n_inplace)) {
      const uint32_t m = global_only ? n : uint32_t(p->n_inplace);
      const uint32_t grid = std::min<uint32_t>(16 * lzgpu_host::device_cus(), (m + 63) / 64);
      hipLaunchKernelGGL(lzgpu_sliced_global_kernel, dim3(grid), dim3(64), 0, st,
                         round_args(r, 1));
      e = hipGetLastError();
    }
    if (!hip_ok(e, "sliced: round launch")) return SZ_ERROR_FAIL;
  }
  return SZ_OK;
}

}  // namespace

extern "C" {

SRes LzmaGpu_PlanSliced(LzmaGpuStreamDesc* descs, size_t n, uint64_t slice_bytes, unsigned kernel,
                        uint32_t* order, LzmaGpuSlicedPlan* plan) {
  if (!plan || (n && !descs)) return SZ_ERROR_PARAM;
  try {
    return plan_sliced(descs, n, slice_bytes, kernel, order, plan);
  } catch (const std::exception&) {
    return SZ_ERROR_MEM;
  }
}

SRes LzmaGpu_DecodeBatchSliced(const LzmaGpuSlicedPlan* plan, const LzmaGpuStreamDesc* d_descs,
                               const uint32_t* d_order, const Byte* d_src, Byte* d_dst,
                               void* d_workspace, LzmaGpuResult* d_results, unsigned first_round,
                               unsigned n_rounds, void* stream) {
  return decode_sliced(plan, d_descs, d_order, d_src, d_dst, d_workspace, d_results, first_round,
                       n_rounds, static_cast<hipStream_t>(stream));
}

SRes LzmaGpu_SlicedActive(const LzmaGpuSlicedPlan* plan, const void* d_workspace, unsigned round,
                          size_t* active, void* stream) {
  if (!plan || !active || round > plan->rounds) return SZ_ERROR_PARAM;
  if (!ensure_device()) return SZ_ERROR_FAIL;
  if (plan->n == 0) {
    *active = 0;
    return SZ_OK;
  }
  const hipStream_t st = static_cast<hipStream_t>(stream);
  const size_t cs = 2 * size_t(plan->rounds) + 2;
  uint32_t v[2] = {0, 0};
  const uint8_t* c = static_cast<const uint8_t*>(d_workspace) + plan->ctr_off;
  for (int k = 0; k < 2; ++k)
    if (!hip_ok(hipMemcpyAsync(&v[k], c + 4 * (size_t(k) * cs + 2 * size_t(round)), sizeof(uint32_t),
                               hipMemcpyDeviceToHost, st),
                "sliced: D2H count"))
      return SZ_ERROR_FAIL;
  if (!hip_ok(hipStreamSynchronize(st), "sliced: sync")) return SZ_ERROR_FAIL;
  *active = size_t(v[0]) + v[1];
  return SZ_OK;
}

SRes LzmaGpu_DecodeBatchSlicedHost(const LzmaGpuStreamDesc* descs, size_t n, const Byte* src,
                                   size_t src_bytes, Byte* dst, size_t dst_bytes,
                                   LzmaGpuResult* results, uint64_t slice_bytes, unsigned kernel,
                                   LzmaGpuSlicedPlan* plan_out) {
  if (!ensure_device()) return SZ_ERROR_FAIL;
  try {
    std::vector<LzmaGpuStreamDesc> d(descs, descs + n);
    std::vector<uint32_t> order(std::max<size_t>(n, 1));
    LzmaGpuSlicedPlan plan;
    const SRes pr = plan_sliced(d.data(), n, slice_bytes, kernel, order.data(), &plan);
    if (pr != SZ_OK) return pr;
    if (plan_out) *plan_out = plan;
    if (n == 0) return SZ_OK;
    lzgpu_host::DevArr<uint8_t> d_src, d_dst, d_ws;
    lzgpu_host::DevArr<LzmaGpuStreamDesc> d_desc;
    lzgpu_host::DevArr<uint32_t> d_order;
    lzgpu_host::DevArr<LzmaGpuResult> d_res;
    if (!d_src.alloc(std::max<size_t>(src_bytes, 16)) || !d_dst.alloc(std::max<size_t>(dst_bytes, 16)) ||
        !d_ws.alloc(size_t(plan.workspace_bytes)) || !d_desc.alloc(n) || !d_order.alloc(n) ||
        !d_res.alloc(n)) {
      set_error("sliced: device allocation failed");
      return SZ_ERROR_MEM;
    }
    if ((src_bytes && !hip_ok(hipMemcpy(d_src.p, src, src_bytes, hipMemcpyHostToDevice), "H2D src")) ||
        !hip_ok(hipMemcpy(d_desc.p, d.data(), n * sizeof(LzmaGpuStreamDesc), hipMemcpyHostToDevice),
                "H2D desc") ||
        !hip_ok(hipMemcpy(d_order.p, order.data(), n * sizeof(uint32_t), hipMemcpyHostToDevice),
                "H2D order"))
      return SZ_ERROR_FAIL;
    const SRes r = decode_sliced(&plan, d_desc.p, d_order.p, d_src.p, d_dst.p, d_ws.p, d_res.p, 0,
                                 0, nullptr);
    if (r != SZ_OK) return r;
    if (!hip_ok(hipDeviceSynchronize(), "sliced: decode") ||
        !hip_ok(hipMemcpy(results, d_res.p, n * sizeof(LzmaGpuResult), hipMemcpyDeviceToHost),
                "D2H results") ||
        (dst_bytes && !hip_ok(hipMemcpy(dst, d_dst.p, dst_bytes, hipMemcpyDeviceToHost), "D2H dst")))
      return SZ_ERROR_FAIL;
    return SZ_OK;
  } catch (const std::exception&) {
    set_error("sliced: host allocation failed");
    return SZ_ERROR_MEM;
  }
}

}  // extern "C"

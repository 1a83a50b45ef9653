// lzma_kernels.hip -- batch LZMA / LZMA2 decode kernels for gfx950.
//
// lzgpu_decode_lds_kernel (fast path, LZMA items whose lo table fits LDS):
//   one stream per lane, L lanes per workgroup (one wave with L active
//   lanes), each lane's lo probability table in its own LDS slice of
//   `stride` cells; the planner picks L so that about four workgroups share a
//   CU's 160 KiB.  The hardware dispatcher starts a new workgroup whenever
//   one retires, so a 64K-stream batch streams through the chip in waves of
//   resident workgroups with no host round trips.
// lzgpu_decode_batch_kernel (generic: any lc/lp/pb, LZMA2 ranges): 64 lanes
//   per workgroup, whole table in the item's global workspace slice.
// lzgpu_session_kernel: one LzmaDec_DecodeToDic call per lane on a
//   device-resident decoder state (dictionary / buffer interfaces).
// `order` (optional) maps lane -> descriptor so the planner can put streams of
// similar length into the same wave (a wave runs until its slowest lane ends).
// The per-lane work is in lzma_lane.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <set>
#include <utility>

#include "lzma_gpu_internal.h"

using namespace lzgpu;

// Dynamic-LDS limit of a kernel raised to the CU's 160 KiB once per device
// (the attribute is per device: a process driving several GPUs, or threads
// whose first launches race, each get it set before their launch).
static int allow_full_lds(const void* kfn) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kLzgpuMaxDevices) return -1;
  static std::mutex mu;
  static std::set<std::pair<const void*, int>> done;
  std::lock_guard<std::mutex> g(mu);
  if (done.count({kfn, dev})) return 0;
  if (hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) !=
      hipSuccess)
    return -1;
  done.insert({kfn, dev});
  return 0;
}

int lzgpu_allow_full_lds(const void* kfn) { return allow_full_lds(kfn); }

__global__ void __launch_bounds__(64) lzgpu_decode_batch_kernel(
    const LzmaGpuStreamDesc* __restrict__ descs, const uint32_t* __restrict__ order, uint32_t n,
    const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint16_t* __restrict__ ws,
    LzmaGpuResult* __restrict__ results) {
  const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= n) return;
  const uint32_t id = order ? order[lane] : lane;
  const LzmaGpuStreamDesc d = descs[id];
  results[id] = lane_decode(d, src, dst, ws);
}

// W = minimum waves per SIMD the register allocation must allow (the
// planner's occupancy target; more resident waves hide the serial decode
// chain of each stream better, at the price of register spills).
// Persistent lanes: the grid is sized to what is resident at once; a lane
// that finishes its stream takes the next one from `queue` (a counter the
// launcher zeroes), so no lane idles behind a slower neighbour in its wave
// and the chip drains without a partial last round of workgroups.  Every
// lane exits once the queue passes n.  Lane l starts on stream l and then
// takes start + (queue ticket): start = the lanes of the launch.
// K2: the build carries the LZMA2 chunk walker (classes with LZMA2 items); the
// LZMA-only build needs fewer registers (169 vs 202 VGPRs at W = 2, 21 vs 153
// spilled at W = 4), so classes without LZMA2 items launch it.
// Lane-interleaved placements (M & kIlvBit): the global sections live in the
// class's slot area (`slot_off` cells into ws) instead of per-stream slices --
// lane group g (32 lanes of one workgroup) owns rows of kIlv cells, `slot_cells`
// rows, and lane l its column l; the lane keeps its column for every stream
// it takes from the queue.

template <int W, uint32_t M, bool K2>
__global__ void __launch_bounds__(64, W) lzgpu_decode_lds_kernel(
    const LzmaGpuStreamDesc* __restrict__ descs, const uint32_t* __restrict__ order, uint32_t n,
    const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint16_t* __restrict__ ws,
    LzmaGpuResult* __restrict__ results, uint32_t stride, uint32_t* __restrict__ queue,
    uint64_t slot_off, uint32_t slot_cells, uint32_t start) {
  extern __shared__ uint32_t lz_smem[];
  // the lane's LDS slice; interleaved (lds_ilv): its column of its 32-lane
  // group's rows
  lds_u16* lo = (lds_u16*)((uint16_t*)lz_smem);
  if constexpr (lds_ilv<M>())
    lo += (threadIdx.x / kIlv) * (kIlv * stride) + (threadIdx.x % kIlv);
  else
    lo += threadIdx.x * stride;
  uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
  gu16* gcol = nullptr;
  if constexpr ((M & kIlvBit) != 0u) {
    const uint32_t grp = blockIdx.x * ((blockDim.x + kIlv - 1) / kIlv) + threadIdx.x / kIlv;
    gcol = (gu16*)(ws + slot_off) + uint64_t(grp) * slot_cells * kIlv +
           (threadIdx.x % kIlv) * kIlvLaneCells;
  }
  (void)slot_off;
  (void)slot_cells;
  while (idx < n) {
    const uint32_t id = order ? order[idx] : idx;
    const LzmaGpuStreamDesc d = descs[id];
    results[id] = lane_decode_lds<M, K2>(d, src, dst, ws, lo, stride, gcol);
    idx = start + atomicAdd(queue, 1u);
  }
}

// One-stream waves of the latency placement (round 5): the one-lane decoder
// run by all D lanes of a workgroup on the same stream -- the instruction
// stream of lzgpu_decode_lds_kernel with one lane per wave, but with D >= 16
// lanes in EXEC.  The SIMD issue micro-benchmark (scripts/ubench/
// simd_issue_ubench.hip lanes, profiles/r05_issue/simd_lanes.jsonl) finds a
// VALU instruction of a wave with 1-8 active lanes issuing once per ~16.7
// cycles alone on its SIMD and at 3.5 cycles per SIMD with four such waves,
// against 4.8 / 2.5 cycles with 16 or more lanes; a dependent LDS decision
// chain takes 98 against 75 cycles per SIMD at four waves.  Config 2 6.28 ->
// 6.86 GB/s, config 5 5.13 -> 5.58 (profiles/r05_dup/).  The lanes share the
// workgroup's LDS slice and store identical values to identical addresses;
// lane 0 writes the result and takes the next stream from the queue.
constexpr int kLaneDup = 32;
template <int W, uint32_t M, bool K2>
__global__ void __launch_bounds__(64, W) lzgpu_decode_dup_kernel(
    const LzmaGpuStreamDesc* __restrict__ descs, const uint32_t* __restrict__ order, uint32_t n,
    const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint16_t* __restrict__ ws,
    LzmaGpuResult* __restrict__ results, uint32_t stride, uint32_t* __restrict__ queue) {
  extern __shared__ uint32_t lz_smem[];
  lds_u16* lo = (lds_u16*)((uint16_t*)lz_smem);
  uint32_t idx = blockIdx.x;
  while (idx < n) {
    const uint32_t id = order ? order[idx] : idx;
    LzmaGpuStreamDesc d = descs[id];
    // keep the shared decoder state in vector registers (lz_vzero)
    const uint32_t z = lz_vzero();
    d.src_off += z;
    d.dst_off += z;
    const LzmaGpuResult r = lane_decode_lds<M | kDupBit, K2>(d, src, dst, ws, lo, stride, nullptr);
    uint32_t next = 0;
    if (threadIdx.x == 0) {
      results[id] = r;
      next = gridDim.x + atomicAdd(queue, 1u);
    }
    idx = uint32_t(__builtin_amdgcn_readfirstlane(int(next)));
  }
}

// Wave-cooperative decode (latency regime): one stream per workgroup of one
// 32-lane wave.  Every lane runs the same decoder on the same state, so control
// flow and memory traffic are those of one lane -- except match copies (byte j
// by lane j mod 32, lz_copy_coop), the direct bits of a distance (several per
// step, direct_coop) and table initialisation.  Lane 0 takes the next stream
// from the queue.
// Under kWinBit the workgroup's LDS holds, after the table (`stride` cells,
// 16-byte aligned), the LDS history window of `win_bytes` (lzma_device.h):
// match copies and matched bytes within its reach are LDS reads.
template <int W, uint32_t M, bool K2>
__global__ void __launch_bounds__(32, W) lzgpu_decode_coop_kernel(
    const LzmaGpuStreamDesc* __restrict__ descs, const uint32_t* __restrict__ order, uint32_t n,
    const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint16_t* __restrict__ ws,
    LzmaGpuResult* __restrict__ results, uint32_t stride, uint32_t* __restrict__ queue,
    uint32_t win_bytes) {
  extern __shared__ uint32_t lz_smem[];
  lds_u16* lo = (lds_u16*)((uint16_t*)lz_smem);
  lds_u8* win = (lds_u8*)((uint8_t*)lz_smem) + ((size_t(stride) * 2 + 15) & ~size_t(15));
  uint32_t idx = blockIdx.x;
  while (idx < n) {
    const uint32_t id = order ? order[idx] : idx;
    LzmaGpuStreamDesc d = descs[id];
    // keep the shared decoder state in vector registers (lz_vzero)
    const uint32_t z = lz_vzero();
    d.src_off += z;
    d.dst_off += z;
    const LzmaGpuResult r =
        lane_decode_lds<M, K2>(d, src, dst, ws, lo, stride, nullptr, win, win_bytes);
    uint32_t next = 0;
    if (threadIdx.x == 0) {
      results[id] = r;
      next = gridDim.x + atomicAdd(queue, 1u);
    }
    idx = uint32_t(__builtin_amdgcn_readfirstlane(int(next)));
  }
}

// One DecodeToDic call per lane on a device-resident decoder state.
__global__ void __launch_bounds__(64) lzgpu_session_kernel(LzgpuSession* __restrict__ sess,
                                                           uint32_t n) {
  const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= n) return;
  lane_session(sess[lane]);
}

// One DecodeToDic / DecodeToBuf call per workgroup of one 32-lane wave on a
// device-resident decoder (the drop-in LzmaDec_DecodeToDic / DecodeToBuf of a
// host CLzmaDec, and small session batches): the wave-cooperative decoder with
// the session's whole table staged in LDS for the call -- loaded from
// q.probs, decoded on (every table access an LDS round trip instead of a
// global one), written back.  Placement
// 0x7FF keeps the all-global layout's offsets, so the copy is a straight one.
// Dynamic LDS: the widest table of the batch's sessions (the launcher checks).
// WIN: the LDS history window (win_bytes, after the table) is preloaded per
// call with the dictionary bytes a match can reach (lane_session).
constexpr uint32_t kSessCoopMask = LZGPU_LDS_MASK_ALL | kCoopBit;
template <bool WIN>
__global__ void __launch_bounds__(32) lzgpu_session_coop_kernel(LzgpuSession* __restrict__ sess,
                                                                 uint32_t n, uint32_t lds_cells,
                                                                 uint32_t win_bytes) {
  extern __shared__ uint32_t lz_smem[];
  lds_u16* lo = (lds_u16*)((uint16_t*)lz_smem);
  lds_u8* win = (lds_u8*)((uint8_t*)lz_smem) + ((size_t(lds_cells) * 2 + 15) & ~size_t(15));
  constexpr uint32_t MS = kSessCoopMask | (WIN ? kWinBit : 0u);
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    LzgpuSession q = sess[i];
    // keep the shared decoder state in vector registers (lz_vzero)
    {
      const uint32_t z = lz_vzero();
      q.in = (const uint8_t*)q.in + z;
      q.dic = (uint8_t*)q.dic + z;
    }
    const uint32_t cells = table_cells(q.lc, q.lp, q.pb);
    if (cells > lds_cells) {  // planned for narrower tables: refuse, state untouched
      if (threadIdx.x == 0) {
        sess[i].res = kErrMem;
        sess[i].status = kStNone;
      }
      continue;
    }
    gu16* gp = (gu16*)q.probs;
    for (uint32_t j = threadIdx.x; j < cells; j += blockDim.x) lo[j] = gp[j];
    __syncthreads();
    lane_session<MS>(q, lo, win, win_bytes);
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < cells; j += blockDim.x) gp[j] = lo[j];
    if (threadIdx.x == 0) sess[i] = q;
    __syncthreads();
  }
}

// Window for a launch of `grid` one-wave workgroups whose tables take
// `table_bytes` of LDS: the largest power of two that still leaves room for
// every workgroup a CU holds at once (one each while the grid fits the CUs),
// at most 128 KiB; 0 (no window) below 4 KiB.  LZGPU_WIN=0 disables it.
static uint32_t window_bytes(uint64_t grid, size_t table_bytes, uint32_t groups_per_cu) {
  static const bool off = [] {
    const char* e = getenv("LZGPU_WIN");
    return e && e[0] == '0';
  }();
  if (off) return 0;
  const uint32_t cus = lzgpu_host::device_cus();
  uint64_t per_cu = (grid + cus - 1) / cus;
  if (groups_per_cu && per_cu > groups_per_cu) per_cu = groups_per_cu;
  if (per_cu == 0) per_cu = 1;
  const size_t share = lzgpu_host::lds_share(per_cu);
  const size_t tb = (table_bytes + 15) & ~size_t(15);
  if (share <= tb + 4096) return 0;
  uint32_t w = 1u << 17;
  while (w > share - tb) w >>= 1;
  return w >= 4096 ? w : 0;
}

extern "C" int lzgpu_launch_session_coop(LzgpuSession* d_sess, uint32_t n, uint32_t lds_cells,
                                         uint32_t max_groups, hipStream_t stream) {
  if (n == 0) return 0;
  if (lds_cells == 0 || size_t(lds_cells) * 2 > 160 * 1024) return -1;
  uint32_t grid = n;
  if (max_groups && grid > max_groups) grid = max_groups;
  const uint32_t win = window_bytes(grid, size_t(lds_cells) * 2, 0);
  const size_t lds = win ? ((size_t(lds_cells) * 2 + 15) & ~size_t(15)) + win : size_t(lds_cells) * 2;
  const void* kfn = win ? reinterpret_cast<const void*>(lzgpu_session_coop_kernel<true>)
                        : reinterpret_cast<const void*>(lzgpu_session_coop_kernel<false>);
  if (lds > 64 * 1024 && allow_full_lds(kfn) != 0) return -1;
  if (win)
    hipLaunchKernelGGL(lzgpu_session_coop_kernel<true>, dim3(grid), dim3(32), lds, stream, d_sess,
                       n, lds_cells, win);
  else
    hipLaunchKernelGGL(lzgpu_session_coop_kernel<false>, dim3(grid), dim3(32), lds, stream,
                       d_sess, n, lds_cells, 0u);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int lzgpu_launch_decode_batch(const LzmaGpuStreamDesc* d_descs, const uint32_t* d_order,
                                         uint32_t n, const uint8_t* d_src, uint8_t* d_dst,
                                         uint16_t* d_ws, LzmaGpuResult* d_results,
                                         hipStream_t stream) {
  if (n == 0) return 0;
  const uint32_t block = 64;
  const uint32_t grid = (n + block - 1) / block;
  hipLaunchKernelGGL(lzgpu_decode_batch_kernel, dim3(grid), dim3(block), 0, stream, d_descs,
                     d_order, n, d_src, d_dst, d_ws, d_results);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// One-stream waves on kLaneDup lanes (lzgpu_decode_dup_kernel): `groups_per_cu`
// one-wave workgroups per CU, each padded to its share of the CU's LDS blocks.
template <int W, uint32_t M, bool K2>
static int launch_dup(const LzmaGpuStreamDesc* d_descs, const uint32_t* d_order, uint32_t n,
                      const uint8_t* d_src, uint8_t* d_dst, uint16_t* d_ws,
                      LzmaGpuResult* d_results, uint32_t stride, uint32_t groups_per_cu,
                      uint32_t max_groups, uint32_t* d_queue, uint32_t dup, hipStream_t stream) {
  auto kd = lzgpu_decode_dup_kernel<W, M, K2>;
  if (allow_full_lds(reinterpret_cast<const void*>(kd)) != 0) return -1;
  if (hipMemsetAsync(d_queue, 0, sizeof(uint32_t), stream) != hipSuccess) return -1;
  size_t lds = size_t(stride) * 2;
  if (groups_per_cu) lds = std::max(lds, lzgpu_host::lds_share(groups_per_cu));
  uint32_t grid = n;
  if (max_groups && grid > max_groups) grid = max_groups;
  hipLaunchKernelGGL(kd, dim3(grid), dim3(dup), lds, stream, d_descs, d_order, n, d_src, d_dst,
                     d_ws, d_results, stride, d_queue);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// kLaneDup, or LZGPU_DUP=D for A/B (D = 1 launches the one-lane kernel)
static int lane_dup() {
  static const int dup = [] {
    const char* e = getenv("LZGPU_DUP");
    return e ? atoi(e) : kLaneDup;
  }();
  return dup;
}

template <int W, uint32_t M, bool K2>
static int launch_lds(const LzmaGpuStreamDesc* d_descs, const uint32_t* d_order, uint32_t n,
                      const uint8_t* d_src, uint8_t* d_dst, uint16_t* d_ws,
                      LzmaGpuResult* d_results, uint32_t lanes, uint32_t stride,
                      uint32_t groups_per_cu, uint32_t max_groups, uint32_t* d_queue,
                      const LzgpuSlots& sl, hipStream_t stream) {
  if (allow_full_lds(reinterpret_cast<const void*>(lzgpu_decode_lds_kernel<W, M, K2>)) != 0)
    return -1;
  if (hipMemsetAsync(d_queue, 0, sizeof(uint32_t), stream) != hipSuccess) return -1;
  // pad each workgroup's LDS so that exactly groups_per_cu fit on a CU (an
  // even split over its four SIMDs), whatever the dispatcher would pack;
  // interleaved slices take whole 32-lane rows
  size_t lds = size_t(lds_ilv<M>() ? (lanes + kIlv - 1) / kIlv * kIlv : lanes) * stride * 2;
  if (groups_per_cu) {
    const size_t share = lzgpu_host::lds_share(groups_per_cu);
    if (share > lds) lds = share;
  }
  uint32_t grid = (n + lanes - 1) / lanes;
  if (max_groups && grid > max_groups) grid = max_groups;
  if constexpr ((M & kIlvBit) != 0u) {
    // the slot area holds sl.groups workgroups' columns; persistent lanes
    // cover the rest of the batch from the queue
    if (sl.groups == 0 || lanes > 64) return -1;
    if (grid > sl.groups) {
      if (!max_groups) return -1;
      grid = sl.groups;
    }
  }
  const uint32_t lanes_total = grid * lanes;
  if constexpr (M == LZGPU_LDS_MASK_LAT) {
    // one-stream waves: kLaneDup lanes per stream
    const int dup = lane_dup();
    if (lanes == 1 && dup > 1 && dup <= 64) {
      auto kd = lzgpu_decode_dup_kernel<W, M, K2>;
      if (allow_full_lds(reinterpret_cast<const void*>(kd)) != 0) return -1;
      hipLaunchKernelGGL(kd, dim3(grid), dim3(dup), lds, stream, d_descs, d_order, n, d_src, d_dst,
                         d_ws, d_results, stride, d_queue);
      return hipGetLastError() == hipSuccess ? 0 : -1;
    }
  }
  auto kfn = lzgpu_decode_lds_kernel<W, M, K2>;
  hipLaunchKernelGGL(kfn, dim3(grid), dim3(lanes), lds, stream, d_descs, d_order, n, d_src, d_dst,
                     d_ws, d_results, stride, d_queue, sl.off, sl.cells, lanes_total);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// MW: the same placement with the LDS history window, launched instead when
// the launch leaves room for one (window_bytes); 0 = no window build.
template <int W, uint32_t M, bool K2, uint32_t MW = 0u>
static int launch_coop(const LzmaGpuStreamDesc* d_descs, const uint32_t* d_order, uint32_t n,
                       const uint8_t* d_src, uint8_t* d_dst, uint16_t* d_ws,
                       LzmaGpuResult* d_results, uint32_t stride, uint32_t groups_per_cu,
                       uint32_t max_groups, uint32_t* d_queue, hipStream_t stream) {
  uint32_t grid = n;
  if (max_groups && grid > max_groups) grid = max_groups;
  const uint32_t win = MW ? window_bytes(grid, size_t(stride) * 2, groups_per_cu) : 0u;
  auto kfn = win ? lzgpu_decode_coop_kernel<W, (MW ? MW : M), K2> : lzgpu_decode_coop_kernel<W, M, K2>;
  if (allow_full_lds(reinterpret_cast<const void*>(kfn)) != 0) return -1;
  if (hipMemsetAsync(d_queue, 0, sizeof(uint32_t), stream) != hipSuccess) return -1;
  size_t lds = size_t(stride) * 2;
  if (win) {
    lds = ((lds + 15) & ~size_t(15)) + win;
  } else if (groups_per_cu) {
    const size_t share = lzgpu_host::lds_share(groups_per_cu);
    if (share > lds) lds = share;
  }
  hipLaunchKernelGGL(kfn, dim3(grid), dim3(32), lds, stream, d_descs, d_order, n, d_src, d_dst,
                     d_ws, d_results, stride, d_queue, win);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <uint32_t M, bool K2>
static int launch_lds_w(const LzmaGpuStreamDesc* d_descs, const uint32_t* d_order, uint32_t n,
                        const uint8_t* d_src, uint8_t* d_dst, uint16_t* d_ws,
                        LzmaGpuResult* d_results, uint32_t lanes, uint32_t stride,
                        uint32_t waves_per_simd, uint32_t groups_per_cu, uint32_t max_groups,
                        uint32_t* d_queue, const LzgpuSlots& sl, hipStream_t stream) {
  if (waves_per_simd <= 1)
    return launch_lds<1, M, K2>(d_descs, d_order, n, d_src, d_dst, d_ws, d_results, lanes, stride,
                                groups_per_cu, max_groups, d_queue, sl, stream);
  if (waves_per_simd == 2)
    return launch_lds<2, M, K2>(d_descs, d_order, n, d_src, d_dst, d_ws, d_results, lanes, stride,
                                groups_per_cu, max_groups, d_queue, sl, stream);
  return launch_lds<4, M, K2>(d_descs, d_order, n, d_src, d_dst, d_ws, d_results, lanes, stride,
                              groups_per_cu, max_groups, d_queue, sl, stream);
}

// Workgroups a CU actually holds at once: the launch's workgroups spread over
// the CUs, so at most min(groups_per_cu, ceil(n / cus)).  The register budget
// (the W of __launch_bounds__) follows it: a plan for 16 narrow-table
// cooperative waves per CU that gets one stream (a lone drop-in call) would
// otherwise run the W = 4 build, 128 VGPRs and 46-218 spilled, instead of the
// W = 2 build without spills.
static uint32_t resident_waves_per_simd(uint32_t n, uint32_t groups_per_cu) {
  const uint32_t cus = std::max(1u, lzgpu_host::device_cus());
  const uint32_t per_cu = std::max(1u, std::min(groups_per_cu, (n + cus - 1) / cus));
  return (per_cu + 3) / 4;
}

template <bool K2>
static int launch_class(const LzmaGpuStreamDesc* d_descs, const uint32_t* d_order, uint32_t n,
                        const uint8_t* d_src, uint8_t* d_dst, uint16_t* d_ws,
                        LzmaGpuResult* d_results, uint32_t lanes, uint32_t stride,
                        uint32_t waves_per_simd, uint32_t groups_per_cu, uint32_t max_groups,
                        uint32_t* d_queue, uint32_t lds_mask, const LzgpuSlots& sl,
                        hipStream_t stream, uint32_t class_flags) {
  if (lds_mask == LZGPU_LDS_MASK)
    return launch_lds_w<LZGPU_LDS_MASK, K2>(d_descs, d_order, n, d_src, d_dst, d_ws, d_results,
                                            lanes, stride, waves_per_simd, groups_per_cu,
                                            max_groups, d_queue, sl, stream);
  if (lds_mask == (LZGPU_LDS_MASK | kIlvBit))
    return launch_lds_w<LZGPU_LDS_MASK | kIlvBit, K2>(d_descs, d_order, n, d_src, d_dst, d_ws,
                                                      d_results, lanes, stride, waves_per_simd,
                                                      groups_per_cu, max_groups, d_queue, sl,
                                                      stream);
  if (lds_mask == (LZGPU_LDS_MASK_LAT | kCoopBit)) {
    // one wave per workgroup: register budget by workgroups per SIMD
    constexpr uint32_t MC = LZGPU_LDS_MASK_LAT | kCoopBit;
    const uint32_t w = resident_waves_per_simd(n, groups_per_cu);
    if (w <= 2)
      return launch_coop<2, MC, K2>(d_descs, d_order, n, d_src, d_dst, d_ws, d_results, stride,
                                    groups_per_cu, max_groups, d_queue, stream);
    return launch_coop<4, MC, K2>(d_descs, d_order, n, d_src, d_dst, d_ws, d_results, stride,
                                  groups_per_cu, max_groups, d_queue, stream);
  }
  if (lds_mask == (LZGPU_LDS_MASK_ALL | kCoopBit)) {
    // the whole table in LDS, plus the history window where the launch has room
    constexpr uint32_t MC = LZGPU_LDS_MASK_ALL | kCoopBit;
    const uint32_t w = resident_waves_per_simd(n, groups_per_cu);
    if (w <= 2)
      return launch_coop<2, MC, K2, MC | kWinBit>(d_descs, d_order, n, d_src, d_dst, d_ws,
                                                  d_results, stride, groups_per_cu, max_groups,
                                                  d_queue, stream);
    return launch_coop<4, MC, K2, MC | kWinBit>(d_descs, d_order, n, d_src, d_dst, d_ws, d_results,
                                                stride, groups_per_cu, max_groups, d_queue,
                                                stream);
  }
  if (lds_mask == kLdsMaskLatSlotG) {
    // planned for one-stream workgroups only (lzma_capi.hip plan_bucket)
    const int dup = lane_dup();
    if (lanes != 1 || dup <= 1 || dup > 64) return -1;
    const uint32_t w = std::min(waves_per_simd, resident_waves_per_simd(n, groups_per_cu));
    if (w <= 1)
      return launch_dup<1, kLdsMaskLatSlotG, K2>(d_descs, d_order, n, d_src, d_dst, d_ws,
                                                 d_results, stride, groups_per_cu, max_groups,
                                                 d_queue, uint32_t(dup), stream);
    if (w == 2)
      return launch_dup<2, kLdsMaskLatSlotG, K2>(d_descs, d_order, n, d_src, d_dst, d_ws,
                                                 d_results, stride, groups_per_cu, max_groups,
                                                 d_queue, uint32_t(dup), stream);
    return launch_dup<4, kLdsMaskLatSlotG, K2>(d_descs, d_order, n, d_src, d_dst, d_ws, d_results,
                                               stride, groups_per_cu, max_groups, d_queue,
                                               uint32_t(dup), stream);
  }
  if (lds_mask == LZGPU_LDS_MASK_LAT)
    return launch_lds_w<LZGPU_LDS_MASK_LAT, K2>(d_descs, d_order, n, d_src, d_dst, d_ws,
                                                d_results, lanes, stride,
                                                lanes == 1 ? std::min(waves_per_simd,
                                                                      resident_waves_per_simd(
                                                                          n, groups_per_cu))
                                                           : waves_per_simd,
                                                groups_per_cu, max_groups, d_queue, sl, stream);
  return -1;  // no kernel built for this placement
}

extern "C" int lzgpu_launch_decode_lds(const LzmaGpuStreamDesc* d_descs, const uint32_t* d_order,
                                       uint32_t n, const uint8_t* d_src, uint8_t* d_dst,
                                       uint16_t* d_ws, LzmaGpuResult* d_results, uint32_t lanes,
                                       uint32_t stride, uint32_t waves_per_simd,
                                       uint32_t groups_per_cu, uint32_t max_groups,
                                       uint32_t* d_queue, uint32_t lds_mask,
                                       uint32_t class_flags, LzgpuSlots slots,
                                       hipStream_t stream) {
  if (n == 0) return 0;
  if (class_flags & LZMA_GPU_CLASS_HAS_LZMA2)
    return launch_class<true>(d_descs, d_order, n, d_src, d_dst, d_ws, d_results, lanes, stride,
                              waves_per_simd, groups_per_cu, max_groups, d_queue, lds_mask,
                              slots, stream, class_flags);
  return launch_class<false>(d_descs, d_order, n, d_src, d_dst, d_ws, d_results, lanes, stride,
                             waves_per_simd, groups_per_cu, max_groups, d_queue, lds_mask, slots,
                             stream, class_flags);
}

extern "C" int lzgpu_launch_session(LzgpuSession* d_sess, uint32_t n, hipStream_t stream) {
  if (n == 0) return 0;
  const uint32_t block = 64;
  const uint32_t grid = (n + block - 1) / block;
  hipLaunchKernelGGL(lzgpu_session_kernel, dim3(grid), dim3(block), 0, stream, d_sess, n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

#if LZGPU_PROF
// profiling builds: read (and optionally clear) the region cycle sums -- 40
// counters, out[22] = the build's LZGPU_PROF level
extern "C" int LzmaGpu_ProfileRead(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(lzgpu::g_lz_prof), 40 * sizeof(unsigned long long)) !=
      hipSuccess)
    return -1;
  out[22] = LZGPU_PROF;
  if (reset) {
    unsigned long long z[40] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(lzgpu::g_lz_prof), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}
#endif

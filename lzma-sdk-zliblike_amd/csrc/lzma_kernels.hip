// lzma_kernels.hip -- batch LZMA / LZMA2 decode kernels for gfx950.
//
// Grid mapping: one stream per lane, 64-lane workgroups (one wave each).
// `order` (optional) maps lane -> descriptor so the host planner can group
// streams of similar size and table width into the same wave (a wave runs
// until its slowest lane finishes).
//
// Per lane the kernels run exactly the reference's one-call contracts:
//   lzgpu_decode_batch_kernel   LzmaDecode      (LzmaDec.c:972-1002)
//   lzgpu_lzma2_batch_kernel    LZMA2 block decode over a flat dictionary
//                               (Lzma2Dec.c:90-289 as driven by 7zDec.c:181-202)
//   lzgpu_session_kernel        LzmaDec_DecodeToDic on a device-resident
//                               decoder state (the dictionary/streaming APIs)
#include <hip/hip_runtime.h>

#include "lzma2_device.h"
#include "lzma_device.h"
#include "lzma_gpu_internal.h"

using namespace lzgpu;

__global__ void __launch_bounds__(64) lzgpu_decode_batch_kernel(
    const LzmaGpuStreamDesc* __restrict__ descs, const uint32_t* __restrict__ order, uint32_t n,
    const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint16_t* __restrict__ ws,
    LzmaGpuResult* __restrict__ results) {
  const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= n) return;
  const uint32_t id = order ? order[lane] : lane;
  const LzmaGpuStreamDesc d = descs[id];
  LzmaGpuResult r;
  r.status = -1;
  r.dest_len = 0;
  r.src_len = 0;
  if (d.kind == LZMA_GPU_KIND_LZMA2) {
    Lz2State p;
    r.res = lz2_init(p, d.props[0], ws + d.probs_off, dst + d.dst_off, d.dst_cap);
    if (r.res == kOk) {
      if (d.probs_off == LZMA_GPU_NO_WORKSPACE) {
        r.res = kErrMem;
      } else {
        uint64_t sl = d.src_len;
        int status = kStNone;
        int res = lz2_decode_to_dic(p, d.dst_cap, src + d.src_off, sl, d.finish_mode, status);
        if (res == kOk && status == kStMoreInput) res = kErrInputEof;
        r.res = res;
        r.status = status;
        r.dest_len = p.dec.pos;
        r.src_len = sl;
      }
    }
    results[id] = r;
    return;
  }
  // LzmaDecode
  if (d.src_len < 5) {
    r.res = kErrInputEof;
    results[id] = r;
    return;
  }
  LzState s;
  r.res = lz_props_parse(d.props, d.props_size, s.lc, s.lp, s.pb, s.dict_size);
  if (r.res != kOk) {
    results[id] = r;
    return;
  }
  if (d.probs_off == LZMA_GPU_NO_WORKSPACE) {
    r.res = kErrMem;
    results[id] = r;
    return;
  }
  s.probs = ws + d.probs_off;
  s.dic = dst + d.dst_off;
  s.cap = d.dst_cap;
  s.pos = 0;
  s.range = s.code = 0;
  s.st = 0;
  s.rep0 = s.rep1 = s.rep2 = s.rep3 = 1;
  s.need_state_init = 0;
  lz_init_dic_state(s, true, true);
  uint64_t sl = d.src_len;
  int status = kStNone;
  int res = lz_decode_to_dic(s, d.dst_cap, src + d.src_off, sl, d.finish_mode, status);
  if (res == kOk && status == kStMoreInput) res = kErrInputEof;
  r.res = res;
  r.status = status;
  r.dest_len = s.pos;
  r.src_len = sl;
  results[id] = r;
}

// One DecodeToDic call per lane on a device-resident decoder state.
__global__ void __launch_bounds__(64) lzgpu_session_kernel(LzgpuSession* __restrict__ sess,
                                                           uint32_t n) {
  const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= n) return;
  LzgpuSession& q = sess[lane];
  LzState s;
  s.lc = q.lc;
  s.lp = q.lp;
  s.pb = q.pb;
  s.dict_size = q.dict_size;
  s.probs = q.probs;
  s.dic = q.dic;
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
  int res = lz_decode_to_dic(s, q.dic_limit, q.in, sl, q.finish_mode, status);
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

extern "C" int lzgpu_launch_session(LzgpuSession* d_sess, uint32_t n, hipStream_t stream) {
  if (n == 0) return 0;
  const uint32_t block = 64;
  const uint32_t grid = (n + block - 1) / block;
  hipLaunchKernelGGL(lzgpu_session_kernel, dim3(grid), dim3(block), 0, stream, d_sess, n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

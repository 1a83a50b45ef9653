// lzma_gpu_internal.h -- structures shared by the kernels and the host C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/lzma_gpu.h"

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

extern "C" int lzgpu_launch_decode_batch(const LzmaGpuStreamDesc* d_descs, const uint32_t* d_order,
                                         uint32_t n, const uint8_t* d_src, uint8_t* d_dst,
                                         uint16_t* d_ws, LzmaGpuResult* d_results,
                                         hipStream_t stream);
extern "C" int lzgpu_launch_session(LzgpuSession* d_sess, uint32_t n, hipStream_t stream);

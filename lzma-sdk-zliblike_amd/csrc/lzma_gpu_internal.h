// lzma_gpu_internal.h -- kernel launch entry points used by the host C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lzma_lane.h"

extern "C" int lzgpu_launch_decode_batch(const LzmaGpuStreamDesc* d_descs, const uint32_t* d_order,
                                         uint32_t n, const uint8_t* d_src, uint8_t* d_dst,
                                         uint16_t* d_ws, LzmaGpuResult* d_results,
                                         hipStream_t stream);
extern "C" int lzgpu_launch_session(LzgpuSession* d_sess, uint32_t n, hipStream_t stream);
extern "C" int lzgpu_launch_decode_lds(const LzmaGpuStreamDesc* d_descs, const uint32_t* d_order,
                                       uint32_t n, const uint8_t* d_src, uint8_t* d_dst,
                                       uint16_t* d_ws, LzmaGpuResult* d_results, uint32_t lanes,
                                       uint32_t stride, uint32_t waves_per_simd,
                                       uint32_t groups_per_cu, uint32_t max_groups,
                                       uint32_t* d_queue, uint32_t lds_mask,
                                       hipStream_t stream);
extern "C" int lzgpu_launch_crc_arrays(const uint8_t* d_data, const uint64_t* d_off,
                                       const uint64_t* d_len, uint32_t n,
                                       const uint32_t* d_chunk_base,
                                       const uint32_t* d_chunk_range, uint32_t n_chunks,
                                       uint32_t init, uint32_t xorout, uint32_t* d_chunk_crc,
                                       uint32_t* d_crc, hipStream_t stream);
extern "C" int lzgpu_launch_crc64_arrays(const uint8_t* d_data, const uint64_t* d_off,
                                         const uint64_t* d_len, uint32_t n,
                                         const uint32_t* d_chunk_base,
                                         const uint32_t* d_chunk_range, uint32_t n_chunks,
                                         uint64_t init, uint64_t xorout, uint64_t* d_chunk_crc,
                                         uint64_t* d_crc, hipStream_t stream);
extern "C" int lzgpu_launch_bcj_x86(uint8_t* d_data, const uint64_t* d_off, const uint64_t* d_len,
                                    const uint32_t* d_ip, uint32_t* d_state, uint64_t* d_done,
                                    uint32_t n, int encoding, hipStream_t stream);

// host-side helpers shared by the C-ABI translation units (lzma_capi.hip)
namespace lzgpu_host {
bool ensure_device();
void set_error(const char* what);
bool hip_ok(hipError_t e, const char* what);
}  // namespace lzgpu_host

extern "C" int lzgpu_launch_crc_decoded(const LzmaGpuStreamDesc* d_descs,
                                        const LzmaGpuResult* d_results, const uint8_t* d_dst,
                                        uint32_t n, const uint32_t* d_chunk_base,
                                        const uint32_t* d_chunk_range, uint32_t n_chunks,
                                        uint32_t* d_chunk_crc, uint32_t* d_crc,
                                        hipStream_t stream);

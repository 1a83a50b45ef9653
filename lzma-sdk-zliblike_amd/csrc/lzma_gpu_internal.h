// lzma_gpu_internal.h -- kernel launch entry points used by the host C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lzma_lane.h"

// Devices the library keeps per-device state for (launch attributes, class
// streams, CU counts, dictionary mirrors).
constexpr int kLzgpuMaxDevices = 64;

extern "C" int lzgpu_launch_decode_batch(const LzmaGpuStreamDesc* d_descs, const uint32_t* d_order,
                                         uint32_t n, const uint8_t* d_src, uint8_t* d_dst,
                                         uint16_t* d_ws, LzmaGpuResult* d_results,
                                         hipStream_t stream);
extern "C" int lzgpu_launch_session(LzgpuSession* d_sess, uint32_t n, hipStream_t stream);
// cooperative sessions: one 32-lane wave per session, tables of at most
// lds_cells cells staged in LDS for the call; max_groups 0 = one per session
extern "C" int lzgpu_launch_session_coop(LzgpuSession* d_sess, uint32_t n, uint32_t lds_cells,
                                         uint32_t max_groups, hipStream_t stream);
// lets a kernel launch with up to 160 KiB of dynamic LDS (once per kernel and
// device, thread-safe); 0 on success
int lzgpu_allow_full_lds(const void* kfn);
// largest table (cells) the cooperative session kernel stages in LDS: lc+lp <= 4
// at any pb (LZMA2's bound, 28 KiB) and wider LZMA tables up to 64 KiB
constexpr uint32_t kSessCoopMaxCells = 32768;
// Slot area of a lane-interleaved class (LZMA_GPU_PLAN_ILV): `off` cells into
// the workspace, `cells` rows of kIlv cells per lane group, room for `groups`
// workgroups.
struct LzgpuSlots {
  uint64_t off;
  uint32_t cells;
  uint32_t groups;
};
extern "C" int lzgpu_launch_decode_lds(const LzmaGpuStreamDesc* d_descs, const uint32_t* d_order,
                                       uint32_t n, const uint8_t* d_src, uint8_t* d_dst,
                                       uint16_t* d_ws, LzmaGpuResult* d_results, uint32_t lanes,
                                       uint32_t stride, uint32_t waves_per_simd,
                                       uint32_t groups_per_cu, uint32_t max_groups,
                                       uint32_t* d_queue, uint32_t lds_mask,
                                       uint32_t class_flags, LzgpuSlots slots,
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
extern "C" int lzgpu_launch_bra(uint32_t kind, uint8_t* d_data, const uint64_t* d_off,
                                const uint64_t* d_len, const uint32_t* d_ip, uint64_t* d_done,
                                uint32_t n, int encoding, hipStream_t stream);
extern "C" int lzgpu_launch_bcj2(const Bcj2GpuJob* d_jobs, uint32_t n, int32_t* d_res,
                                 hipStream_t stream);
extern "C" int lzgpu_launch_delta(uint8_t* d_data, const uint64_t* d_off, const uint64_t* d_len,
                                  const uint32_t* d_delta, uint8_t* d_state, uint32_t n,
                                  int encoding, hipStream_t stream);

// host-side helpers shared by the C-ABI translation units (lzma_capi.hip)
namespace lzgpu_host {

// LDS is given to a workgroup in whole blocks: 128 blocks of 1,280 bytes make a
// CU's 160 KiB (measured, profiles/r05_cfg5groups/: a launch padded to 160 KiB
// / 15 = 10,752 bytes per workgroup fitted 14 per CU, not 15 -- 9 blocks
// each).  Workgroup counts and the LDS padding that forces them are computed in
// blocks.
constexpr uint32_t kLdsBytesPerCu = 160u * 1024u;
constexpr uint32_t kLdsGrain = 1280u;
constexpr uint32_t kLdsBlocksPerCu = kLdsBytesPerCu / kLdsGrain;
inline uint32_t lds_blocks(size_t bytes) {
  return uint32_t((bytes + kLdsGrain - 1) / kLdsGrain);
}
// workgroups of `bytes` of LDS that fit a CU at once
inline uint32_t lds_groups_fit(size_t bytes) {
  const uint32_t b = lds_blocks(bytes);
  return b ? kLdsBlocksPerCu / b : 0xFFFFu;
}
// the most LDS each of `groups` workgroups can take with all of them resident
inline size_t lds_share(uint32_t groups) {
  return size_t(kLdsBlocksPerCu / (groups ? groups : 1u)) * kLdsGrain;
}
bool ensure_device();
void set_error(const char* what);
bool hip_ok(hipError_t e, const char* what);
// CUs of the current device once the library has started the HIP runtime
// (ensure_device), else MI355X's 256 without touching the runtime
uint32_t device_cus();

// host CRC-32 for container metadata (7zCrc.c semantics; headers, a few
// bytes per block -- decoded data is checked on the GPU)
inline uint32_t crc32_host(const uint8_t* p, size_t n) {
  static uint32_t t[256];
  static bool init = false;
  if (!init) {
    for (uint32_t v = 0; v < 256; ++v) {
      uint32_t r = v;
      for (int j = 0; j < 8; ++j) r = (r >> 1) ^ ((r & 1u) ? 0xEDB88320u : 0u);
      t[v] = r;
    }
    init = true;
  }
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) c = t[(c ^ p[i]) & 0xFFu] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

// Grow-only device buffer on one device (per-call scratch of the host-buffer
// entry points; pooled per device, see CallScratch).
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  void* get(size_t n) {
    if (n == 0) n = 16;
    if (p && cap >= n) return p;
    size_t want = n > cap * 2 ? n : cap * 2;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(&p, want) != hipSuccess) {
      (void)hipGetLastError();
      p = nullptr;
      if (hipMalloc(&p, n) != hipSuccess) {
        (void)hipGetLastError();
        p = nullptr;
        return nullptr;
      }
      want = n;
    }
    cap = want;
    return p;
  }
};

// Scratch of one host-buffer call (LzmaDecode, LzmaUncompress, the CRC
// drop-ins, ...): device buffers plus a non-blocking stream of its own, taken
// from a per-device pool for the call and returned after it.  The pool grows
// to the number of calls in flight at once, not to the number of threads that
// ever called (nothing is thread-local, nothing leaks per thread).
struct CallScratch {
  DevBuf buf[4];
  hipStream_t stream = nullptr;
  int dev = 0;
  uint8_t* pin = nullptr;  // pinned host staging (scratch_pinned)
  size_t pin_cap = 0;
};
CallScratch* scratch_acquire();  // current device; nullptr (error set) on failure
void scratch_release(CallScratch* s);
// The scratch's pinned host staging, at least n bytes (grown geometrically from
// 256 KiB, at most kPinnedStageMax); nullptr when n is larger or the allocation
// fails -- the caller then copies from / to pageable memory directly.  A
// pageable hipMemcpyAsync goes through the runtime's own staging buffer, one
// per device, so concurrent callers' small copies queue behind each other.
constexpr size_t kPinnedStageMax = size_t(8) << 20;
uint8_t* scratch_pinned(CallScratch* s, size_t n);

// owning device array for the container drivers' per-call buffers
template <class T>
struct DevArr {
  T* p = nullptr;
  DevArr() = default;
  DevArr(const DevArr&) = delete;
  DevArr& operator=(const DevArr&) = delete;
  ~DevArr() {
    if (p) (void)hipFree(p);
  }
  bool alloc(size_t n) { return hipMalloc(&p, (n ? n : 1) * sizeof(T)) == hipSuccess; }
};
}  // namespace lzgpu_host

extern "C" int lzgpu_launch_crc_decoded(const LzmaGpuStreamDesc* d_descs,
                                        const LzmaGpuResult* d_results, const uint8_t* d_dst,
                                        uint32_t n, const uint32_t* d_chunk_base,
                                        const uint32_t* d_chunk_range, uint32_t n_chunks,
                                        uint32_t* d_chunk_crc, uint32_t* d_crc,
                                        hipStream_t stream);

// traffic_calib.hip -- calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for
// the access shapes of the decode kernel (MI355X_MICROARCH.md: only 16-byte-per-
// lane streaming reads/writes are calibrated; other widths must be measured).
//
// Every kernel uses the decoder's layout: one lane per stream, lane l owning a
// window of W bytes at l * W (256 CUs x 8 workgroups x 32 lanes = 65,536
// windows of 4 KiB = 256 MiB, the config-3 batch), walking it front to back:
//   st1   1-byte stores              (literals)
//   st8u  8-byte stores at +3        (unaligned match copies)
//   st16  16-byte aligned stores     (the guide's calibrated case)
//   ld1   1-byte loads               (input bytes / dictionary reads)
//   ld16  16-byte aligned loads      (the input reader's refills)
// Run each under separate --pmc passes (FETCH_SIZE, WRITE_SIZE) plus a kernel
// trace; scripts/ubench/traffic_calib.py divides the counters by the bytes.
//
//   hipcc -O3 --offload-arch=gfx950 -o traffic_calib scripts/ubench/traffic_calib.hip
//   ./traffic_calib <kernel>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

constexpr unsigned kW = 4096;
constexpr unsigned kLanes = 32;
constexpr unsigned kGroups = 256 * 8;
constexpr size_t kBytes = size_t(kW) * kLanes * kGroups;

__global__ void __launch_bounds__(32) st1(unsigned char* d) {
  unsigned char* w = d + size_t(blockIdx.x * kLanes + threadIdx.x) * kW;
  for (unsigned i = 0; i < kW; ++i) w[i] = (unsigned char)(i ^ threadIdx.x);
}

__global__ void __launch_bounds__(32) st8u(unsigned char* d) {
  unsigned char* w = d + size_t(blockIdx.x * kLanes + threadIdx.x) * kW;
  // 8-byte stores at offset 3 mod 8 (the window's first 3 and last 5 bytes by bytes)
  for (unsigned i = 0; i < 3; ++i) w[i] = 1;
  for (unsigned i = 3; i + 8 <= kW; i += 8) {
    const unsigned long long v = 0x0101010101010101ull * (i & 0xFF);
    __builtin_memcpy(w + i, &v, 8);
  }
  for (unsigned i = kW - 5; i < kW; ++i) w[i] = 2;
}

__global__ void __launch_bounds__(32) st16(unsigned char* d) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  u32x4* w = (u32x4*)(d + size_t(blockIdx.x * kLanes + threadIdx.x) * kW);
  for (unsigned i = 0; i < kW / 16; ++i) w[i] = u32x4{i, i + 1, i + 2, threadIdx.x};
}

__global__ void __launch_bounds__(32) ld1(const unsigned char* d, unsigned* out) {
  const unsigned char* w = d + size_t(blockIdx.x * kLanes + threadIdx.x) * kW;
  unsigned acc = 0;
  for (unsigned i = 0; i < kW; ++i) acc = acc * 31 + w[i];
  out[blockIdx.x * kLanes + threadIdx.x] = acc;
}

__global__ void __launch_bounds__(32) ld16(const unsigned char* d, unsigned* out) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4* w = (const u32x4*)(d + size_t(blockIdx.x * kLanes + threadIdx.x) * kW);
  unsigned acc = 0;
  for (unsigned i = 0; i < kW / 16; ++i) {
    const u32x4 v = w[i];
    acc = acc * 31 + (v.x ^ v.y ^ v.z ^ v.w);
  }
  out[blockIdx.x * kLanes + threadIdx.x] = acc;
}

int main(int argc, char** argv) {
  const char* k = argc > 1 ? argv[1] : "st1";
  unsigned char* d = nullptr;
  unsigned* out = nullptr;
  if (hipMalloc(&d, kBytes) != hipSuccess || hipMalloc(&out, kLanes * kGroups * 4) != hipSuccess)
    return 2;
  hipMemset(d, 7, kBytes);
  // 2 untimed launches then 3 measured ones (the counters are per dispatch)
  for (int rep = 0; rep < 5; ++rep) {
    if (!strcmp(k, "st1")) hipLaunchKernelGGL(st1, dim3(kGroups), dim3(kLanes), 0, 0, d);
    else if (!strcmp(k, "st8u")) hipLaunchKernelGGL(st8u, dim3(kGroups), dim3(kLanes), 0, 0, d);
    else if (!strcmp(k, "st16")) hipLaunchKernelGGL(st16, dim3(kGroups), dim3(kLanes), 0, 0, d);
    else if (!strcmp(k, "ld1")) hipLaunchKernelGGL(ld1, dim3(kGroups), dim3(kLanes), 0, 0, d, out);
    else if (!strcmp(k, "ld16")) hipLaunchKernelGGL(ld16, dim3(kGroups), dim3(kLanes), 0, 0, d, out);
    else return 3;
  }
  if (hipDeviceSynchronize() != hipSuccess) return 4;
  printf("%s bytes_per_launch %zu\n", k, kBytes);
  hipFree(d);
  hipFree(out);
  return 0;
}

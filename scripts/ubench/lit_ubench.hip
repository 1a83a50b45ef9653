// Micro-benchmark (analysis only, not part of the product): cycles per plain
// literal (8-level tree in LDS) for code shapes of the range decoder, in the
// kernel's own launch shape (16 lanes per wave, 16 workgroups per CU).
//   hipcc -O3 --offload-arch=gfx950 -I../../lzma-sdk-zliblike_amd/csrc lit_ubench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
#include "lzma_device.h"
using namespace lzgpu;

constexpr int STRIDE = 256;

template <int V>
__global__ void __launch_bounds__(64, 4) lit_kernel(const uint8_t* src, uint32_t in_bytes,
                                                    uint8_t* dst, uint32_t n_lit,
                                                    uint32_t* sink, uint32_t slices) {
  extern __shared__ uint32_t smem[];
  lds_u16* lo = (lds_u16*)((uint16_t*)smem) + (threadIdx.x % slices) * STRIDE;
  for (int i = 0; i < 256; ++i) lo[i] = 1024;
  const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
  GlobalReader16 rd;
  rd.init((const gbyte*)(src + size_t(lane) * in_bytes), in_bytes);
  Rc<GlobalReader16> rc{0xFFFFFFFFu, 0, &rd};
  for (int k = 0; k < 4; ++k) rc.code = (rc.code << 8) | rd.next();
  gbyte* out = (gbyte*)(dst + size_t(lane) * n_lit);
  uint32_t acc = 0;
  uint64_t win = 0x0123456789ABCDEFull ^ lane;
  uint32_t range = rc.range, code = rc.code;
  for (uint32_t i = 0; i < n_lit; ++i) {
    uint32_t sym;
    if constexpr (V == 0 || V == 1) sym = rc.template tree<8>(lo);
    if constexpr (V >= 6) {
      // children-pair prefetch: the next level's two cells are read while
      // the current decision resolves (lo must be 4-byte aligned)
      uint32_t m = 1;
      uint32_t p = lo[1];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        uint32_t pair = 0;
        if (k < 7) pair = *wide(lo + 2 * m);
        if constexpr (V == 6) {
          const bool n = range < kTop;
          range = n ? range << 8 : range;
          code = n ? code << 8 : code;
        } else {
          if (range < kTop) {
            range <<= 8;
            code = (code << 8) | uint32_t(win & 0xFF);
            win = (win >> 8) | (win << 56);
          }
        }
        const uint32_t bound = (range >> 11) * p;
        const bool b = code >= bound;
        const int32_t mm = b ? 0 : int32_t(kProbOne - 31);
        lo[m] = uint16_t(int32_t(p) - ((int32_t(p) - mm) >> 5));
        range = b ? range - bound : bound;
        code = b ? code - bound : code;
        m = (m << 1) | (b ? 1u : 0u);
        if (k < 7) p = b ? (pair >> 16) : (pair & 0xFFFFu);
      }
      sym = m;
    } else if constexpr (V >= 2) {
      uint32_t m = 1;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if constexpr (V == 2) {  // normalize with a zero byte, branch-free
          const bool n = range < kTop;
          range = n ? range << 8 : range;
          code = n ? code << 8 : code;
        } else if constexpr (V == 3) {  // branch-free, byte from a 64-bit window
          const bool n = range < kTop;
          range = n ? range << 8 : range;
          code = n ? ((code << 8) | uint32_t(win & 0xFF)) : code;
          win = n ? (win >> 8) | (win << 56) : win;
        } else if constexpr (V == 4) {  // branchy, window, no refill check
          if (range < kTop) {
            range <<= 8;
            code = (code << 8) | uint32_t(win & 0xFF);
            win = (win >> 8) | (win << 56);
          }
        } else if constexpr (V == 5) {  // branch-free, 32-bit rotating window
          const bool n = range < kTop;
          range = n ? range << 8 : range;
          const uint32_t w = uint32_t(win);
          code = n ? ((code << 8) | (w & 0xFF)) : code;
          win = n ? uint64_t(__builtin_rotateright32(w, 8)) : win;
        }
        const uint32_t p = lo[m];
        const uint32_t bound = (range >> 11) * p;
        const bool b = code >= bound;
        const int32_t mm = b ? 0 : int32_t(kProbOne - 31);
        lo[m] = uint16_t(int32_t(p) - ((int32_t(p) - mm) >> 5));
        range = b ? range - bound : bound;
        code = b ? code - bound : code;
        m = (m << 1) | (b ? 1u : 0u);
      }
      sym = m;
    }
    if constexpr (V == 0) out[i] = uint8_t(sym);
    if constexpr (V >= 1) acc += sym;
  }
  acc += range + code;
  if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char** argv) {
  const int cus = 256;
  const uint32_t n_lit = 1000, in_bytes = 2048, max_lanes = cus * 16 * 64;
  std::vector<uint8_t> h(size_t(max_lanes) * in_bytes);
  srand(1);
  for (auto& b : h) b = uint8_t(rand());
  uint8_t *src, *dst;
  uint32_t* sink;
  (void)hipMalloc(&src, h.size());
  (void)hipMalloc(&dst, size_t(max_lanes) * n_lit);
  (void)hipMalloc(&sink, 64);
  (void)hipMemcpy(src, h.data(), h.size(), hipMemcpyHostToDevice);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  auto run = [&](auto kfn, const char* name, int lanes, int gpc) {
    (void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    const size_t lds = 160 * 1024 / gpc;
    const uint32_t slices = std::min<uint32_t>(lanes, lds / (STRIDE * 2));
    for (int r = 0; r < 3; ++r) {
      (void)hipEventRecord(a);
      hipLaunchKernelGGL(kfn, dim3(cus * gpc), dim3(lanes), lds, 0, src, in_bytes, dst, n_lit,
                         sink, slices);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      if (r == 2) {
        const double cyc = ms * 1e-3 * 2.4e9 / n_lit / 8;
        printf("%-28s lanes %2d x %2d WG/CU (%d waves/SIMD, %u slices): %7.1f cyc/decision/wave, "
               "%.3f lane-decisions/SIMD-cycle\n",
               name, lanes, gpc, (gpc + 3) / 4, slices, cyc, lanes * gpc / 4.0 / cyc);
      }
    }
  };
  const int shapes[][2] = {{32, 8}, {16, 16}, {32, 4}};
  for (auto& sh : shapes) {
    run(lit_kernel<1>, "tree<8> (product code)", sh[0], sh[1]);
    run(lit_kernel<2>, "norm zero-byte branch-free", sh[0], sh[1]);
    run(lit_kernel<4>, "norm win64 branchy", sh[0], sh[1]);
    run(lit_kernel<5>, "norm win32 branch-free", sh[0], sh[1]);
    run(lit_kernel<6>, "zero-byte + pair prefetch", sh[0], sh[1]);
    run(lit_kernel<7>, "win64 branchy + pair prefetch", sh[0], sh[1]);
  }
  return 0;
}

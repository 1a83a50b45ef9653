// Micro-benchmark (analysis only, not part of the product): the issue and
// latency constants the decision-level loop design depends on (DESIGN.md §3,
// round 4), measured in the throughput kernel's launch shape.
//   hipcc -O3 --offload-arch=gfx950 -o issue_ubench issue_ubench.hip
// Every test launches W one-wave workgroups per SIMD (4W per CU, 256 CUs),
// each wave with `lanes` active lanes, and reports the median over waves of
// s_memtime cycles per loop step.
//   valu_ilp : 4 independent v_add chains, 16 adds per step
//   valu_dep : one dependent v_add chain, 16 adds per step
//   lds_dep  : dependent ds_read_u16 chain (address from the loaded value)
//   gl_dep   : dependent global_load_ushort chain over an L2-resident table
//   st_gl    : global_store_byte, then a global load of another (L2-hot)
//              address consumed in the same step -- the in-order vmcnt queue
//              makes the load wait for the store's acknowledgement
//   st_gl_far: the same, the load issued 4 steps before it is consumed
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CHECK(x)                                                        \
  do {                                                                  \
    hipError_t e_ = (x);                                                \
    if (e_ != hipSuccess) {                                             \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
      exit(1);                                                          \
    }                                                                   \
  } while (0)

constexpr int kSteps = 512;

template <int T>
__global__ void __launch_bounds__(64) bench_kernel(uint32_t lanes, uint64_t* cyc,
                                                   const uint16_t* __restrict__ tab,
                                                   uint8_t* __restrict__ out, uint32_t* sink) {
  __shared__ uint16_t lt[4096];
  for (int i = threadIdx.x; i < 4096; i += 64) lt[i] = uint16_t((i * 97 + 13) & 4095);
  __syncthreads();
  uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7;
  uint64_t t0 = 0, t1 = 0;
  if (threadIdx.x < lanes) {
    t0 = __builtin_amdgcn_s_memtime();
    if constexpr (T == 0) {
      for (int s = 0; s < kSteps; ++s) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          asm volatile("v_add_u32 %0, %0, 1\n v_add_u32 %1, %1, 1\n v_add_u32 %2, %2, 1\n v_add_u32 %3, %3, 1"
                       : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
        }
      }
    } else if constexpr (T == 1) {
      for (int s = 0; s < kSteps; ++s) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          asm volatile("v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, 1"
                       : "+v"(a0));
        }
      }
    } else if constexpr (T == 2) {
      uint32_t i = a0 & 4095;
      for (int s = 0; s < kSteps; ++s) i = lt[i];
      a0 = i;
    } else if constexpr (T == 3) {
      uint32_t i = (a0 * 16) & 65535;
      for (int s = 0; s < kSteps; ++s) i = tab[i] * 16u + (threadIdx.x & 15);
      a0 = i;
    } else if constexpr (T == 4) {
      uint32_t i = (a0 * 16) & 65535;
      uint8_t* o = out + (size_t(blockIdx.x) * 64 + threadIdx.x) * kSteps;
      for (int s = 0; s < kSteps; ++s) {
        o[s] = uint8_t(i);
        i = tab[(i + s) & 65535] * 16u + (threadIdx.x & 15);
      }
      a0 = i;
    } else if constexpr (T == 5) {
      // loads issued 4 steps ahead of use, one store per step
      uint8_t* o = out + (size_t(blockIdx.x) * 64 + threadIdx.x) * kSteps;
      uint32_t q0 = tab[a0 & 65535], q1 = tab[(a0 + 1) & 65535], q2 = tab[(a0 + 2) & 65535],
               q3 = tab[(a0 + 3) & 65535];
      uint32_t acc = 0;
      for (int s = 0; s < kSteps; s += 4) {
        o[s] = uint8_t(acc);
        acc += q0;
        q0 = tab[(acc + s) & 65535];
        o[s + 1] = uint8_t(acc);
        acc += q1;
        q1 = tab[(acc + s + 1) & 65535];
        o[s + 2] = uint8_t(acc);
        acc += q2;
        q2 = tab[(acc + s + 2) & 65535];
        o[s + 3] = uint8_t(acc);
        acc += q3;
        q3 = tab[(acc + s + 3) & 65535];
      }
      a0 = acc;
    }
    t1 = __builtin_amdgcn_s_memtime();
  }
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  if (a0 + a1 + a2 + a3 == 0x12345678u) sink[0] = 1;
}

template <int T>
static double run(int W, uint32_t lanes, const uint16_t* tab, uint8_t* out, uint32_t* sink,
                  uint64_t* d_cyc) {
  const int grid = 256 * 4 * W;
  hipLaunchKernelGGL(bench_kernel<T>, dim3(grid), dim3(64), 0, 0, lanes, d_cyc, tab, out, sink);
  CHECK(hipDeviceSynchronize());
  hipLaunchKernelGGL(bench_kernel<T>, dim3(grid), dim3(64), 0, 0, lanes, d_cyc, tab, out, sink);
  CHECK(hipDeviceSynchronize());
  std::vector<uint64_t> c(grid);
  CHECK(hipMemcpy(c.data(), d_cyc, grid * 8, hipMemcpyDeviceToHost));
  std::sort(c.begin(), c.end());
  return double(c[grid / 2]) / kSteps;
}

int main() {
  uint16_t* tab;
  uint8_t* out;
  uint32_t* sink;
  uint64_t* cyc;
  CHECK(hipMalloc(&tab, 65536 * 2 + 64));
  std::vector<uint16_t> h(65536);
  for (int i = 0; i < 65536; ++i) h[i] = uint16_t((i * 2654435761u) >> 20) & 4095;
  CHECK(hipMemcpy(tab, h.data(), 65536 * 2, hipMemcpyHostToDevice));
  CHECK(hipMalloc(&out, size_t(256) * 4 * 8 * 64 * kSteps));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMalloc(&cyc, 256 * 4 * 8 * 8));
  const char* names[] = {"valu_ilp(16 adds)", "valu_dep(16 adds)", "lds_dep", "gl_dep",
                         "st_gl", "st_gl_far"};
  for (int t = 0; t < 6; ++t)
    for (int W : {1, 2, 4, 8})
      for (uint32_t lanes : {16u, 32u, 64u}) {
        double v = 0;
        switch (t) {
          case 0: v = run<0>(W, lanes, tab, out, sink, cyc); break;
          case 1: v = run<1>(W, lanes, tab, out, sink, cyc); break;
          case 2: v = run<2>(W, lanes, tab, out, sink, cyc); break;
          case 3: v = run<3>(W, lanes, tab, out, sink, cyc); break;
          case 4: v = run<4>(W, lanes, tab, out, sink, cyc); break;
          case 5: v = run<5>(W, lanes, tab, out, sink, cyc); break;
        }
        printf("{\"test\": \"%s\", \"waves_per_simd\": %d, \"lanes\": %u, \"cycles_per_step\": %.1f}\n",
               names[t], W, lanes, v);
        fflush(stdout);
      }
  return 0;
}

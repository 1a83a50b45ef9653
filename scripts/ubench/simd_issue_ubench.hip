// Micro-benchmark (analysis only, not part of the product): the rate at which
// ONE SIMD issues instructions for 1, 2, 4 and 8 co-resident waves, timed over
// the whole kernel (the round-4 issue roofline priced a
// SIMD at one wave64 VALU per 4 cycles, from per-wave s_memtime medians that
// cannot see what co-resident waves get).
//   hipcc -O3 --offload-arch=gfx950 -o simd_issue_ubench simd_issue_ubench.hip
//
// Every launch puts W one-wave workgroups on each SIMD of every CU (grid =
// CUs x 4 x W, all resident at once), each wave with `lanes` active lanes.
// A test runs N and 2N loop iterations; the difference of the two kernel
// durations (HIP events) over the difference of the wave-instructions issued
// chip-wide gives the sustained rate with launch and ramp costs cancelled:
//   issue_per_simd_cycle = d(wave-instructions) / (d(seconds) * clock * SIMDs)
// `clock` is measured in the same run: the median wave's s_memtime cycles
// (shader clock, MI355X_MICROARCH.md "s_memtime tick") of the 2N launch minus
// the N launch's, over the difference of their durations.
//   valu_ilp8  : 8 independent v_add_u32 chains (64 per iteration)
//   valu_dep   : one dependent v_add_u32 chain (64 per iteration)
//   salu_ilp8  : 8 independent s_add_u32 chains (64 per iteration)
//   mix_vs     : 4 v_add + 4 s_add chains interleaved (64 per iteration)
//   dec_lds    : the LZMA range-coder decision of the decoder (LzmaDec.c:
//                8-45: prob load, bound, compare, update, range/code select,
//                next node) as a dependent chain through an LDS bit tree;
//                reported as cycles per decision per wave and decisions per
//                SIMD-cycle
//   dec_glb    : the same with the tree in global memory (L2-resident)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <string>
#include <vector>

#define CHECK(x)                                              \
  do {                                                        \
    hipError_t e_ = (x);                                      \
    if (e_ != hipSuccess) {                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
      exit(1);                                                \
    }                                                         \
  } while (0)

constexpr int kPerIter = 64;  // instructions (or decisions / 8) per loop iteration

// per-wave record of the occupancy check (rec != nullptr): shader-clock and
// constant 100 MHz stamps at the start and end of the timed loop, HW_ID and
// XCC_ID -- which SIMD of which CU the wave ran on, and with whom at once
struct WaveRec {
  uint64_t t0, t1, r0, r1;
  uint32_t hw_id, xcc_id;
};

template <int T>
__global__ void __launch_bounds__(64) ub_kernel(uint32_t lanes, uint32_t iters, uint64_t* cyc,
                                                const uint16_t* __restrict__ tab,
                                                uint32_t* __restrict__ sink,
                                                WaveRec* __restrict__ rec) {
  __shared__ uint16_t lt[2048];  // 4 KiB: 32 workgroups per CU fit (W = 8)
  for (int i = threadIdx.x; i < 2048; i += 64) lt[i] = uint16_t(200 + ((i * 2654435761u) >> 21) % 1600);
  __syncthreads();
  uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 + 11, a5 = a0 + 13,
           a6 = a0 + 17, a7 = a0 + 19;
  uint64_t t0 = 0, t1 = 0, r0 = 0, r1 = 0;
  if (threadIdx.x < lanes) {
    r0 = __builtin_amdgcn_s_memrealtime();
    t0 = __builtin_amdgcn_s_memtime();
    if constexpr (T == 0) {
      for (uint32_t s = 0; s < iters; ++s) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
          asm volatile(
              "v_add_u32 %0, %0, 1\n v_add_u32 %1, %1, 1\n v_add_u32 %2, %2, 1\n v_add_u32 %3, %3, 1\n"
              "v_add_u32 %4, %4, 1\n v_add_u32 %5, %5, 1\n v_add_u32 %6, %6, 1\n v_add_u32 %7, %7, 1"
              : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
      }
    } else if constexpr (T == 1) {
      for (uint32_t s = 0; s < iters; ++s) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
          asm volatile(
              "v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, 1\n"
              "v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, 1\n v_add_u32 %0, %0, 1"
              : "+v"(a0));
      }
    } else if constexpr (T == 2) {
      uint32_t s0 = 1, s1 = 2, s2 = 3, s3 = 4, s4 = 5, s5 = 6, s6 = 7, s7 = 8;
      for (uint32_t s = 0; s < iters; ++s) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
          asm volatile(
              "s_add_u32 %0, %0, 1\n s_add_u32 %1, %1, 1\n s_add_u32 %2, %2, 1\n s_add_u32 %3, %3, 1\n"
              "s_add_u32 %4, %4, 1\n s_add_u32 %5, %5, 1\n s_add_u32 %6, %6, 1\n s_add_u32 %7, %7, 1"
              : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(s4), "+s"(s5), "+s"(s6), "+s"(s7)
              :
              : "scc");
      }
      a0 += s0 + s1 + s2 + s3 + s4 + s5 + s6 + s7;
    } else if constexpr (T == 3) {
      uint32_t s0 = 1, s1 = 2, s2 = 3, s3 = 4;
      for (uint32_t s = 0; s < iters; ++s) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
          asm volatile(
              "v_add_u32 %0, %0, 1\n s_add_u32 %4, %4, 1\n v_add_u32 %1, %1, 1\n s_add_u32 %5, %5, 1\n"
              "v_add_u32 %2, %2, 1\n s_add_u32 %6, %6, 1\n v_add_u32 %3, %3, 1\n s_add_u32 %7, %7, 1"
              : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3)
              :
              : "scc");
      }
      a0 += s0 + s1 + s2 + s3;
    } else {
      // range-coder decisions (the shared-form update of lzma_device.h Rc::bit)
      uint32_t range = 0xFFFFFFFFu, code = (threadIdx.x * 0x9E3779B9u) >> 1;
      uint32_t m = 1, w = threadIdx.x * 0x85EBCA6Bu;
      for (uint32_t s = 0; s < iters; ++s) {
#pragma unroll
        for (int k = 0; k < kPerIter / 8; ++k) {
          uint32_t p;
          if constexpr (T == 4)
            p = lt[m];
          else
            p = tab[m];
          if (range < (1u << 24)) {  // NORMALIZE from a register "input"
            range <<= 8;
            code = (code << 8) | (w & 0xFFu);
            w = (w >> 8) | (w << 24);
          }
          const uint32_t bound = (range >> 11) * p;
          const bool b = code >= bound;
          const int32_t mm = b ? 0 : int32_t(2048 - 31);
          const uint16_t np = uint16_t(int32_t(p) - ((int32_t(p) - mm) >> 5));
          if constexpr (T == 4)
            lt[m] = np;
          else
            ((uint16_t*)tab)[m] = np;
          range = b ? range - bound : bound;
          code = b ? code - bound : code;
          m = (m << 1) | (b ? 1u : 0u);
          m = m >= 2048u ? 1u : m;
        }
      }
      a0 = m + range + code;
    }
    t1 = __builtin_amdgcn_s_memtime();
    r1 = __builtin_amdgcn_s_memrealtime();
  }
  if (threadIdx.x == 0) {
    cyc[blockIdx.x] = t1 - t0;
    if (rec) {
      // hwreg(HW_REG_HW_ID) and hwreg(HW_REG_XCC_ID), whole registers
      rec[blockIdx.x] = WaveRec{t0, t1, r0, r1, __builtin_amdgcn_s_getreg((31 << 11) | 4),
                                __builtin_amdgcn_s_getreg((31 << 11) | 20)};
    }
  }
  if (a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 == 0x12345678u) sink[0] = 1;
}

struct Res {
  double ms, med_cyc;
};

template <int T>
static Res run(int grid, uint32_t lanes, uint32_t iters, uint16_t* tab, uint32_t* sink,
               uint64_t* d_cyc) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(ub_kernel<T>, dim3(grid), dim3(64), 0, 0, lanes, iters, d_cyc, tab, sink,
                     (WaveRec*)nullptr);
  CHECK(hipDeviceSynchronize());
  double best = 1e30;
  std::vector<uint64_t> c(grid), keep;
  for (int r = 0; r < 3; ++r) {
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(ub_kernel<T>, dim3(grid), dim3(64), 0, 0, lanes, iters, d_cyc, tab, sink,
                       (WaveRec*)nullptr);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) {
      best = ms;
      CHECK(hipMemcpy(c.data(), d_cyc, grid * 8, hipMemcpyDeviceToHost));
      keep = c;
    }
  }
  std::sort(keep.begin(), keep.end());
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return {best, double(keep[grid / 2])};
}

template <int T>
static void test(const char* name, int cus, int W, uint32_t lanes, uint32_t iters, uint16_t* tab,
                 uint32_t* sink, uint64_t* cyc) {
  const int grid = cus * 4 * W;
  const Res a = run<T>(grid, lanes, iters, tab, sink, cyc);
  const Res b = run<T>(grid, lanes, 2 * iters, tab, sink, cyc);
  const double dsec = (b.ms - a.ms) * 1e-3;
  const double clock = (b.med_cyc - a.med_cyc) / dsec;  // shader cycles per second (slope)
  const int per_iter = T >= 4 ? kPerIter / 8 : kPerIter;
  const double dinst = double(grid) * iters * per_iter;  // wave-instructions (or decisions)
  const double per_simd_cycle = dinst / (dsec * clock * cus * 4);
  // cycles one wave takes per instruction (decision), from the slope
  const double wave_cyc = (b.med_cyc - a.med_cyc) / (double(iters) * per_iter);
  printf("{\"test\": \"%s\", \"waves_per_simd\": %d, \"lanes\": %u, \"iters\": %u, "
         "\"ms_N\": %.4f, \"ms_2N\": %.4f, \"clock_ghz\": %.3f, "
         "\"per_simd_cycle\": %.4f, \"simd_cycles_per_inst\": %.3f, \"wave_cycles_per_inst\": %.2f}\n",
         name, W, lanes, iters, a.ms, b.ms, clock * 1e-9, per_simd_cycle, 1.0 / per_simd_cycle,
         wave_cyc);
  fflush(stdout);
}

// Occupancy check: one launch of test T with per-wave records; reports the
// shader clock (memtime cycles over the 100 MHz realtime span) and how many
// waves shared a SIMD at once (the maximum over SIMDs of overlapping
// [r0, r1) spans), i.e. whether W waves per SIMD were really co-resident.
template <int T>
static void occupancy(const char* name, int cus, int W, uint32_t lanes, uint32_t iters,
                      uint16_t* tab, uint32_t* sink, uint64_t* cyc) {
  const int grid = cus * 4 * W;
  WaveRec* d_rec;
  CHECK(hipMalloc(&d_rec, size_t(grid) * sizeof(WaveRec)));
  hipLaunchKernelGGL(ub_kernel<T>, dim3(grid), dim3(64), 0, 0, lanes, iters, cyc, tab, sink, d_rec);
  CHECK(hipDeviceSynchronize());
  std::vector<WaveRec> r(grid);
  CHECK(hipMemcpy(r.data(), d_rec, grid * sizeof(WaveRec), hipMemcpyDeviceToHost));
  CHECK(hipFree(d_rec));
  std::vector<double> clk;
  uint64_t rmin = ~0ull, rmax = 0;
  for (const WaveRec& w : r) {
    if (w.r1 > w.r0) clk.push_back(double(w.t1 - w.t0) / (double(w.r1 - w.r0) / 100e6));
    rmin = std::min(rmin, w.r0);
    rmax = std::max(rmax, w.r1);
  }
  std::sort(clk.begin(), clk.end());
  // SIMD key: XCC, SE, SH, CU, SIMD fields of HW_ID (gfx9 layout)
  std::vector<std::pair<uint64_t, int>> ev;  // (time, +1/-1) per SIMD key
  std::vector<std::pair<uint32_t, std::pair<uint64_t, int>>> evk;
  for (const WaveRec& w : r) {
    const uint32_t key = ((w.xcc_id & 0xF) << 16) | (((w.hw_id >> 13) & 7) << 12) |
                         (((w.hw_id >> 12) & 1) << 11) | (((w.hw_id >> 8) & 0xF) << 4) |
                         ((w.hw_id >> 4) & 3);
    evk.push_back({key, {w.r0, +1}});
    evk.push_back({key, {w.r1, -1}});
  }
  std::sort(evk.begin(), evk.end(), [](const auto& a, const auto& b) {
    if (a.first != b.first) return a.first < b.first;
    if (a.second.first != b.second.first) return a.second.first < b.second.first;
    return a.second.second < b.second.second;  // ends before starts at equal times
  });
  int best = 0, cur = 0, simds = 0;
  uint32_t last = ~0u;
  for (const auto& e : evk) {
    if (e.first != last) {
      last = e.first;
      cur = 0;
      ++simds;
    }
    cur += e.second.second;
    best = std::max(best, cur);
  }
  printf("{\"occupancy\": \"%s\", \"waves_per_simd\": %d, \"lanes\": %u, \"simds_seen\": %d, "
         "\"max_coresident_per_simd\": %d, \"clock_ghz_median\": %.3f, \"clock_ghz_min\": %.3f, "
         "\"span_us\": %.1f}\n",
         name, W, lanes, simds, best, clk[clk.size() / 2] * 1e-9, clk.front() * 1e-9,
         double(rmax - rmin) / 100.0);
  fflush(stdout);
}

int main(int argc, char** argv) {
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  uint16_t* tab;
  uint32_t* sink;
  uint64_t* cyc;
  CHECK(hipMalloc(&tab, 4096 * 2 * 2));
  std::vector<uint16_t> h(4096);
  for (int i = 0; i < 4096; ++i) h[i] = uint16_t(200 + ((i * 2654435761u) >> 21) % 1600);
  CHECK(hipMemcpy(tab, h.data(), 4096 * 2, hipMemcpyHostToDevice));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMalloc(&cyc, size_t(cus) * 4 * 8 * 8));
  fprintf(stderr, "CUs %d\n", cus);
  if (argc > 1 && std::string(argv[1]) == "lanes") {
    // active lanes per wave: does a wave with one active lane issue slower?
    for (int W : {1, 2, 4})
      for (uint32_t lanes : {1u, 2u, 4u, 8u, 16u, 32u}) {
        test<0>("valu_ilp8", cus, W, lanes, 2000, tab, sink, cyc);
        test<2>("salu_ilp8", cus, W, lanes, 2000, tab, sink, cyc);
        test<4>("dec_lds", cus, W, lanes, 200, tab, sink, cyc);
      }
    return 0;
  }
  for (int W : {1, 2, 4, 8}) {
    occupancy<0>("valu_ilp8", cus, W, 64, 20000, tab, sink, cyc);
    occupancy<4>("dec_lds", cus, W, 32, 2000, tab, sink, cyc);
  }
  for (int W : {1, 2, 4, 8})
    for (uint32_t lanes : {1u, 32u, 64u}) {
      test<0>("valu_ilp8", cus, W, lanes, 2000, tab, sink, cyc);
      test<1>("valu_dep", cus, W, lanes, 1000, tab, sink, cyc);
      test<2>("salu_ilp8", cus, W, lanes, 2000, tab, sink, cyc);
      test<3>("mix_vs", cus, W, lanes, 2000, tab, sink, cyc);
    }
  // decisions: a dependent chain per wave (no ILP inside a wave); the
  // decision test's "instructions" are decisions (8 per loop body x 8)
  for (int W : {1, 2, 4, 8})
    for (uint32_t lanes : {1u, 32u}) {
      test<4>("dec_lds", cus, W, lanes, 200, tab, sink, cyc);
      test<5>("dec_glb", cus, W, lanes, 50, tab, sink, cyc);
    }
  return 0;
}

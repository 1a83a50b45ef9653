// fuzz_containers.cpp -- TEST INFRASTRUCTURE ONLY (libFuzzer target).
//
// The host-side parsers of liblzmagpu.so that read untrusted bytes -- the 7z
// header walk (LzmaGpu_7zOpen, restating 7zIn.c:1214-1320), the xz backward
// index (LzmaGpu_XzIndex, XzIn.c:141-306), the LZMA2 chunk-header splitter
// (Lzma2Gpu_SplitBlocks) and the batch planner over arbitrary descriptors --
// built from the product sources with host AddressSanitizer + UBSan
// (tests/fuzz/Makefile; device code is not instrumented and never runs: the
// fuzzer runs in the CPU container, where every decode entry returns
// SZ_ERROR_FAIL before touching a device).  The first input byte picks the
// parser.
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../../include/lzma_gpu.h"

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  if (size < 1) return 0;
  const uint8_t sel = data[0] % 4;
  const uint8_t* p = data + 1;
  const size_t n = size - 1;
  switch (sel) {
    case 0: {  // 7z: open with and without output arrays
      size_t nfo = 0, nfi = 0, nn = 0;
      UInt64 total = 0;
      SRes r = LzmaGpu_7zOpen(p, n, nullptr, 0, &nfo, nullptr, 0, &nfi, nullptr, 0, &nn, &total);
      if (r == SZ_OK && nfo < 4096 && nfi < 65536 && nn < (1u << 20)) {
        std::vector<LzmaGpu7zFolder> fo(nfo + 1);
        std::vector<LzmaGpu7zFile> fi(nfi + 1);
        std::vector<UInt16> names(nn + 1);
        LzmaGpu_7zOpen(p, n, fo.data(), nfo, &nfo, fi.data(), nfi, &nfi, names.data(), nn, &nn,
                       &total);
      }
      break;
    }
    case 1: {  // xz: index twice (count, then fill)
      size_t nb = 0;
      uint64_t total = 0;
      if (LzmaGpu_XzIndex(p, n, nullptr, 0, &nb, &total) == SZ_OK && nb < (1u << 16)) {
        std::vector<LzmaGpuXzBlock> b(nb + 1);
        LzmaGpu_XzIndex(p, n, b.data(), nb, &nb, &total);
      }
      break;
    }
    case 2: {  // LZMA2 chunk headers
      uint64_t o[64], l[64], u[64];
      Lzma2Gpu_SplitBlocks(p, n, o, l, u, 64);
      break;
    }
    default: {  // the planner over arbitrary descriptors (48 bytes each)
      const size_t k = n / sizeof(LzmaGpuStreamDesc);
      if (k == 0 || k > 4096) break;
      std::vector<LzmaGpuStreamDesc> d(k);
      memcpy(d.data(), p, k * sizeof(LzmaGpuStreamDesc));
      std::vector<uint32_t> order(k);
      LzmaGpuPlan plan;
      LzmaGpuPlanOptions opt;
      memset(&opt, 0, sizeof opt);
      opt.kernel = p[0] % 5;
      opt.cus = 1 + p[n - 1] % 300;
      LzmaGpu_PlanBatchOpt(d.data(), k, order.data(), &plan, &opt);
      LzmaGpu_PlanBatch(d.data(), k, order.data());
      break;
    }
  }
  return 0;
}

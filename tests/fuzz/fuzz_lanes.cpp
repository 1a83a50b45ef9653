// fuzz_lanes.cpp -- TEST INFRASTRUCTURE ONLY (libFuzzer target).
//
// The kernels' per-lane code (lzma_lane.h, bcj2_device.h, bcj_device.h,
// bra_device.h) built for the host (-DLZGPU_HOST_EMU, the same build the CPU
// tests use) with AddressSanitizer + UBSan, fed arbitrary bytes: one LZMA
// stream (props, capacity and finish mode from the input) through the generic
// and the LDS-placement lanes, one LZMA2 range, BCJ2 over four streams cut
// from the input, x86 BCJ (lane-serial and tiled) and the RISC converters.
// Output buffers are exactly sized and inputs padded only to the 16-byte
// blocks the readers load, so an out-of-bounds read or write in the
// decoder's handling of corrupt input is reported.
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../lzma-sdk-zliblike_amd/csrc/lzma_lane.h"  // first: the host-emulation macros
#include "../../lzma-sdk-zliblike_amd/csrc/bcj2_device.h"
#include "../../lzma-sdk-zliblike_amd/csrc/bcj_device.h"
#include "../../lzma-sdk-zliblike_amd/csrc/bra_device.h"

using namespace lzgpu;

static uint32_t rd32(const uint8_t* p) {
  return uint32_t(p[0]) | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 24);
}

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  if (size < 12) return 0;
  const uint8_t sel = data[0] % 5;
  const uint32_t cap = rd32(data + 1) % (1u << 18);
  const uint8_t fin = data[5] & 1;
  const uint8_t* p = data + 6;
  const size_t n = size - 6;
  switch (sel) {
    case 0:
    case 1: {  // LZMA: props = first 5 bytes, stream = the rest (exact-size buffers)
      if (n < 5) break;
      LzmaGpuStreamDesc d;
      memset(&d, 0, sizeof d);
      memcpy(d.props, p, 5);
      d.props_size = 5;
      d.finish_mode = fin;
      d.kind = sel == 0 ? LZMA_GPU_KIND_LZMA : LZMA_GPU_KIND_LZMA2;
      d.src_len = n - 5;
      d.dst_cap = cap;
      // the input readers load aligned 16-byte blocks that hold a valid byte
      // (device allocations are 256-byte granular, so never unmapped there):
      // the source buffer is padded to a whole block, the output is exact
      std::vector<uint8_t> src(((n - 5) + 15) & ~size_t(15), 0);
      memcpy(src.data(), p + 5, n - 5);
      std::vector<uint8_t> dst(cap ? cap : 1);
      uint32_t plc, plp, ppb, pdict;
      uint32_t cells = 64;
      if (d.kind == LZMA_GPU_KIND_LZMA2)
        cells = table_cells(4, 0, 4);
      else if (lz_props_parse(d.props, 5, plc, plp, ppb, pdict) == kOk)
        cells = table_cells(plc, plp, ppb);
      std::vector<uint16_t> ws(cells + 64);
      d.probs_off = 0;
      LzmaGpuResult r = lane_decode(d, src.data(), dst.data(), ws.data());
      if (r.dest_len > cap || r.src_len > d.src_len) abort();
      // the LDS-placement lane (the throughput kernel's code) on a slice of
      // exactly the planner's width
      uint32_t lc, lp, pb, dict;
      uint32_t w = 0;
      if (d.kind == LZMA_GPU_KIND_LZMA2)
        w = lzma2_lds_cells(LZGPU_LDS_MASK);
      else if (lz_props_parse(d.props, 5, lc, lp, pb, dict) == kOk)
        w = make_layout(lc, lp, pb, LZGPU_LDS_MASK).lds_cells;
      if (w && w <= 16384) {
        std::vector<uint16_t> lds(w);
        LzmaGpuResult r2 = lane_decode_lds<LZGPU_LDS_MASK, true>(d, src.data(), dst.data(),
                                                                  ws.data(), lds.data(), w);
        if (r2.res != r.res || r2.status != r.status || r2.dest_len != r.dest_len ||
            r2.src_len != r.src_len)
          abort();  // the two lanes disagree
      }
      break;
    }
    case 2: {  // BCJ2: four streams cut from the input
      const size_t a = n / 4;
      std::vector<uint8_t> s0(p, p + a), s1(p + a, p + 2 * a), s2(p + 2 * a, p + 3 * a),
          s3(p + 3 * a, p + n);
      std::vector<uint8_t> out(cap % 65536 + 1);
      uint16_t probs[258];
      bcj2_decode(s0.data(), s0.size(), s1.data(), s1.size(), s2.data(), s2.size(), s3.data(),
                  s3.size(), out.data(), uint64_t(out.size()), probs);
      break;
    }
    case 3: {  // x86 BCJ (the window loads 16-byte blocks: the buffer is padded to 16)
      std::vector<uint8_t> b((n + 15) & ~size_t(15), 0);
      memcpy(b.data(), p, n);
      uint32_t st = data[5] & 7;
      bcj_x86(b.data(), n, rd32(data + 1), &st, data[5] >> 7);
      break;
    }
    default: {  // RISC converters
      std::vector<uint8_t> b(p, p + n);
      const uint32_t kind = kBraPPC + data[5] % 5;  // PPC, IA64, ARM, ARMT, SPARC
      const uint64_t units = bra_done_units(kind, n);
      const uint32_t u = bra_unit(kind);
      for (uint64_t k = 0; k < units; ++k)
        bra_unit_convert(kind, b.data() + k * u, rd32(data + 1) + uint32_t(k * u), 0);
      break;
    }
  }
  return 0;
}

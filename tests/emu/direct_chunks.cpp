// TEST INFRASTRUCTURE: direct_coop (lzma_device.h, the cooperative kernel's
// direct bits several per step) against the bit-serial loop of the reference
// (LzmaDec.c:323-344, here Rc::direct) on random well-formed and corrupt
// (code >= range) range-coder states: the host-emulation branch and a
// lane-by-lane model of the device branch (32 lanes' S(j), the ballot, the
// readlane).  Exit status 0 = every case bit-exact (range, code, distance bits,
// input bytes consumed).  Usage: direct_chunks [cases]
#define LZGPU_HOST_EMU 1
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include "lzma_device.h"
using namespace lzgpu;
struct ArrRd {
  const uint8_t* p; uint32_t i = 0;
  uint32_t next() { return p[i++]; }
};
// the device branch of direct_coop, lane by lane
static void direct_lanes(uint32_t& range, uint32_t& code, uint32_t& dist, uint32_t left, ArrRd& rd) {
  Rc<ArrRd> rc{range, code, &rd};
  do {
    rc.norm();
    const uint32_t R = rc.range, C = rc.code;
    uint32_t k = 8u - uint32_t(__builtin_clz(R));
    k = k < left ? k : left;
    k = k < 5u ? k : 5u;
    const uint32_t Rk = R >> k;
    if (C >= 0x80000000u + Rk) {
      for (uint32_t i = 0; i < k; ++i) {
        if (i) rc.norm();
        rc.range >>= 1; rc.code -= rc.range;
        const uint32_t t = 0u - (rc.code >> 31);
        dist = (dist << 1) + (t + 1u); rc.code += rc.range & t;
      }
    } else {
      uint32_t Sl[32]; uint64_t ball = 0;
      for (uint32_t j = 0; j < 32; ++j) {
        uint32_t S = 0;
        for (uint32_t t = 0; t < 5u; ++t) S += ((j >> t) & 1u) ? (R >> ((k - t) & 31u)) : 0u;
        Sl[j] = S;
        if ((j >> k) == 0u && S <= C) ball |= 1ull << j;
      }
      const uint32_t v = uint32_t(__builtin_popcountll(ball)) - 1u;
      rc.code = C - Sl[v]; rc.range = Rk; dist = (dist << k) | v;
    }
    left -= k;
  } while (left != 0);
  range = rc.range; code = rc.code;
}
int main(int argc, char** argv) {
  std::mt19937_64 g(7);
  uint8_t buf[64];
  long bad = 0, n = 0;
  const long cases = argc > 1 ? atol(argv[1]) : 1000000;
  for (long it = 0; it < cases; ++it) {
    for (auto& b : buf) b = uint8_t(g());
    uint32_t R, C;
    int mode = it % 4;
    R = uint32_t(g()) | 1u;
    if ((g() & 3) == 0) R >>= (g() % 12);  // some ranges that need normalising
    if (R < (1u << 18)) R |= 1u << 18;  // the decoder never enters with less (a decision leaves >= 2^24 * 31 / 2048)
    if (mode < 2) C = uint32_t(g() % R);          // well-formed: code < range
    else if (mode == 2) C = uint32_t(g());        // anything (corrupt)
    else C = R - 1 - uint32_t(g() % 4);           // edge near range
    uint32_t left = 1 + uint32_t(g() % 26);
    uint32_t d0 = uint32_t(g() % 4) | 2u;
    // reference
    ArrRd r1{buf}; Rc<ArrRd> a{R, C, &r1};
    uint32_t da = d0;
    for (uint32_t k = 0; k < left; ++k) a.direct(da);
    ArrRd r2{buf}; Rc<ArrRd> b{R, C, &r2};
    uint32_t db = d0;
    direct_coop(b, db, left);
    ++n;
    { ArrRd r3{buf}; uint32_t R3 = R, C3 = C, d3 = d0; direct_lanes(R3, C3, d3, left, r3);
      if (R3 != a.range || C3 != a.code || d3 != da || r3.i != r1.i) {
        if (bad++ < 5) printf("lanes mismatch R=%08x C=%08x left=%u\n", R, C, left); } }
    if (a.range != b.range || a.code != b.code || da != db || r1.i != r2.i) {
      if (bad++ < 5) printf("mismatch R=%08x C=%08x left=%u: ref %08x %08x %08x %u / got %08x %08x %08x %u\n",
                            R, C, left, a.range, a.code, da, r1.i, b.range, b.code, db, r2.i);
    }
  }
  printf("%ld cases, %ld mismatches\n", n, bad);
  return bad != 0;
}

// xz_capi.hip -- host side of the xz block batch, x86 BCJ and CRC-64 C ABI
// (include/lzma_gpu.h).
//
// The reference reads xz strictly forward (XzUnpacker_Code, XzDec.c:604-870)
// or indexes it backwards from the footer (Xzs_ReadBackward, XzIn.c:141-306).
// Here the backward index is the plan: every block of every stream becomes
// one LZMA2 item of a single GPU batch (LzmaGpu_PlanBatchEx /
// LzmaGpu_DecodeBatchEx), followed by the x86 BCJ kernel for blocks that
// carry the filter and the CRC-32 / CRC-64 kernels for the block checks.
// The host keeps what the reference keeps outside its coders: container
// parsing with its small CRC-32s (stream header, block headers, index,
// footer) and SHA-256 checks.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <exception>
#include <vector>

#include "lzma_gpu_internal.h"

static_assert(sizeof(LzmaGpuXzBlock) == 104, "LzmaGpuXzBlock layout (lzmagpu.py XzBlock)");

using lzgpu_host::ensure_device;
using lzgpu_host::hip_ok;
using lzgpu_host::set_error;
using lzgpu_host::crc32_host;
using lzgpu_host::DevArr;

namespace {

constexpr size_t kXzHeader = 12, kXzFooter = 12;

uint32_t le32(const Byte* p) {
  return uint32_t(p[0]) | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 24);
}

// Xz_ReadVarInt (XzDec.c:30-44): 0 on failure
unsigned read_varint(const Byte* p, size_t max, uint64_t* v) {
  *v = 0;
  const unsigned limit = max > 9 ? 9 : unsigned(max);
  for (unsigned i = 0; i < limit;) {
    const Byte b = p[i];
    *v |= uint64_t(b & 0x7F) << (7 * i++);
    if ((b & 0x80) == 0) return (b == 0 && i != 1) ? 0 : i;
  }
  return 0;
}

// XzFlags_GetCheckSize (Xz.c:40-44)
uint32_t check_size(uint32_t t) { return t == 0 ? 0 : (4u << ((t - 1) / 3)); }

// FIPS 180-4 SHA-256 (the XZ_CHECK_SHA256 block check, Sha256.c)
struct Sha256 {
  uint32_t h[8];
  uint64_t n = 0;
  Byte buf[64];
  size_t fill = 0;
  static uint32_t rotr(uint32_t x, int r) { return (x >> r) | (x << (32 - r)); }
  Sha256() {
    static const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    memcpy(h, iv, sizeof h);
  }
  void block(const Byte* p) {
    static const uint32_t k[64] = {
        0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4,
        0xab1c5ed5, 0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe,
        0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f,
        0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7,
        0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc,
        0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b,
        0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116,
        0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
        0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
        0xc67178f2};
    uint32_t w[64];
    for (int i = 0; i < 16; ++i)
      w[i] = (uint32_t(p[4 * i]) << 24) | (uint32_t(p[4 * i + 1]) << 16) |
             (uint32_t(p[4 * i + 2]) << 8) | p[4 * i + 3];
    for (int i = 16; i < 64; ++i) {
      const uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
      const uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; ++i) {
      const uint32_t t1 = hh + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) +
                          k[i] + w[i];
      const uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
      hh = g;
      g = f;
      f = e;
      e = d + t1;
      d = c;
      c = b;
      b = a;
      a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
  void update(const Byte* p, size_t len) {
    n += len;
    while (len) {
      const size_t take = std::min(len, 64 - fill);
      memcpy(buf + fill, p, take);
      fill += take;
      p += take;
      len -= take;
      if (fill == 64) {
        block(buf);
        fill = 0;
      }
    }
  }
  void final(Byte* out) {
    const uint64_t bits = n * 8;
    const Byte one = 0x80, zero = 0;
    update(&one, 1);
    while (fill != 56) update(&zero, 1);
    Byte l[8];
    for (int i = 0; i < 8; ++i) l[i] = Byte(bits >> (56 - 8 * i));
    update(l, 8);
    for (int i = 0; i < 8; ++i)
      for (int j = 0; j < 4; ++j) out[4 * i + j] = Byte(h[i] >> (24 - 8 * j));
  }
};

// One stream, read backwards from the footer ending at `end` (Xz_ReadBackward,
// XzIn.c:141-224); blocks appended in stream order; *start = stream start.
SRes index_stream(const Byte* f, size_t end, uint32_t stream, std::vector<LzmaGpuXzBlock>* out,
                  size_t* start) {
  if ((end & 3) != 0 || end < kXzFooter) return SZ_ERROR_NO_ARCHIVE;
  const Byte* ft = f + end - kXzFooter;
  if (ft[10] != 'Y' || ft[11] != 'Z') return SZ_ERROR_NO_ARCHIVE;
  const uint32_t flags = (uint32_t(ft[8]) << 8) | ft[9];
  if (flags > 0xF) return SZ_ERROR_UNSUPPORTED;
  if (le32(ft) != crc32_host(ft + 4, 6)) return SZ_ERROR_ARCHIVE;
  const uint64_t index_size = (uint64_t(le32(ft + 4)) + 1) << 2;
  if (index_size > end - kXzFooter) return SZ_ERROR_ARCHIVE;
  const size_t ix = end - kXzFooter - size_t(index_size);
  // Xz_ReadIndex2 (XzIn.c:62-106)
  const Byte* b = f + ix;
  size_t size = size_t(index_size);
  if (size < 5 || b[0] != 0) return SZ_ERROR_ARCHIVE;
  size -= 4;
  if (crc32_host(b, size) != le32(b + size)) return SZ_ERROR_ARCHIVE;
  size_t pos = 1;
  uint64_t nblocks;
  unsigned s = read_varint(b + pos, size - pos, &nblocks);
  if (s == 0) return SZ_ERROR_ARCHIVE;
  pos += s;
  if (nblocks * 2 > size) return SZ_ERROR_ARCHIVE;
  std::vector<uint64_t> unpadded(nblocks), unpack(nblocks);
  uint64_t packed_total = 0;
  for (uint64_t i = 0; i < nblocks; ++i) {
    s = read_varint(b + pos, size - pos, &unpadded[i]);
    if (s == 0) return SZ_ERROR_ARCHIVE;
    pos += s;
    s = read_varint(b + pos, size - pos, &unpack[i]);
    if (s == 0) return SZ_ERROR_ARCHIVE;
    pos += s;
    if (unpadded[i] == 0) return SZ_ERROR_ARCHIVE;
    packed_total += (unpadded[i] + 3) & ~uint64_t(3);
    if (packed_total >= (uint64_t(1) << 62)) return SZ_ERROR_ARCHIVE;
  }
  while ((pos & 3) != 0)
    if (b[pos++] != 0) return SZ_ERROR_ARCHIVE;
  if (pos != size) return SZ_ERROR_ARCHIVE;
  // stream header (Xz_ReadHeader / Xz_ParseHeader, XzIn.c:10-17, XzDec.c:482-489)
  const uint64_t sum = kXzHeader + packed_total + index_size;
  if (sum > end - kXzFooter) return SZ_ERROR_ARCHIVE;
  const size_t st = end - kXzFooter - size_t(sum);
  static const Byte kSig[6] = {0xFD, '7', 'z', 'X', 'Z', 0};
  if (memcmp(f + st, kSig, 6) != 0) return SZ_ERROR_NO_ARCHIVE;
  if (crc32_host(f + st + 6, 2) != le32(f + st + 8)) return SZ_ERROR_NO_ARCHIVE;
  const uint32_t hflags = (uint32_t(f[st + 6]) << 8) | f[st + 7];
  if (hflags > 0xF) return SZ_ERROR_UNSUPPORTED;
  if (hflags != flags) return SZ_ERROR_ARCHIVE;
  const uint32_t ctype = flags & 0xF, csize = check_size(ctype);
  // blocks (XzBlock_Parse, XzDec.c:505-556)
  size_t at = st + kXzHeader;
  for (uint64_t i = 0; i < nblocks; ++i) {
    const Byte* h = f + at;
    const uint32_t hsize = (uint32_t(h[0]) << 2) + 4;
    if (h[0] == 0 || uint64_t(hsize) + csize >= unpadded[i]) return SZ_ERROR_ARCHIVE;
    const uint32_t hs = hsize - 4;
    if (crc32_host(h, hs) != le32(h + hs)) return SZ_ERROR_ARCHIVE;
    size_t p = 1;
    const Byte bflags = h[p++];
    uint64_t v;
    const uint64_t pack = unpadded[i] - hsize - csize;
    if (bflags & 0x40) {
      s = read_varint(h + p, hs - p, &v);
      if (s == 0 || v == 0 || v != pack) return SZ_ERROR_ARCHIVE;
      p += s;
    }
    if (bflags & 0x80) {
      s = read_varint(h + p, hs - p, &v);
      if (s == 0 || v != unpack[i]) return SZ_ERROR_ARCHIVE;
      p += s;
    }
    const int nf = (bflags & 3) + 1;
    uint64_t ids[4];
    uint32_t psz[4];
    const Byte* props[4];
    for (int k = 0; k < nf; ++k) {
      s = read_varint(h + p, hs - p, &ids[k]);
      if (s == 0) return SZ_ERROR_ARCHIVE;
      p += s;
      s = read_varint(h + p, hs - p, &v);
      if (s == 0) return SZ_ERROR_ARCHIVE;
      p += s;
      if (v > hs - p || v > 20) return SZ_ERROR_ARCHIVE;
      psz[k] = uint32_t(v);
      props[k] = h + p;
      p += size_t(v);
    }
    while (p < hs)
      if (h[p++] != 0) return SZ_ERROR_ARCHIVE;
    LzmaGpuXzBlock blk;
    memset(&blk, 0, sizeof blk);
    // chains: up to three of Delta / x86 / PPC / IA64 / ARM / ARMT / SPARC, then
    // LZMA2 (XZ_ID_LZMA2 0x21); props validated as BraState_SetProps does
    // (XzDec.c:71-109)
    const int last = nf - 1;
    if (ids[last] != 0x21 || psz[last] != 1 || props[last][0] > 40) return SZ_ERROR_UNSUPPORTED;
    blk.num_filters = uint32_t(last);
    for (int k = 0; k < last; ++k) {
      const uint64_t id = ids[k];
      uint32_t prop = 0;
      if (id == 3) {  // XZ_ID_Delta: one byte, distance = byte + 1
        if (psz[k] != 1) return SZ_ERROR_UNSUPPORTED;
        prop = uint32_t(props[k][0]) + 1;
      } else if (id >= 4 && id <= 9) {
        if (psz[k] == 4) {
          prop = le32(props[k]);
          const uint32_t align = id == 6 ? 0xF : (id == 8 ? 1 : (id == 4 ? 0 : 3));
          if (prop & align) return SZ_ERROR_UNSUPPORTED;
        } else if (psz[k] != 0) {
          return SZ_ERROR_UNSUPPORTED;
        }
        if (id == 4) {
          blk.x86 = 1;
          blk.x86_ip = prop;
        }
      } else {
        return SZ_ERROR_UNSUPPORTED;
      }
      blk.filter_id[k] = uint32_t(id);
      blk.filter_prop[k] = prop;
    }
    blk.header_off = at;
    blk.data_off = at + hsize;
    blk.pack_size = pack;
    blk.unpack_size = unpack[i];
    blk.check_off = at + ((uint64_t(hsize) + pack + 3) & ~uint64_t(3));
    blk.check_type = ctype;
    blk.check_size = csize;
    blk.lzma2_prop = props[last][0];
    blk.stream = stream;
    out->push_back(blk);
    at += size_t((unpadded[i] + 3) & ~uint64_t(3));
  }
  *start = st;
  return SZ_OK;
}

SRes index_file(const Byte* f, size_t size, std::vector<LzmaGpuXzBlock>* blocks,
                uint64_t* total) {
  std::vector<std::vector<LzmaGpuXzBlock>> streams;
  size_t end = size;
  if (size < kXzFooter + kXzHeader) return SZ_ERROR_NO_ARCHIVE;
  for (;;) {
    // stream padding: zero bytes in multiples of 4 (XzIn.c:153-187)
    size_t e = end;
    while (e > 0 && f[e - 1] == 0) --e;
    if (e != end) {
      if (((end - e) & 3) != 0) return SZ_ERROR_NO_ARCHIVE;
      end = e;
    }
    std::vector<LzmaGpuXzBlock> one;
    size_t start = 0;
    const SRes r = index_stream(f, end, 0, &one, &start);
    if (r != SZ_OK) return r;
    streams.push_back(std::move(one));
    if (start == 0) break;
    end = start;
  }
  blocks->clear();
  uint64_t dst = 0;
  for (size_t k = streams.size(); k-- > 0;) {
    for (LzmaGpuXzBlock& b : streams[k]) {
      b.stream = uint32_t(streams.size() - 1 - k);
      b.dst_off = dst;
      dst += b.unpack_size;
      blocks->push_back(b);
    }
  }
  *total = dst;
  return SZ_OK;
}

}  // namespace

static SRes xz_index(const Byte* file, size_t size, LzmaGpuXzBlock* blocks, size_t cap,
                     size_t* n_blocks, uint64_t* unpack_total) {
  std::vector<LzmaGpuXzBlock> v;
  uint64_t total = 0;
  const SRes r = index_file(file, size, &v, &total);
  if (n_blocks) *n_blocks = r == SZ_OK ? v.size() : 0;
  if (unpack_total) *unpack_total = r == SZ_OK ? total : 0;
  if (r != SZ_OK) return r;
  if (blocks)
    for (size_t i = 0; i < v.size() && i < cap; ++i) blocks[i] = v[i];
  return SZ_OK;
}

SRes BcjGpu_X86Batch(Byte* d_data, const uint64_t* d_off, const uint64_t* d_len,
                     const uint32_t* d_ip, uint32_t* d_state, uint64_t* d_done, size_t n,
                     int encoding, void* stream) {
  if (!ensure_device()) return SZ_ERROR_FAIL;
  if (n > 0xFFFFFFFFull) return SZ_ERROR_PARAM;
  if (lzgpu_launch_bcj_x86(d_data, d_off, d_len, d_ip, d_state, d_done, uint32_t(n), encoding,
                           static_cast<hipStream_t>(stream)) != 0) {
    set_error("BCJ kernel launch failed");
    return SZ_ERROR_FAIL;
  }
  return SZ_OK;
}

SRes Crc64Gpu_Batch(const Byte* d_data, const uint64_t* d_off, const uint64_t* d_len, size_t n,
                    const uint32_t* d_chunk_base, const uint32_t* d_chunk_range, size_t n_chunks,
                    uint64_t init, uint64_t xorout, uint64_t* d_chunk_crc, uint64_t* d_crc,
                    void* stream) {
  if (!ensure_device()) return SZ_ERROR_FAIL;
  if (n > 0xFFFFFFFFull || n_chunks > 0xFFFFFFFFull) return SZ_ERROR_PARAM;
  if (lzgpu_launch_crc64_arrays(d_data, d_off, d_len, uint32_t(n), d_chunk_base, d_chunk_range,
                                uint32_t(n_chunks), init, xorout, d_chunk_crc, d_crc,
                                static_cast<hipStream_t>(stream)) != 0) {
    set_error("CRC-64 kernel launch failed");
    return SZ_ERROR_FAIL;
  }
  return SZ_OK;
}

// x86_Convert over a host buffer: upload, one lane, download
SizeT x86_Convert(Byte* data, SizeT size, UInt32 ip, UInt32* state, int encoding) {
  if (!ensure_device()) return 0;
  if (size < 5) return 0;
  DevArr<Byte> d;
  DevArr<uint64_t> meta;  // off, len, done
  DevArr<uint32_t> m32;   // ip, state
  const uint64_t ol[2] = {0, uint64_t(size)};
  const uint32_t is[2] = {ip, *state};
  uint64_t done = 0;
  uint32_t st = 0;
  if (!d.alloc(size) || !meta.alloc(3) || !m32.alloc(2)) {
    set_error("x86_Convert: device allocation failed");
    return 0;
  }
  if (!hip_ok(hipMemcpy(d.p, data, size, hipMemcpyHostToDevice), "x86_Convert H2D") ||
      !hip_ok(hipMemcpy(meta.p, ol, 16, hipMemcpyHostToDevice), "x86_Convert H2D") ||
      !hip_ok(hipMemcpy(m32.p, is, 8, hipMemcpyHostToDevice), "x86_Convert H2D"))
    return 0;
  if (lzgpu_launch_bcj_x86(d.p, meta.p, meta.p + 1, m32.p, m32.p + 1, meta.p + 2, 1, encoding,
                           nullptr) != 0 ||
      !hip_ok(hipDeviceSynchronize(), "x86_Convert kernel") ||
      !hip_ok(hipMemcpy(data, d.p, size, hipMemcpyDeviceToHost), "x86_Convert D2H") ||
      !hip_ok(hipMemcpy(&done, meta.p + 2, 8, hipMemcpyDeviceToHost), "x86_Convert D2H") ||
      !hip_ok(hipMemcpy(&st, m32.p + 1, 4, hipMemcpyDeviceToHost), "x86_Convert D2H"))
    return 0;
  *state = st;
  return SizeT(done);
}

namespace {

bool bra_kind_ok(unsigned kind) {
  return kind == 5 || kind == 6 || kind == 7 || kind == 8 || kind == 9;
}

// one RISC converter over a host buffer: upload, one range, download
SizeT bra_convert_host(unsigned kind, const char* name, Byte* data, SizeT size, UInt32 ip,
                       int encoding) {
  if (!ensure_device()) return 0;
  if (size < (kind == 6 ? 16u : 4u)) return 0;
  DevArr<Byte> d;
  DevArr<uint64_t> meta;  // off, len, done
  DevArr<uint32_t> m32;   // ip
  const uint64_t ol[2] = {0, uint64_t(size)};
  uint64_t done = 0;
  if (!d.alloc(size) || !meta.alloc(3) || !m32.alloc(1)) {
    set_error("Bra converter: device allocation failed");
    return 0;
  }
  if (!hip_ok(hipMemcpy(d.p, data, size, hipMemcpyHostToDevice), name) ||
      !hip_ok(hipMemcpy(meta.p, ol, 16, hipMemcpyHostToDevice), name) ||
      !hip_ok(hipMemcpy(m32.p, &ip, 4, hipMemcpyHostToDevice), name))
    return 0;
  if (lzgpu_launch_bra(kind, d.p, meta.p, meta.p + 1, m32.p, meta.p + 2, 1, encoding, nullptr) !=
          0 ||
      !hip_ok(hipDeviceSynchronize(), name) ||
      !hip_ok(hipMemcpy(data, d.p, size, hipMemcpyDeviceToHost), name) ||
      !hip_ok(hipMemcpy(&done, meta.p + 2, 8, hipMemcpyDeviceToHost), name))
    return 0;
  return SizeT(done);
}

void delta_host(Byte* state, unsigned delta, Byte* data, SizeT size, int encoding) {
  if (!ensure_device()) return;
  if (delta == 0 || delta > 256) {
    set_error("Delta: delta outside 1..256");
    return;
  }
  DevArr<Byte> d, st;
  DevArr<uint64_t> meta;  // off, len
  DevArr<uint32_t> dl;
  const uint64_t ol[2] = {0, uint64_t(size)};
  if (!d.alloc(size ? size : 1) || !st.alloc(256) || !meta.alloc(2) || !dl.alloc(1)) {
    set_error("Delta: device allocation failed");
    return;
  }
  if ((size && !hip_ok(hipMemcpy(d.p, data, size, hipMemcpyHostToDevice), "Delta H2D")) ||
      !hip_ok(hipMemcpy(st.p, state, delta, hipMemcpyHostToDevice), "Delta H2D") ||
      !hip_ok(hipMemcpy(meta.p, ol, 16, hipMemcpyHostToDevice), "Delta H2D") ||
      !hip_ok(hipMemcpy(dl.p, &delta, 4, hipMemcpyHostToDevice), "Delta H2D"))
    return;
  if (lzgpu_launch_delta(d.p, meta.p, meta.p + 1, dl.p, st.p, 1, encoding, nullptr) != 0 ||
      !hip_ok(hipDeviceSynchronize(), "Delta kernel") ||
      (size && !hip_ok(hipMemcpy(data, d.p, size, hipMemcpyDeviceToHost), "Delta D2H")) ||
      !hip_ok(hipMemcpy(state, st.p, delta, hipMemcpyDeviceToHost), "Delta D2H"))
    return;
}

}  // namespace

SizeT ARM_Convert(Byte* data, SizeT size, UInt32 ip, int encoding) {
  return bra_convert_host(7, "ARM_Convert", data, size, ip, encoding);
}
SizeT ARMT_Convert(Byte* data, SizeT size, UInt32 ip, int encoding) {
  return bra_convert_host(8, "ARMT_Convert", data, size, ip, encoding);
}
SizeT PPC_Convert(Byte* data, SizeT size, UInt32 ip, int encoding) {
  return bra_convert_host(5, "PPC_Convert", data, size, ip, encoding);
}
SizeT SPARC_Convert(Byte* data, SizeT size, UInt32 ip, int encoding) {
  return bra_convert_host(9, "SPARC_Convert", data, size, ip, encoding);
}
SizeT IA64_Convert(Byte* data, SizeT size, UInt32 ip, int encoding) {
  return bra_convert_host(6, "IA64_Convert", data, size, ip, encoding);
}
void Delta_Init(Byte* state) { memset(state, 0, 256); }
void Delta_Encode(Byte* state, unsigned delta, Byte* data, SizeT size) {
  delta_host(state, delta, data, size, 1);
}
void Delta_Decode(Byte* state, unsigned delta, Byte* data, SizeT size) {
  delta_host(state, delta, data, size, 0);
}

SRes BraGpu_Batch(unsigned kind, Byte* d_data, const uint64_t* d_off, const uint64_t* d_len,
                  const uint32_t* d_ip, uint64_t* d_done, size_t n, int encoding, void* stream) {
  if (!bra_kind_ok(kind)) return SZ_ERROR_UNSUPPORTED;
  if (!ensure_device()) return SZ_ERROR_FAIL;
  if (n > 0xFFFFFFFFull) return SZ_ERROR_PARAM;
  if (lzgpu_launch_bra(kind, d_data, d_off, d_len, d_ip, d_done, uint32_t(n), encoding,
                       static_cast<hipStream_t>(stream)) != 0) {
    set_error("branch converter kernel launch failed");
    return SZ_ERROR_FAIL;
  }
  return SZ_OK;
}

SRes DeltaGpu_Batch(Byte* d_data, const uint64_t* d_off, const uint64_t* d_len,
                    const uint32_t* d_delta, Byte* d_state, size_t n, int encoding, void* stream) {
  if (!ensure_device()) return SZ_ERROR_FAIL;
  if (n > 0xFFFFFFFFull) return SZ_ERROR_PARAM;
  if (lzgpu_launch_delta(d_data, d_off, d_len, d_delta, d_state, uint32_t(n), encoding,
                         static_cast<hipStream_t>(stream)) != 0) {
    set_error("delta kernel launch failed");
    return SZ_ERROR_FAIL;
  }
  return SZ_OK;
}

SRes Bcj2Gpu_Batch(const Bcj2GpuJob* d_jobs, size_t n, int32_t* d_res, void* stream) {
  if (!ensure_device()) return SZ_ERROR_FAIL;
  if (n > 0xFFFFFFFFull) return SZ_ERROR_PARAM;
  if (lzgpu_launch_bcj2(d_jobs, uint32_t(n), d_res, static_cast<hipStream_t>(stream)) != 0) {
    set_error("BCJ2 kernel launch failed");
    return SZ_ERROR_FAIL;
  }
  return SZ_OK;
}

// Bcj2_Decode over host buffers: the four streams and the output go to the
// device (buf0 inside outBuf, as 7zDec.c:367-372 places it, stays inside the
// device copy of outBuf at the same offset), one lane decodes, the output
// comes back.
static int bcj2_host(const Byte* buf0, SizeT size0, const Byte* buf1, SizeT size1,
                     const Byte* buf2, SizeT size2, const Byte* buf3, SizeT size3, Byte* outBuf,
                     SizeT outSize) {
  if (!ensure_device()) return SZ_ERROR_FAIL;
  const uintptr_t o0 = uintptr_t(outBuf), o1 = o0 + outSize, b0 = uintptr_t(buf0);
  const bool inside = size0 && b0 >= o0 && b0 < o1;
  // device layout: [out (+ main tail beyond it) | buf0 | buf1 | buf2 | buf3]
  const uint64_t out_room = inside ? std::max<uint64_t>(outSize, (b0 - o0) + size0) : outSize;
  const uint64_t off0 = out_room, off1 = off0 + (inside ? 0 : size0), off2 = off1 + size1,
                 off3 = off2 + size2, total = off3 + size3;
  DevArr<Byte> d;
  DevArr<Bcj2GpuJob> dj;
  DevArr<int32_t> dr;
  if (!d.alloc(size_t(total)) || !dj.alloc(1) || !dr.alloc(1)) {
    set_error("Bcj2_Decode: device allocation failed");
    return SZ_ERROR_MEM;
  }
  auto up = [&](uint64_t at, const Byte* p, uint64_t n) {
    return n == 0 || hip_ok(hipMemcpy(d.p + at, p, size_t(n), hipMemcpyHostToDevice), "Bcj2 H2D");
  };
  bool ok = true;
  if (inside) {
    // the host bytes of outBuf (main stream included) and any main tail beyond it
    ok = up(0, outBuf, outSize);
    if (ok && (b0 - o0) + size0 > outSize)
      ok = up(outSize, reinterpret_cast<const Byte*>(o1), (b0 - o0) + size0 - outSize);
  } else {
    // bytes the decoder does not write (an error exit) keep the caller's values
    ok = up(0, outBuf, outSize) && up(off0, buf0, size0);
  }
  ok = ok && up(off1, buf1, size1) && up(off2, buf2, size2) && up(off3, buf3, size3);
  if (!ok) return SZ_ERROR_FAIL;
  Bcj2GpuJob j;
  j.buf0 = inside ? d.p + (b0 - o0) : d.p + off0;
  j.buf1 = d.p + off1;
  j.buf2 = d.p + off2;
  j.buf3 = d.p + off3;
  j.size0 = size0;
  j.size1 = size1;
  j.size2 = size2;
  j.size3 = size3;
  j.out = d.p;
  j.out_size = outSize;
  int32_t r = SZ_ERROR_FAIL;
  if (!hip_ok(hipMemcpy(dj.p, &j, sizeof j, hipMemcpyHostToDevice), "Bcj2 H2D") ||
      Bcj2Gpu_Batch(dj.p, 1, dr.p, nullptr) != SZ_OK || !hip_ok(hipDeviceSynchronize(), "Bcj2") ||
      !hip_ok(hipMemcpy(&r, dr.p, 4, hipMemcpyDeviceToHost), "Bcj2 D2H") ||
      (outSize && !hip_ok(hipMemcpy(outBuf, d.p, outSize, hipMemcpyDeviceToHost), "Bcj2 D2H")))
    return SZ_ERROR_FAIL;
  return r;
}

int Bcj2_Decode(const Byte* buf0, SizeT size0, const Byte* buf1, SizeT size1, const Byte* buf2,
                SizeT size2, const Byte* buf3, SizeT size3, Byte* outBuf, SizeT outSize) {
  try {
    return bcj2_host(buf0, size0, buf1, size1, buf2, size2, buf3, size3, outBuf, outSize);
  } catch (const std::exception&) {
    set_error("Bcj2_Decode: host allocation failed");
    return SZ_ERROR_MEM;
  }
}

UInt64 Crc64Calc(const void* data, size_t size) {
  if (!ensure_device()) return 0;
  if (size == 0) return 0;
  const uint64_t cap = size;
  const size_t nch = CrcGpu_PlanChunks(&cap, 1, nullptr, nullptr);
  std::vector<uint32_t> meta(1 + nch);
  CrcGpu_PlanChunks(&cap, 1, meta.data(), meta.data() + 1);
  DevArr<Byte> d;
  DevArr<uint64_t> ol, chunks;
  DevArr<uint32_t> m;
  const uint64_t olh[3] = {0, cap, 0};
  if (!d.alloc(size) || !ol.alloc(3) || !chunks.alloc(nch) || !m.alloc(1 + nch)) {
    set_error("Crc64Calc: device allocation failed");
    return 0;
  }
  uint64_t out = 0;
  if (!hip_ok(hipMemcpy(d.p, data, size, hipMemcpyHostToDevice), "CRC-64 H2D") ||
      !hip_ok(hipMemcpy(ol.p, olh, 24, hipMemcpyHostToDevice), "CRC-64 H2D") ||
      !hip_ok(hipMemcpy(m.p, meta.data(), 4 * (1 + nch), hipMemcpyHostToDevice), "CRC-64 H2D"))
    return 0;
  if (lzgpu_launch_crc64_arrays(d.p, ol.p, ol.p + 1, 1, m.p, m.p + 1, uint32_t(nch), ~0ull, ~0ull,
                                chunks.p, ol.p + 2, nullptr) != 0 ||
      !hip_ok(hipDeviceSynchronize(), "CRC-64 kernel") ||
      !hip_ok(hipMemcpy(&out, ol.p + 2, 8, hipMemcpyDeviceToHost), "CRC-64 D2H"))
    return 0;
  return out;
}

static SRes xz_decode(Byte* dest, SizeT* destLen, const Byte* file, size_t size,
                      int64_t* bad_block) {
  const SizeT cap = *destLen;
  *destLen = 0;
  if (bad_block) *bad_block = -1;
  std::vector<LzmaGpuXzBlock> blk;
  uint64_t total = 0;
  SRes r = index_file(file, size, &blk, &total);
  if (r != SZ_OK) return r;
  if (total > cap) return SZ_ERROR_OUTPUT_EOF;
  const size_t n = blk.size();
  if (n == 0) return SZ_OK;
  if (!ensure_device()) return SZ_ERROR_FAIL;
  // per-block failure in the reference's order: data, then padding, then check
  std::vector<int> fail(n, SZ_OK);
  for (size_t i = 0; i < n; ++i) {
    for (uint64_t p = blk[i].data_off + blk[i].pack_size; p < blk[i].check_off; ++p)
      if (file[p] != 0) fail[i] = SZ_ERROR_CRC;
  }
  // one LZMA2 item per block, FINISH_END at exactly its indexed size
  std::vector<LzmaGpuStreamDesc> descs(n);
  for (size_t i = 0; i < n; ++i) {
    LzmaGpuStreamDesc& d = descs[i];
    memset(&d, 0, sizeof d);
    d.src_off = blk[i].data_off;
    d.src_len = blk[i].pack_size;
    d.dst_off = blk[i].dst_off;
    d.dst_cap = blk[i].unpack_size;
    d.props[0] = Byte(blk[i].lzma2_prop);
    d.props_size = 1;
    d.finish_mode = LZMA_FINISH_END;
    d.kind = LZMA_GPU_KIND_LZMA2;
  }
  std::vector<uint32_t> order(n);
  LzmaGpuPlan plan;
  if ((r = LzmaGpu_PlanBatchEx(descs.data(), n, order.data(), &plan)) != SZ_OK) return r;
  // check ranges (after BCJ): CRC-32 and CRC-64 blocks, chunk plans
  std::vector<uint64_t> off32, len32, off64, len64;
  std::vector<size_t> idx32, idx64;
  for (size_t i = 0; i < n; ++i) {
    if (blk[i].check_type == LZMA_GPU_XZ_CHECK_CRC32) {
      idx32.push_back(i);
      off32.push_back(blk[i].dst_off);
      len32.push_back(blk[i].unpack_size);
    } else if (blk[i].check_type == LZMA_GPU_XZ_CHECK_CRC64) {
      idx64.push_back(i);
      off64.push_back(blk[i].dst_off);
      len64.push_back(blk[i].unpack_size);
    }
  }
  const size_t nch32 = CrcGpu_PlanChunks(len32.data(), len32.size(), nullptr, nullptr);
  const size_t nch64 = CrcGpu_PlanChunks(len64.data(), len64.size(), nullptr, nullptr);
  if (nch32 == size_t(-1) || nch64 == size_t(-1)) return SZ_ERROR_PARAM;
  std::vector<uint32_t> cb32(len32.size() + nch32), cb64(len64.size() + nch64);
  CrcGpu_PlanChunks(len32.data(), len32.size(), cb32.data(), cb32.data() + len32.size());
  CrcGpu_PlanChunks(len64.data(), len64.size(), cb64.data(), cb64.data() + len64.size());

  DevArr<Byte> d_src, d_dst, d_ws;
  DevArr<LzmaGpuStreamDesc> d_desc;
  DevArr<uint32_t> d_order, d_cb32, d_cb64, d_crc32, d_chunk32;
  DevArr<LzmaGpuResult> d_res;
  DevArr<uint64_t> d_ol32, d_ol64, d_chunk64, d_crc64;
  if (!d_src.alloc(size) || !d_dst.alloc(total) || !d_ws.alloc(plan.workspace_bytes) ||
      !d_desc.alloc(n) || !d_order.alloc(n) || !d_res.alloc(n) ||
      !d_ol32.alloc(2 * off32.size()) || !d_cb32.alloc(cb32.size()) ||
      !d_chunk32.alloc(nch32) || !d_crc32.alloc(off32.size()) ||
      !d_ol64.alloc(2 * off64.size()) || !d_cb64.alloc(cb64.size()) ||
      !d_chunk64.alloc(nch64) || !d_crc64.alloc(off64.size())) {
    set_error("XzDecode: device allocation failed");
    return SZ_ERROR_MEM;
  }
  auto h2d = [](void* d, const void* h, size_t bytes) {
    return bytes == 0 || hip_ok(hipMemcpy(d, h, bytes, hipMemcpyHostToDevice), "XzDecode H2D");
  };
  std::vector<uint64_t> ol32(off32), ol64(off64);
  ol32.insert(ol32.end(), len32.begin(), len32.end());
  ol64.insert(ol64.end(), len64.begin(), len64.end());
  if (!h2d(d_src.p, file, size) || !h2d(d_desc.p, descs.data(), n * sizeof(LzmaGpuStreamDesc)) ||
      !h2d(d_order.p, order.data(), n * 4) || !h2d(d_ol32.p, ol32.data(), ol32.size() * 8) ||
      !h2d(d_cb32.p, cb32.data(), cb32.size() * 4) ||
      !h2d(d_ol64.p, ol64.data(), ol64.size() * 8) ||
      !h2d(d_cb64.p, cb64.data(), cb64.size() * 4))
    return SZ_ERROR_FAIL;
  if ((r = LzmaGpu_DecodeBatchEx(&plan, d_desc.p, d_order.p, d_src.p, d_dst.p, d_ws.p, d_res.p,
                                 nullptr)) != SZ_OK)
    return r;
  // filter chains, last filter first (MixCoder order, XzDec.c:574-585): at each
  // depth, one batch per filter kind over the blocks that have that many
  for (uint32_t depth = 0; depth < 3; ++depth) {
    for (uint32_t kind = 3; kind <= 9; ++kind) {
      std::vector<uint64_t> fo, fl;
      std::vector<uint32_t> fp;
      for (size_t i = 0; i < n; ++i) {
        const uint32_t nf = blk[i].num_filters;
        if (nf > depth && blk[i].filter_id[nf - 1 - depth] == kind) {
          fo.push_back(blk[i].dst_off);
          fl.push_back(blk[i].unpack_size);
          fp.push_back(blk[i].filter_prop[nf - 1 - depth]);
        }
      }
      const size_t nb = fo.size();
      if (nb == 0) continue;
      DevArr<uint64_t> d64;  // off, len, done
      DevArr<uint32_t> d32;  // ip / distance, x86 state
      DevArr<Byte> dstate;   // delta states
      fo.insert(fo.end(), fl.begin(), fl.end());
      fo.resize(3 * nb, 0);
      fp.resize(2 * nb, 0);  // states start at 0 (x86_Convert_Init, Delta_Init)
      if (!d64.alloc(3 * nb) || !d32.alloc(2 * nb) || !dstate.alloc(kind == 3 ? 256 * nb : 1)) {
        set_error("XzDecode: device allocation failed");
        return SZ_ERROR_MEM;
      }
      if (!h2d(d64.p, fo.data(), fo.size() * 8) || !h2d(d32.p, fp.data(), fp.size() * 4) ||
          (kind == 3 && !hip_ok(hipMemset(dstate.p, 0, 256 * nb), "XzDecode memset")))
        return SZ_ERROR_FAIL;
      if (kind == 3)
        r = DeltaGpu_Batch(d_dst.p, d64.p, d64.p + nb, d32.p, dstate.p, nb, 0, nullptr);
      else if (kind == 4)
        r = BcjGpu_X86Batch(d_dst.p, d64.p, d64.p + nb, d32.p, d32.p + nb, d64.p + 2 * nb, nb, 0,
                            nullptr);
      else
        r = BraGpu_Batch(kind, d_dst.p, d64.p, d64.p + nb, d32.p, d64.p + 2 * nb, nb, 0, nullptr);
      if (r != SZ_OK) return r;
      if (!hip_ok(hipDeviceSynchronize(), "XzDecode filters")) return SZ_ERROR_FAIL;
    }
  }
  const size_t n32 = off32.size(), n64 = off64.size();
  if (n32 && (r = CrcGpu_Batch(d_dst.p, d_ol32.p, d_ol32.p + n32, n32, d_cb32.p, d_cb32.p + n32,
                               nch32, 0xFFFFFFFFu, 0xFFFFFFFFu, d_chunk32.p, d_crc32.p,
                               nullptr)) != SZ_OK)
    return r;
  if (n64 && (r = Crc64Gpu_Batch(d_dst.p, d_ol64.p, d_ol64.p + n64, n64, d_cb64.p, d_cb64.p + n64,
                                 nch64, ~0ull, ~0ull, d_chunk64.p, d_crc64.p, nullptr)) != SZ_OK)
    return r;
  std::vector<LzmaGpuResult> res(n);
  std::vector<uint32_t> crc32(n32);
  std::vector<uint64_t> crc64(n64);
  if (!hip_ok(hipDeviceSynchronize(), "XzDecode kernels") ||
      !hip_ok(hipMemcpy(res.data(), d_res.p, n * sizeof(LzmaGpuResult), hipMemcpyDeviceToHost),
              "XzDecode D2H") ||
      (n32 && !hip_ok(hipMemcpy(crc32.data(), d_crc32.p, n32 * 4, hipMemcpyDeviceToHost),
                      "XzDecode D2H")) ||
      (n64 && !hip_ok(hipMemcpy(crc64.data(), d_crc64.p, n64 * 8, hipMemcpyDeviceToHost),
                      "XzDecode D2H")) ||
      !hip_ok(hipMemcpy(dest, d_dst.p, total, hipMemcpyDeviceToHost), "XzDecode D2H"))
    return SZ_ERROR_FAIL;
  for (size_t i = 0; i < n; ++i) {
    const LzmaGpuResult& q = res[i];
    if (q.res != SZ_OK || q.status != LZMA_STATUS_FINISHED_WITH_MARK ||
        q.dest_len != blk[i].unpack_size || q.src_len != blk[i].pack_size)
      fail[i] = SZ_ERROR_DATA;
  }
  for (size_t k = 0; k < n32; ++k) {
    const size_t i = idx32[k];
    if (fail[i] == SZ_OK && crc32[k] != le32(file + blk[i].check_off)) fail[i] = SZ_ERROR_CRC;
  }
  for (size_t k = 0; k < n64; ++k) {
    const size_t i = idx64[k];
    const uint64_t want = uint64_t(le32(file + blk[i].check_off)) |
                          (uint64_t(le32(file + blk[i].check_off + 4)) << 32);
    if (fail[i] == SZ_OK && crc64[k] != want) fail[i] = SZ_ERROR_CRC;
  }
  for (size_t i = 0; i < n; ++i)
    if (fail[i] == SZ_OK && blk[i].check_type == LZMA_GPU_XZ_CHECK_SHA256) {
      Sha256 h;
      Byte dig[32];
      h.update(dest + blk[i].dst_off, size_t(blk[i].unpack_size));
      h.final(dig);
      if (memcmp(dig, file + blk[i].check_off, 32) != 0) fail[i] = SZ_ERROR_CRC;
    }
  for (size_t i = 0; i < n; ++i)
    if (fail[i] != SZ_OK) {
      if (bad_block) *bad_block = int64_t(i);
      return fail[i];
    }
  *destLen = SizeT(total);
  return SZ_OK;
}

// C ABI: no exception crosses it (host allocation failure -> SZ_ERROR_MEM).
SRes LzmaGpu_XzIndex(const Byte* file, size_t size, LzmaGpuXzBlock* blocks, size_t cap,
                     size_t* n_blocks, uint64_t* unpack_total) {
  try {
    return xz_index(file, size, blocks, cap, n_blocks, unpack_total);
  } catch (const std::exception&) {
    set_error("xz: host allocation failed");
    return SZ_ERROR_MEM;
  }
}

SRes LzmaGpu_XzDecode(Byte* dest, SizeT* destLen, const Byte* file, size_t size,
                      int64_t* bad_block) {
  try {
    return xz_decode(dest, destLen, file, size, bad_block);
  } catch (const std::exception&) {
    set_error("xz: host allocation failed");
    return SZ_ERROR_MEM;
  }
}

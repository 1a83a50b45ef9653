// lzma_capi.hip -- host side of liblzmagpu.so: the batch extension
// (include/lzma_gpu.h: planner, batch launches, streaming sessions, LZMA2
// block splitter), the 7zCrc.h drop-ins and the library's shared host state
// (device check, per-device call scratch and class-stream pools).  The
// LzmaDec / LzmaLib / Lzma2Dec drop-ins are in dropin_capi.hip.
//
// Without a HIP device every decode entry returns SZ_ERROR_FAIL (no CPU
// fallback).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <mutex>
#include <new>
#include <numeric>
#include <string>
#include <vector>

#include "crc32_device.h"
#include "lzma_device.h"
#include "lzma_gpu_internal.h"

namespace {

thread_local std::string g_last_error;

void set_error(const std::string& s) { g_last_error = s; }

bool hip_ok(hipError_t e, const char* what) {
  if (e == hipSuccess) return true;
  set_error(std::string(what) + ": " + hipGetErrorString(e));
  return false;
}

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// set once the library has started the HIP runtime with a device present
std::atomic<bool> g_runtime_up{false};

bool ensure_device() {
  static std::once_flag once;
  static int count = 0;
  std::call_once(once, [] {
    count = device_count();
    if (count > 0) g_runtime_up.store(true);
  });
  if (count <= 0) {
    set_error("liblzmagpu: no HIP device available (GPU decoder only, no CPU fallback)");
    static std::atomic<bool> warned{false};
    if (!warned.exchange(true))
      fprintf(stderr, "liblzmagpu: no HIP device available -- decode calls return SZ_ERROR_FAIL\n");
    return false;
  }
  return true;
}

// CUs the planner and launchers size for: the current device's, cached per
// device, once ensure_device() has started the runtime; before that (a
// launcher process that plans before it starts its ranks) MI355X's 256, with
// no HIP call -- planning alone never initialises the GPU.
uint32_t device_cus() {
  if (!g_runtime_up.load()) return 256;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kLzgpuMaxDevices) return 256;
  static std::atomic<uint32_t> cache[kLzgpuMaxDevices];
  uint32_t c = cache[dev].load();
  if (c) return c;
  int v = 0;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
    return 256;
  cache[dev].store(uint32_t(v));
  return uint32_t(v);
}

int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return (v && *v) ? atoi(v) : dflt;
}

}  // namespace

extern "C" {

// ------------------------------------------------------------------ batch extension

// Workspace: each item gets a 16-byte aligned slice of table_cells() cells
// (LZMA2 ranges: the lc+lp=4, pb=4 maximum).  Returns per-item lo-table
// widths (0 = not LDS-eligible) through lo_w when given.
// `skip` (optional): items whose global sections live in a class slot area
// (lane-interleaved throughput classes) get no slice (probs_off 0, unused).
static uint64_t plan_workspace(LzmaGpuStreamDesc* descs, size_t n, std::vector<uint32_t>* lo_w,
                               std::vector<uint32_t>* lat_w = nullptr,
                               const std::vector<uint8_t>* skip = nullptr) {
  uint64_t off = 0;
  if (lo_w) lo_w->assign(n, 0);
  if (lat_w) lat_w->assign(n, 0);
  for (size_t i = 0; i < n; ++i) {
    LzmaGpuStreamDesc& d = descs[i];
    if (skip && (*skip)[i]) {
      d.probs_off = 0;
      continue;
    }
    uint32_t np = 0;
    if (d.kind == LZMA_GPU_KIND_LZMA2) {
      np = lzgpu::table_cells(4, 0, 4);
      if (lo_w && d.props[0] <= 40) (*lo_w)[i] = lzgpu::lzma2_lds_cells(LZGPU_LDS_MASK);
      if (lat_w && d.props[0] <= 40) (*lat_w)[i] = lzgpu::lzma2_lds_cells(LZGPU_LDS_MASK_LAT);
    } else {
      uint32_t lc, lp, pb, dict;
      if (lzgpu::lz_props_parse(d.props, d.props_size, lc, lp, pb, dict) == SZ_OK) {
        np = lzgpu::table_cells(lc, lp, pb);
        if (lo_w) (*lo_w)[i] = lzgpu::make_layout(lc, lp, pb, LZGPU_LDS_MASK).lds_cells;
        if (lat_w) (*lat_w)[i] = lzgpu::make_layout(lc, lp, pb, LZGPU_LDS_MASK_LAT).lds_cells;
      }
    }
    d.probs_off = off;
    off += (uint64_t(np) + 7) & ~uint64_t(7);
  }
  return off * 2;
}

// LDS cells of an item's slice under the slot-global latency placement
// (lzgpu::kLdsMaskLatSlotG); 0 = bad props
static uint32_t lat_slotg_cells(const LzmaGpuStreamDesc& d) {
  if (d.kind == LZMA_GPU_KIND_LZMA2)
    return d.props[0] <= 40 ? lzgpu::lzma2_lds_cells(lzgpu::kLdsMaskLatSlotG) : 0u;
  uint32_t lc, lp, pb, dict;
  if (lzgpu::lz_props_parse(d.props, d.props_size, lc, lp, pb, dict) != SZ_OK) return 0;
  return lzgpu::make_layout(lc, lp, pb, lzgpu::kLdsMaskLatSlotG).lds_cells;
}

static size_t plan_simple(LzmaGpuStreamDesc* descs, size_t n, uint32_t* order) {
  std::vector<uint32_t> w;
  const uint64_t bytes = plan_workspace(descs, n, &w);
  if (order) {
    std::vector<uint32_t> idx(n);
    std::iota(idx.begin(), idx.end(), 0u);
    std::stable_sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) {
      if (descs[a].dst_cap != descs[b].dst_cap) return descs[a].dst_cap > descs[b].dst_cap;
      return w[a] > w[b];
    });
    for (size_t i = 0; i < n; ++i) order[i] = idx[i];
  }
  return size_t(bytes);
}

size_t LzmaGpu_PlanBatch(LzmaGpuStreamDesc* descs, size_t n, uint32_t* order) {
  try {
    return plan_simple(descs, n, order);
  } catch (const std::exception&) {
    set_error("plan: host allocation failed");
    return 0;
  }
}

// Planner defaults with the experiment overrides of the environment, read at
// call time (LZGPU_KERNEL=global|throughput|latency|coop, LZGPU_MASK=1|2,
// LZGPU_COOP=0|1, LZGPU_CUS, LZGPU_LANES, LZGPU_GROUPS, LZGPU_OCC,
// LZGPU_PERSIST=0, LZGPU_CLASSES=1, LZGPU_SLICE_ALIGN8=1, LZGPU_KERNEL_LZMA2=1,
// LZGPU_COOP_LAT=1, LZGPU_MERGE_LAT=0, LZGPU_ILV=0, LZGPU_ILV_ANY=1, LZGPU_THR_FIT=0,
// LZGPU_SLOTG=0).  Only LzmaGpu_PlanBatchEx reads them;
// LzmaGpu_PlanBatchOpt takes its options from the caller alone.
static LzmaGpuPlanOptions env_options() {
  LzmaGpuPlanOptions o;
  memset(&o, 0, sizeof o);
  const char* kv = getenv("LZGPU_KERNEL");
  if (env_int("LZGPU_KERNEL_GLOBAL", 0) || (kv && strcmp(kv, "global") == 0))
    o.kernel = LZMA_GPU_KERNEL_GLOBAL;
  else if (kv && strcmp(kv, "throughput") == 0)
    o.kernel = LZMA_GPU_KERNEL_THROUGHPUT;
  else if (kv && strcmp(kv, "latency") == 0)
    o.kernel = LZMA_GPU_KERNEL_LATENCY;
  else if (kv && strcmp(kv, "coop") == 0)
    o.kernel = LZMA_GPU_KERNEL_COOP;
  const int mask = env_int("LZGPU_MASK", 0), coop = env_int("LZGPU_COOP", -1);
  if (o.kernel == LZMA_GPU_KERNEL_AUTO) {
    if (mask == 1) o.kernel = LZMA_GPU_KERNEL_THROUGHPUT;
    if (mask == 2) o.kernel = coop == 1 ? LZMA_GPU_KERNEL_COOP : LZMA_GPU_KERNEL_LATENCY;
  }
  o.coop = coop < 0 ? 0u : (coop ? 1u : 2u);
  o.cus = uint32_t(std::max(0, env_int("LZGPU_CUS", 0)));
  o.lanes_per_group = uint32_t(std::max(0, env_int("LZGPU_LANES", 0)));
  o.groups_per_cu = uint32_t(std::max(0, env_int("LZGPU_GROUPS", 0)));
  o.waves_per_simd = uint32_t(std::max(0, env_int("LZGPU_OCC", 0)));
  o.persistent = env_int("LZGPU_PERSIST", 1) ? 0u : 2u;
  o.one_class = env_int("LZGPU_CLASSES", 0) == 1 ? 1u : 0u;
  o.flags = (env_int("LZGPU_SLICE_ALIGN8", 0) ? LZMA_GPU_PLAN_SLICE_ALIGN8 : 0u) |
            (env_int("LZGPU_KERNEL_LZMA2", 0) ? LZMA_GPU_PLAN_KERNEL_LZMA2 : 0u) |
            (env_int("LZGPU_COOP_LAT", 0) ? LZMA_GPU_PLAN_COOP_LAT : 0u) |
            (env_int("LZGPU_MERGE_LAT", 1) ? 0u : LZMA_GPU_PLAN_NO_MERGE_LAT) |
            (env_int("LZGPU_ILV", 1) ? 0u : LZMA_GPU_PLAN_NO_ILV) |
            (env_int("LZGPU_ILV_ANY", 0) ? LZMA_GPU_PLAN_ILV_ANY : 0u) |
            (env_int("LZGPU_THR_FIT", 1) ? 0u : LZMA_GPU_PLAN_NO_THR_FIT) |
            (env_int("LZGPU_SLOTG", 1) ? 0u : LZMA_GPU_PLAN_NO_SLOTG);
  return o;
}

// Launch shape of one LDS class: `stride` cells per stream, `count` streams,
// `cus` CUs.  `regime`: 0 = by the batch (throughput when LDS holds >= 64
// streams per CU and the batch fills them), 1 = throughput shape forced,
// 2 = latency shape (one stream per wave) forced.
static LzmaGpuLdsClass plan_lds_class(uint32_t stride, uint64_t count, uint32_t mask,
                                      uint32_t cus, int regime, const LzmaGpuPlanOptions& o,
                                      bool* latency = nullptr, bool any_groups = false,
                                      bool allow_fit = false) {
  LzmaGpuLdsClass c;
  memset(&c, 0, sizeof c);
  c.lds_mask = mask;
  // Per-lane slice: an odd number of dwords, so that the 32 lanes of a wave
  // reading the same cell index (literal-tree top levels, IsRep of one state)
  // fall in 32 different LDS banks (bank = dword mod 32 for 2- and 4-byte
  // reads); 8-byte aligned slices (158 dwords at lc0/pb0) put lanes l and
  // l + 16 in one bank.  Cells are read 2 or 4 bytes at a time: 4-byte
  // aligned slices suffice.
  if (o.flags & LZMA_GPU_PLAN_SLICE_ALIGN8)
    stride = (stride + 3) & ~3u;
  else
    stride = ((stride + 1) & ~1u) | 2u;  // cells = 2 mod 4: odd dword count
  const uint32_t lds_per_cu = 160 * 1024;
  const uint32_t per_cu = std::max<uint32_t>(1, lds_per_cu / (stride * 2));  // streams/CU
  uint32_t occ = 4;
  const uint32_t occ_over = o.waves_per_simd;
  if (occ_over == 1 || occ_over == 2 || occ_over == 4 || occ_over == 6 || occ_over == 8)
    occ = occ_over;
  // Two regimes (profiles/r01_variants v17-v28):
  //  * throughput -- LDS holds >= 64 streams per CU and the batch fills them:
  //    up to 32 streams per wave with at least 8 waves per CU (64K x 4 KiB:
  //    32 lanes x 8 waves per CU).  A VALU instruction of a wave whose active
  //    lanes all sit in its low half costs one pass whether 16 or 32 lanes are
  //    active, so 32 lanes halve the instructions per stream (ubench:
  //    scripts/ubench/lit_ubench.hip; v38-v41: 24.6 -> 27.0 GB/s with the
  //    checkpoint reader);
  //  * latency -- few streams per CU (small batches, or wide lc+lp tables):
  //    one stream per wave, 16 waves per CU (config 2: 5.8 GB/s vs 2.5 GB/s
  //    with 4 lanes x 4 waves; config 5: 2.6 GB/s vs 2.2 GB/s with 2 lanes).
  // Throughput shapes keep lanes and workgroups per CU powers of two; every
  // count is checked in LDS blocks below (lds_groups_fit).
  auto pow2floor = [](uint32_t v) {
    while (v & (v - 1)) v &= v - 1;
    return v;
  };
  const uint64_t per_cu_batch = (count + cus - 1) / cus;
  const bool thr = regime == 1 || (regime == 0 && per_cu >= 64 && per_cu_batch >= 64);
  uint32_t lanes = 1, groups = 16;
  if (latency) *latency = !thr;
  if (thr) {
    lanes = std::max<uint32_t>(1, std::min<uint32_t>(32, pow2floor(std::max<uint32_t>(1, per_cu / 8))));
    groups = pow2floor(std::max<uint32_t>(1, std::min<uint32_t>(per_cu / lanes, 16)));
  } else {
    // one lane per wave: as many waves as LDS allows -- counted in the CU's
    // 1,280-byte LDS blocks (lzgpu_host::lds_groups_fit) -- up to the 16 the
    // register budget keeps resident.  Round 1's "a power of two, 6 / 10 / 12
    // per CU run 10-30 % slower" was this count taken in bytes: the padded
    // slices of 6, 10, 12 or 15 workgroups do not all fit, the last one waits
    // for the queue to drain (config 5: 15 planned, 14 resident, 5.6 GB/s;
    // 14 planned 7.2, profiles/r05_cfg5groups/)
    groups = std::min<uint32_t>(lzgpu_host::lds_groups_fit(size_t(stride) * 2), 16);
    (void)any_groups;
    // Fitted latency shape (strong-scaling shares, profiles/r03_shares/): a
    // batch of 17-63 streams per CU would run one-stream waves in two or more
    // rounds; widen the waves instead so that every stream is resident at
    // once -- 8,192 x 4 KiB (32 per CU): 2 lanes x 16 waves 5.64 ms vs 7.46 ms
    // in two rounds (and vs 5.95 ms for 4-lane throughput waves).  Only for a
    // batch that is one class (mixed-width batches merge their one-lane
    // classes instead: config 5 4.58 GB/s fitted vs 5.00).
    // LZMA_GPU_PLAN_NO_THR_FIT: the round-2 shape.
    if (allow_fit && !(o.flags & LZMA_GPU_PLAN_NO_THR_FIT) && regime != 2 &&
        per_cu_batch > groups && per_cu_batch < 64 && groups > 0) {
      uint32_t want = uint32_t((per_cu_batch + groups - 1) / groups);
      uint32_t l = 1;
      while (l < want) l <<= 1;
      while (l > 1 && uint64_t(l) * groups > per_cu) l >>= 1;
      lanes = l;
    }
  }
  const uint32_t over = o.lanes_per_group;
  if (over > 0 && over <= 64 && over * stride * 2 <= lds_per_cu) {
    lanes = over;
    groups = pow2floor(std::max<uint32_t>(1, std::min<uint32_t>(per_cu / lanes, 16)));
  }
  if (occ_over) groups = std::min<uint32_t>(groups, 4 * occ);
  // every planned workgroup resident at once, in whole LDS blocks
  const uint32_t fit = lzgpu_host::lds_groups_fit(size_t(lanes) * stride * 2);
  while (groups > 1 && groups > fit) groups = lanes == 1 ? groups - 1 : pow2floor(groups - 1);
  const uint32_t g_over = o.groups_per_cu;
  if (g_over > 0 && g_over <= fit) groups = g_over;
  c.n = count;
  c.lanes_per_group = lanes;
  c.lds_cells_per_lane = stride;
  c.groups_per_cu = std::max<uint32_t>(1, groups);
  // register budget = the waves per SIMD that are actually resident (one
  // wave per workgroup): 8 workgroups per CU -> 2 waves/SIMD -> 256 VGPRs,
  // enough for the decoder state without spills
  c.waves_per_simd = occ_over ? occ : std::max<uint32_t>(1, (c.groups_per_cu + 3) / 4);
  return c;
}

// LDS class of a stream by its table width (cells): narrow tables share a
// launch with many streams per CU, wide ones (lc + lp >= 3) get their own.
static int lds_bucket(uint32_t cells) {
  if (cells <= 768) return 0;
  if (cells <= 1536) return 1;
  if (cells <= 3072) return 2;
  return 3;
}

// cells of an item's whole table (every section in LDS); 0 = bad props
static uint32_t all_cells(const LzmaGpuStreamDesc& d) {
  if (d.kind == LZMA_GPU_KIND_LZMA2) return d.props[0] <= 40 ? lzgpu::table_cells(4, 0, 4) : 0u;
  uint32_t lc, lp, pb, dict;
  if (lzgpu::lz_props_parse(d.props, d.props_size, lc, lp, pb, dict) != SZ_OK) return 0;
  return lzgpu::table_cells(lc, lp, pb);
}

static SRes plan_batch(LzmaGpuStreamDesc* descs, size_t n, uint32_t* order, LzmaGpuPlan* plan,
                       const LzmaGpuPlanOptions& o) {
  if (!order || !plan) return SZ_ERROR_PARAM;
  if (o.kernel > LZMA_GPU_KERNEL_GLOBAL) return SZ_ERROR_PARAM;
  memset(plan, 0, sizeof *plan);
  std::vector<uint32_t> w, w_lat;
  plan->workspace_bytes = plan_workspace(descs, n, &w, &w_lat);
  plan->n = n;
  const uint32_t cus = o.cus ? o.cus : device_cus();
  // LDS-eligible: lo table <= 16384 cells (32 KiB, >= 5 streams per CU)
  const uint32_t kMaxLdsCells = 16384;
  const bool global_only = o.kernel == LZMA_GPU_KERNEL_GLOBAL;
  const bool one_class = o.one_class != 0;
  std::vector<uint32_t> bucket_idx[LZMA_GPU_MAX_CLASSES], glob_idx;
  uint32_t bucket_stride[LZMA_GPU_MAX_CLASSES] = {0, 0, 0, 0};
  for (size_t i = 0; i < n; ++i) {
    if (!global_only && w[i] != 0 && w[i] <= kMaxLdsCells) {
      const int b = one_class ? 0 : lds_bucket(w[i]);
      bucket_idx[b].push_back(uint32_t(i));
      bucket_stride[b] = std::max(bucket_stride[b], w[i]);
    } else {
      glob_idx.push_back(uint32_t(i));
    }
  }
  // Longest work first, and streams of similar work side by side: a wave
  // runs until its slowest lane is done.  Work ~ range-coder decisions, which
  // track the compressed bits (~1.5 decisions per input bit on text), plus a
  // little per output byte for literals writes and match copies.
  auto work = [&](uint32_t i) { return 24 * descs[i].src_len + descs[i].dst_cap; };
  auto by_len = [&](uint32_t a, uint32_t b) {
    const uint64_t wa = work(a), wb = work(b);
    if (wa != wb) return wa > wb;
    return w[a] > w[b];
  };
  // One class per width bucket: the throughput placement first; a class that
  // lands in the latency regime is re-planned with the latency placement (more
  // tables in LDS, few streams per CU); few streams per CU go cooperative.
  // The cooperative kernel is for few streams per CU -- counted over every
  // LDS-eligible stream of the batch, since the classes run side by side and
  // share the CUs (round 6: config 5's 4,096-stream share -- 16 per CU -- was
  // four classes of ~4 per CU, each planned cooperative with the whole CU's
  // LDS to itself and then starved of it when launched together: 246 ms,
  // against 132 ms for 16,384 streams of the same mix)
  size_t lds_total = 0;
  for (int b = 0; b < LZMA_GPU_MAX_CLASSES; ++b) lds_total += bucket_idx[b].size();
  const uint64_t per_cu_lds = (lds_total + cus - 1) / cus;
  auto plan_bucket = [&](const std::vector<uint32_t>& idx, uint32_t stride_lo,
                         bool any_groups, bool allow_fit = false) -> LzmaGpuLdsClass {
    bool lat = false;
    const int regime = o.kernel == LZMA_GPU_KERNEL_THROUGHPUT ? 1 : 0;
    LzmaGpuLdsClass c = plan_lds_class(stride_lo, idx.size(), LZGPU_LDS_MASK, cus, regime, o, &lat);
    const bool want_lat = o.kernel == LZMA_GPU_KERNEL_LATENCY || o.kernel == LZMA_GPU_KERNEL_COOP ||
                          (o.kernel == LZMA_GPU_KERNEL_AUTO && lat);
    if (!want_lat) return c;
    uint32_t stride_lat = 0;
    for (uint32_t i : idx) stride_lat = std::max(stride_lat, w_lat[i]);
    if (stride_lat > kMaxLdsCells) return c;
    c = plan_lds_class(stride_lat, idx.size(), LZGPU_LDS_MASK_LAT, cus,
                       o.kernel == LZMA_GPU_KERNEL_AUTO ? 0 : 2, o, nullptr, any_groups,
                       allow_fit);
    // few streams per CU: the wave-cooperative kernel (all 32 lanes on one
    // stream, copies and direct bits spread over the lanes) -- config 4
    // 1.71 -> 2.85 GB/s and the xz leg 1.45 -> 2.36 at 4 streams per CU;
    // at 16 per CU (config 2) the single-lane waves are faster (5.9 vs 5.2)
    const uint64_t per_cu_batch = (idx.size() + cus - 1) / cus;
    const bool coop = o.kernel == LZMA_GPU_KERNEL_COOP ||
                      (o.kernel == LZMA_GPU_KERNEL_AUTO &&
                       (o.coop == 1 || (o.coop == 0 && per_cu_lds <= 8)));
    if (c.lanes_per_group == 1 && coop) {
      c.lds_mask = LZGPU_LDS_MASK_LAT | lzgpu::kCoopBit;
      if (!(o.flags & LZMA_GPU_PLAN_COOP_LAT)) {
        // the whole table in LDS if it still fits the streams per CU the
        // latency plan gives this class: no global round trip left in the
        // match path (SpecPos, LenHigh) or the matched literal
        uint32_t stride_all = 0;
        for (uint32_t i : idx) stride_all = std::max(stride_all, all_cells(descs[i]));
        if (stride_all != 0 && stride_all <= kMaxLdsCells) {
          LzmaGpuLdsClass ca = plan_lds_class(stride_all, idx.size(),
                                              LZGPU_LDS_MASK_ALL | lzgpu::kCoopBit, cus, 2, o);
          const uint64_t want = std::min<uint64_t>(per_cu_batch, c.groups_per_cu);
          if (ca.lanes_per_group == 1 && ca.groups_per_cu >= want) c = ca;
        }
      }
    }
    // more streams per CU than the widest slice lets resident: the slot trees
    // to the global rows where that fits more one-stream workgroups per CU
    // (config 5: 14 -> 16)
    if (c.lds_mask == LZGPU_LDS_MASK_LAT && c.lanes_per_group == 1 && c.groups_per_cu < 16 &&
        per_cu_batch > c.groups_per_cu && !(o.flags & LZMA_GPU_PLAN_NO_SLOTG)) {
      uint32_t stride_sg = 0;
      for (uint32_t i : idx) stride_sg = std::max(stride_sg, lat_slotg_cells(descs[i]));
      if (stride_sg != 0 && stride_sg <= kMaxLdsCells) {
        const LzmaGpuLdsClass cs =
            plan_lds_class(stride_sg, idx.size(), lzgpu::kLdsMaskLatSlotG, cus,
                           o.kernel == LZMA_GPU_KERNEL_AUTO ? 0 : 2, o, nullptr, any_groups);
        if (cs.lanes_per_group == 1 && cs.groups_per_cu > c.groups_per_cu) c = cs;
      }
    }
    return c;
  };
  // Several buckets in the one-lane latency regime (mixed-props batches,
  // config 5) become one class: its lanes draw from one queue in one launch,
  // so the batch has one tail instead of one per class, and its workgroup
  // count per CU is what the widest slice allows (up to 16, any number: the
  // queue balances the SIMDs) -- config 5 4.6-4.8 -> 4.9 GB/s, and steadier
  // (profiles/r02_ab/cfg5_merge_lat_ab.log).  LZMA_GPU_PLAN_NO_MERGE_LAT keeps
  // one class per bucket.
  int merged = -1;  // the bucket holding the merged latency class
  if (!one_class && !(o.flags & LZMA_GPU_PLAN_NO_MERGE_LAT)) {
    int lat_b[LZMA_GPU_MAX_CLASSES], n_lat = 0;
    for (int b = 0; b < LZMA_GPU_MAX_CLASSES; ++b) {
      if (bucket_idx[b].empty()) continue;
      const LzmaGpuLdsClass c = plan_bucket(bucket_idx[b], bucket_stride[b], false);
      if ((c.lds_mask == LZGPU_LDS_MASK_LAT || c.lds_mask == lzgpu::kLdsMaskLatSlotG) &&
          c.lanes_per_group == 1)
        lat_b[n_lat++] = b;
    }
    if (n_lat >= 2) {
      const int t = lat_b[0];
      for (int j = 1; j < n_lat; ++j) {
        const int b = lat_b[j];
        bucket_idx[t].insert(bucket_idx[t].end(), bucket_idx[b].begin(), bucket_idx[b].end());
        bucket_stride[t] = std::max(bucket_stride[t], bucket_stride[b]);
        bucket_idx[b].clear();
      }
      merged = t;
    }
  }
  int n_buckets = 0;
  for (int b = 0; b < LZMA_GPU_MAX_CLASSES; ++b) n_buckets += bucket_idx[b].empty() ? 0 : 1;
  size_t k = 0;
  uint64_t best = 0;
  std::vector<uint8_t> in_slots;  // items of lane-interleaved classes
  uint64_t slot_total[LZMA_GPU_MAX_CLASSES] = {0, 0, 0, 0};
  for (int b = 0; b < LZMA_GPU_MAX_CLASSES; ++b) {
    if (bucket_idx[b].empty()) continue;
    std::stable_sort(bucket_idx[b].begin(), bucket_idx[b].end(), by_len);
    for (uint32_t i : bucket_idx[b]) order[k++] = i;
    LzmaGpuLdsClass c = plan_bucket(bucket_idx[b], bucket_stride[b], b == merged,
                                    n_buckets == 1);
    if (o.flags & LZMA_GPU_PLAN_KERNEL_LZMA2) c.flags |= LZMA_GPU_CLASS_HAS_LZMA2;
    for (uint32_t i : bucket_idx[b])
      if (descs[i].kind == LZMA_GPU_KIND_LZMA2) {
        c.flags |= LZMA_GPU_CLASS_HAS_LZMA2;
        break;
      }
    const bool ilv_any = (o.flags & LZMA_GPU_PLAN_ILV_ANY) != 0;
    if (!(o.flags & LZMA_GPU_PLAN_NO_ILV) && c.lds_mask == LZGPU_LDS_MASK &&
        (c.lanes_per_group == 32 || c.lanes_per_group == 64 || (ilv_any && c.lanes_per_group <= 64))) {
      // lane-interleaved global sections: one column per resident lane (the
      // lanes keep it across the streams they take from the queue); config 3
      // 28.1 -> 29.9 GB/s (profiles/r02_ilv/ilv_ab.log).  Only for whole lane
      // groups: a narrower workgroup would leave most of every row unused.
      uint32_t rows = 0;
      for (uint32_t i : bucket_idx[b]) {
        const LzmaGpuStreamDesc& d = descs[i];
        uint32_t lc = 4, lp = 0, pb = 4, dict;
        if (d.kind != LZMA_GPU_KIND_LZMA2 &&
            lzgpu::lz_props_parse(d.props, d.props_size, lc, lp, pb, dict) != SZ_OK)
          continue;
        rows = std::max(rows, lzgpu::make_layout(lc, lp, pb, LZGPU_LDS_MASK).glb_cells);
      }
      const uint64_t grid = (c.n + c.lanes_per_group - 1) / c.lanes_per_group;
      const uint64_t groups =
          o.persistent == 2 ? grid : std::min<uint64_t>(grid, uint64_t(cus) * c.groups_per_cu);
      const uint64_t lane_groups = (c.lanes_per_group + lzgpu::kIlv - 1) / lzgpu::kIlv;
      c.slot_cells = std::max<uint32_t>((rows + 1) & ~1u, 2);  // even: pairs of cells
      c.slot_groups = uint32_t(groups);
      slot_total[plan->n_classes] = groups * lane_groups * lzgpu::kIlv * c.slot_cells;
      c.lds_mask |= lzgpu::kIlvBit;
      if (in_slots.empty()) in_slots.assign(n, 0);
      for (uint32_t i : bucket_idx[b]) in_slots[i] = 1;
    }
    plan->classes[plan->n_classes++] = c;
    plan->n_lds += c.n;
    if (c.n > best) {
      best = c.n;
      plan->lanes_per_group = c.lanes_per_group;
      plan->lds_cells_per_lane = c.lds_cells_per_lane;
      plan->groups_per_cu = c.groups_per_cu;
      plan->waves_per_simd = c.waves_per_simd;
    }
  }
  std::stable_sort(glob_idx.begin(), glob_idx.end(), by_len);
  for (uint32_t i : glob_idx) order[k++] = i;
  plan->persistent = o.persistent == 2 ? 0u : 1u;
  // per-stream slices only for items outside the slot areas, then the slot
  // areas (128-byte aligned), then the LDS launches' work counters
  uint64_t ws_cells = plan->workspace_bytes / 2;
  if (!in_slots.empty()) ws_cells = plan_workspace(descs, n, nullptr, nullptr, &in_slots) / 2;
  for (uint32_t c = 0; c < plan->n_classes; ++c) {
    if (!slot_total[c]) continue;
    ws_cells = (ws_cells + 63) & ~uint64_t(63);
    plan->classes[c].slot_off = ws_cells;
    ws_cells += slot_total[c];
  }
  plan->workspace_bytes = ws_cells * 2;
  plan->queue_offset = (plan->workspace_bytes + 63) & ~uint64_t(63);
  plan->workspace_bytes = plan->queue_offset + 64 * LZMA_GPU_MAX_CLASSES;
  return SZ_OK;
}

// C ABI: no exception crosses it (host allocation failure -> SZ_ERROR_MEM).
static SRes plan_batch_nothrow(LzmaGpuStreamDesc* descs, size_t n, uint32_t* order,
                               LzmaGpuPlan* plan, const LzmaGpuPlanOptions& o) {
  try {
    return plan_batch(descs, n, order, plan, o);
  } catch (const std::exception&) {
    set_error("plan: host allocation failed");
    return SZ_ERROR_MEM;
  }
}

SRes LzmaGpu_PlanBatchEx(LzmaGpuStreamDesc* descs, size_t n, uint32_t* order,
                         LzmaGpuPlan* plan) {
  return plan_batch_nothrow(descs, n, order, plan, env_options());
}

SRes LzmaGpu_PlanBatchOpt(LzmaGpuStreamDesc* descs, size_t n, uint32_t* order, LzmaGpuPlan* plan,
                          const LzmaGpuPlanOptions* opt) {
  if (opt && (opt->flags & ~LZMA_GPU_PLAN_KNOWN_FLAGS)) return SZ_ERROR_PARAM;
  return plan_batch_nothrow(descs, n, order, plan, opt ? *opt : env_options());
}

// Internal streams for concurrent class launches: a pool per device, guarded
// by a mutex.  A call takes a set for the duration of its enqueueing and puts
// it back; sets are created only when every existing one is taken, so the
// pool grows to the number of threads that enqueue batches at the same time,
// not to the number of threads that ever did.  Reusing a set from another
// thread is safe: work on its streams only orders behind earlier work, and a
// wait on an event captures the event's state at the time of the wait.
struct ClassStreams {
  hipStream_t s[LZMA_GPU_MAX_CLASSES] = {};
  hipEvent_t fork = nullptr, join[LZMA_GPU_MAX_CLASSES] = {};
  int dev = 0;
};
static void destroy_class_streams(ClassStreams* c) {
  if (!c) return;
  for (int k = 0; k < LZMA_GPU_MAX_CLASSES; ++k) {
    if (c->s[k]) (void)hipStreamDestroy(c->s[k]);
    if (c->join[k]) (void)hipEventDestroy(c->join[k]);
  }
  if (c->fork) (void)hipEventDestroy(c->fork);
  delete c;
}
struct ClassStreamPool {
  std::mutex mu;
  std::vector<ClassStreams*> free_sets[kLzgpuMaxDevices];
};
static ClassStreamPool& class_stream_pool() {
  static ClassStreamPool* p = new ClassStreamPool();  // process lifetime (HIP teardown order)
  return *p;
}
static ClassStreams* class_streams_acquire() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kLzgpuMaxDevices) return nullptr;
  ClassStreamPool& P = class_stream_pool();
  {
    std::lock_guard<std::mutex> g(P.mu);
    if (!P.free_sets[dev].empty()) {
      ClassStreams* c = P.free_sets[dev].back();
      P.free_sets[dev].pop_back();
      return c;
    }
  }
  ClassStreams* c = new (std::nothrow) ClassStreams();
  if (!c) return nullptr;
  c->dev = dev;
  bool ok = hipEventCreateWithFlags(&c->fork, hipEventDisableTiming) == hipSuccess;
  for (int k = 0; k < LZMA_GPU_MAX_CLASSES && ok; ++k)
    ok = hipStreamCreateWithFlags(&c->s[k], hipStreamNonBlocking) == hipSuccess &&
         hipEventCreateWithFlags(&c->join[k], hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    destroy_class_streams(c);  // whatever part of the set was created
    (void)hipGetLastError();
    return nullptr;
  }
  return c;
}
static void class_streams_release(ClassStreams* c) {
  if (!c) return;
  ClassStreamPool& P = class_stream_pool();
  std::lock_guard<std::mutex> g(P.mu);
  try {
    P.free_sets[c->dev].push_back(c);
  } catch (const std::exception&) {
    destroy_class_streams(c);
  }
}

SRes LzmaGpu_DecodeBatchEx(const LzmaGpuPlan* plan, const LzmaGpuStreamDesc* d_descs,
                           const uint32_t* d_order, const Byte* d_src, Byte* d_dst,
                           void* d_workspace, LzmaGpuResult* d_results, void* stream) {
  if (!ensure_device()) return SZ_ERROR_FAIL;
  if (!plan || !d_order || plan->n > 0xFFFFFFFFull || plan->n_lds > plan->n ||
      plan->n_classes > LZMA_GPU_MAX_CLASSES)
    return SZ_ERROR_PARAM;
  hipStream_t st = static_cast<hipStream_t>(stream);
  uint16_t* ws = static_cast<uint16_t*>(d_workspace);
  const uint32_t cus = device_cus();
  // Several width classes (mixed lc/lp/pb batches, config 5): each class is a
  // persistent launch whose workgroups leave only when its queue is drained,
  // so on one stream every class ends in a tail of a few long streams while
  // the rest of the chip idles.  On their own streams (forked from and joined
  // back into the caller's) the next class's workgroups fill the CUs the
  // previous one frees.  LZGPU_CLASS_STREAMS=0: one stream (A/B).
  uint32_t live = 0;
  for (uint32_t k = 0; k < plan->n_classes; ++k) live += plan->classes[k].n ? 1u : 0u;
  {
    uint64_t sum = 0;
    for (uint32_t k = 0; k < plan->n_classes; ++k) sum += plan->classes[k].n;
    if (sum > plan->n_lds) return SZ_ERROR_PARAM;
  }
  const bool fork = live > 1 && env_int("LZGPU_CLASS_STREAMS", 1) != 0;
  // concurrent classes are a speed-up only: without a stream set (resource
  // exhaustion) the classes run one after another on the caller's stream
  ClassStreams* cs = fork ? class_streams_acquire() : nullptr;
  if (cs && hipEventRecord(cs->fork, st) != hipSuccess) {
    (void)hipGetLastError();
    class_streams_release(cs);
    cs = nullptr;
  }
  SRes ret = SZ_OK;
  uint64_t first = 0;
  for (uint32_t k = 0; k < plan->n_classes && ret == SZ_OK; ++k) {
    const LzmaGpuLdsClass& c = plan->classes[k];
    if (c.n == 0) continue;
    const uint32_t max_groups = plan->persistent ? cus * c.groups_per_cu : 0u;
    uint32_t* queue = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(d_workspace) +
                                                  plan->queue_offset + 64 * k);
    hipStream_t sk = st;
    if (cs) {
      sk = cs->s[k];
      if (!hip_ok(hipStreamWaitEvent(sk, cs->fork, 0), "class fork")) {
        ret = SZ_ERROR_FAIL;
        break;
      }
    }
    if (lzgpu_launch_decode_lds(d_descs, d_order + first, uint32_t(c.n), d_src, d_dst, ws,
                                d_results, c.lanes_per_group, c.lds_cells_per_lane,
                                c.waves_per_simd, c.groups_per_cu, max_groups, queue, c.lds_mask,
                                c.flags, LzgpuSlots{c.slot_off, c.slot_cells, c.slot_groups},
                                sk) != 0) {
      set_error("LDS decode kernel launch failed");
      ret = SZ_ERROR_FAIL;
      break;
    }
    if (cs && (!hip_ok(hipEventRecord(cs->join[k], sk), "class join") ||
               !hip_ok(hipStreamWaitEvent(st, cs->join[k], 0), "class join"))) {
      ret = SZ_ERROR_FAIL;
      break;
    }
    first += c.n;
  }
  class_streams_release(cs);
  if (ret != SZ_OK) return ret;
  const uint32_t n_lds = uint32_t(plan->n_lds), n_glob = uint32_t(plan->n - plan->n_lds);
  if (n_glob && lzgpu_launch_decode_batch(d_descs, d_order + n_lds, n_glob, d_src, d_dst, ws,
                                          d_results, st) != 0) {
    set_error("generic decode kernel launch failed");
    return SZ_ERROR_FAIL;
  }
  return SZ_OK;
}

SRes LzmaGpu_DecodeBatch(const LzmaGpuStreamDesc* d_descs, const uint32_t* d_order, size_t n,
                         const Byte* d_src, Byte* d_dst, void* d_workspace, size_t workspace_bytes,
                         LzmaGpuResult* d_results, void* stream) {
  (void)workspace_bytes;
  if (!ensure_device()) return SZ_ERROR_FAIL;
  if (n > 0xFFFFFFFFull) return SZ_ERROR_PARAM;
  if (lzgpu_launch_decode_batch(d_descs, d_order, uint32_t(n), d_src, d_dst,
                                static_cast<uint16_t*>(d_workspace), d_results,
                                static_cast<hipStream_t>(stream)) != 0) {
    set_error("batch kernel launch failed");
    return SZ_ERROR_FAIL;
  }
  return SZ_OK;
}

static SRes decode_batch_host(const LzmaGpuStreamDesc* descs, size_t n, const Byte* src,
                              size_t src_bytes, Byte* dst, size_t dst_bytes,
                              LzmaGpuResult* results, const LzmaGpuPlanOptions* opt,
                              LzmaGpuPlan* plan_out) {
  if (!ensure_device()) return SZ_ERROR_FAIL;
  if (n == 0) return SZ_OK;
  std::vector<LzmaGpuStreamDesc> d(descs, descs + n);
  std::vector<uint32_t> order(n);
  LzmaGpuPlan plan;
  {
    const SRes pr = LzmaGpu_PlanBatchOpt(d.data(), n, order.data(), &plan, opt);
    if (pr != SZ_OK) return pr;
  }
  if (plan_out) *plan_out = plan;
  const size_t ws = size_t(plan.workspace_bytes);
  void *d_src = nullptr, *d_dst = nullptr, *d_ws = nullptr, *d_desc = nullptr, *d_order = nullptr,
       *d_res = nullptr;
  SRes r = SZ_ERROR_MEM;
  do {
    if (!hip_ok(hipMalloc(&d_src, std::max<size_t>(src_bytes, 16)), "alloc src")) break;
    if (!hip_ok(hipMalloc(&d_dst, std::max<size_t>(dst_bytes, 16)), "alloc dst")) break;
    if (!hip_ok(hipMalloc(&d_ws, std::max<size_t>(ws, 16)), "alloc workspace")) break;
    if (!hip_ok(hipMalloc(&d_desc, n * sizeof(LzmaGpuStreamDesc)), "alloc desc")) break;
    if (!hip_ok(hipMalloc(&d_order, n * sizeof(uint32_t)), "alloc order")) break;
    if (!hip_ok(hipMalloc(&d_res, n * sizeof(LzmaGpuResult)), "alloc results")) break;
    r = SZ_ERROR_FAIL;
    if (src_bytes && !hip_ok(hipMemcpy(d_src, src, src_bytes, hipMemcpyHostToDevice), "H2D src"))
      break;
    if (!hip_ok(hipMemcpy(d_desc, d.data(), n * sizeof(LzmaGpuStreamDesc), hipMemcpyHostToDevice),
                "H2D desc"))
      break;
    if (!hip_ok(hipMemcpy(d_order, order.data(), n * sizeof(uint32_t), hipMemcpyHostToDevice),
                "H2D order"))
      break;
    if (LzmaGpu_DecodeBatchEx(&plan, static_cast<LzmaGpuStreamDesc*>(d_desc),
                              static_cast<uint32_t*>(d_order), static_cast<Byte*>(d_src),
                              static_cast<Byte*>(d_dst), d_ws, static_cast<LzmaGpuResult*>(d_res),
                              nullptr) != SZ_OK)
      break;
    if (!hip_ok(hipDeviceSynchronize(), "decode kernel")) break;
    if (!hip_ok(hipMemcpy(results, d_res, n * sizeof(LzmaGpuResult), hipMemcpyDeviceToHost),
                "D2H results"))
      break;
    if (dst_bytes && !hip_ok(hipMemcpy(dst, d_dst, dst_bytes, hipMemcpyDeviceToHost), "D2H dst"))
      break;
    r = SZ_OK;
  } while (0);
  (void)hipFree(d_src);
  (void)hipFree(d_dst);
  (void)hipFree(d_ws);
  (void)hipFree(d_desc);
  (void)hipFree(d_order);
  (void)hipFree(d_res);
  return r;
}

SRes LzmaGpu_DecodeBatchHostOpt(const LzmaGpuStreamDesc* descs, size_t n, const Byte* src,
                                size_t src_bytes, Byte* dst, size_t dst_bytes,
                                LzmaGpuResult* results, const LzmaGpuPlanOptions* opt,
                                LzmaGpuPlan* plan_out) {
  try {
    return decode_batch_host(descs, n, src, src_bytes, dst, dst_bytes, results, opt, plan_out);
  } catch (const std::exception&) {
    set_error("batch: host allocation failed");
    return SZ_ERROR_MEM;
  }
}

SRes LzmaGpu_DecodeBatchHost(const LzmaGpuStreamDesc* descs, size_t n, const Byte* src,
                             size_t src_bytes, Byte* dst, size_t dst_bytes,
                             LzmaGpuResult* results) {
  return LzmaGpu_DecodeBatchHostOpt(descs, n, src, src_bytes, dst, dst_bytes, results, nullptr,
                                    nullptr);
}

size_t Lzma2Gpu_SplitBlocks(const Byte* src, size_t src_len, uint64_t* src_off,
                            uint64_t* block_src_len, uint64_t* unpack, size_t max_blocks) {
  size_t pos = 0, nb = 0;
  uint64_t cur_unpack = 0;
  bool open = false;
  auto close_block = [&](size_t end) {
    if (open && nb - 1 < max_blocks) {
      block_src_len[nb - 1] = end - src_off[nb - 1];
      unpack[nb - 1] = cur_unpack;
    }
  };
  while (pos < src_len) {
    const Byte c = src[pos];
    if (c == 0) {
      close_block(pos);
      return nb;
    }
    const bool is_lzma = (c & 0x80) != 0;
    if (!is_lzma && c > 2) return size_t(-1);
    const bool reset = (c == 1) || (c >= 0xE0);
    if (reset) {
      close_block(pos);
      if (nb < max_blocks) src_off[nb] = pos;
      nb++;
      open = true;
      cur_unpack = 0;
    } else if (!open) {
      return size_t(-1);  // stream must start with a dictionary reset
    }
    if (is_lzma) {
      if (pos + 5 > src_len) return size_t(-1);
      const uint64_t u = (uint64_t(c & 0x1F) << 16) + (uint64_t(src[pos + 1]) << 8) + src[pos + 2] + 1;
      const uint64_t pk = (uint64_t(src[pos + 3]) << 8) + src[pos + 4] + 1;
      const size_t hdr = (((c >> 5) & 3) >= 2) ? 6 : 5;
      cur_unpack += u;
      pos += hdr + pk;
    } else {
      if (pos + 3 > src_len) return size_t(-1);
      const uint64_t u = (uint64_t(src[pos + 1]) << 8) + src[pos + 2] + 1;
      cur_unpack += u;
      pos += 3 + u;
    }
  }
  if (pos > src_len) return size_t(-1);
  close_block(src_len);  // no EOS byte: the last block runs to the end
  return nb;
}

// ------------------------------------------------------------------ streaming sessions

static_assert(sizeof(LzmaGpuSession) == 192, "LzmaGpuSession layout");
static_assert(sizeof(LzmaGpuPlan) == 248, "LzmaGpuPlan layout");

size_t LzmaGpu_SessionProbsBytes(const Byte* props, unsigned propsSize) {
  CLzmaProps pr;
  if (LzmaProps_Decode(&pr, props, propsSize) != SZ_OK) return 0;
  return size_t(lzgpu::table_cells(pr.lc, pr.lp, pr.pb)) * 2;
}

SRes LzmaGpu_SessionInit(LzmaGpuSession* s, const Byte* props, unsigned propsSize,
                         uint16_t* d_probs, Byte* d_dic, size_t dic_buf_size) {
  if (!s) return SZ_ERROR_PARAM;
  CLzmaProps pr;
  const SRes r = LzmaProps_Decode(&pr, props, propsSize);
  if (r != SZ_OK) return r;
  if (!d_probs || !d_dic || dic_buf_size == 0) return SZ_ERROR_PARAM;
  memset(s, 0, sizeof *s);
  s->lc = pr.lc;
  s->lp = pr.lp;
  s->pb = pr.pb;
  s->dict_size = pr.dicSize;
  s->probs = d_probs;
  s->dic = d_dic;
  s->dic_buf_size = dic_buf_size;
  // LzmaDec_Init (LzmaDec.c:701-705): dicPos = 0, InitDicAndState(True, True)
  s->dic_pos = 0;
  s->need_flush = 1;
  s->remain_len = 0;
  s->temp_buf_size = 0;
  s->processed_pos = 0;
  s->check_dic_size = 0;
  s->need_init_state = 1;
  return SZ_OK;
}

SRes LzmaGpu_SessionDecodeBatch(LzmaGpuSession* d_sessions, size_t n, void* stream) {
  if (!ensure_device()) return SZ_ERROR_FAIL;
  if (n > 0xFFFFFFFFull) return SZ_ERROR_PARAM;
  if (lzgpu_launch_session(d_sessions, uint32_t(n), static_cast<hipStream_t>(stream)) != 0) {
    set_error("session kernel launch failed");
    return SZ_ERROR_FAIL;
  }
  return SZ_OK;
}

// ------------------------------------------------------------------ CRC-32

size_t CrcGpu_PlanChunks(const uint64_t* caps, size_t n, uint32_t* chunk_base,
                         uint32_t* chunk_range) {
  uint64_t total = 0;
  for (size_t i = 0; i < n; ++i) {
    const uint64_t c = (caps[i] + lzgpu::kCrcChunk - 1) / lzgpu::kCrcChunk;
    if (total + c > 0xFFFFFFFFull) return size_t(-1);
    if (chunk_base) chunk_base[i] = uint32_t(total);
    if (chunk_range)
      for (uint64_t k = 0; k < c; ++k) chunk_range[total + k] = uint32_t(i);
    total += c;
  }
  return size_t(total);
}

size_t LzmaGpu_Crc32Plan(const LzmaGpuStreamDesc* descs, size_t n, uint32_t* chunk_base,
                         uint32_t* chunk_range) {
  uint64_t total = 0;
  for (size_t i = 0; i < n; ++i) {
    const uint64_t c = (descs[i].dst_cap + lzgpu::kCrcChunk - 1) / lzgpu::kCrcChunk;
    if (total + c > 0xFFFFFFFFull) return size_t(-1);
    if (chunk_base) chunk_base[i] = uint32_t(total);
    if (chunk_range)
      for (uint64_t k = 0; k < c; ++k) chunk_range[total + k] = uint32_t(i);
    total += c;
  }
  return size_t(total);
}

SRes CrcGpu_Batch(const Byte* d_data, const uint64_t* d_off, const uint64_t* d_len, size_t n,
                  const uint32_t* d_chunk_base, const uint32_t* d_chunk_range, size_t n_chunks,
                  uint32_t init, uint32_t xorout, uint32_t* d_chunk_crc, uint32_t* d_crc,
                  void* stream) {
  if (!ensure_device()) return SZ_ERROR_FAIL;
  if (n > 0xFFFFFFFFull || n_chunks > 0xFFFFFFFFull) return SZ_ERROR_PARAM;
  if (lzgpu_launch_crc_arrays(d_data, d_off, d_len, uint32_t(n), d_chunk_base, d_chunk_range,
                              uint32_t(n_chunks), init, xorout, d_chunk_crc, d_crc,
                              static_cast<hipStream_t>(stream)) != 0) {
    set_error("CRC kernel launch failed");
    return SZ_ERROR_FAIL;
  }
  return SZ_OK;
}

SRes LzmaGpu_Crc32Batch(const LzmaGpuStreamDesc* d_descs, const LzmaGpuResult* d_results,
                        size_t n, const Byte* d_dst, const uint32_t* d_chunk_base,
                        const uint32_t* d_chunk_range, size_t n_chunks, uint32_t* d_chunk_crc,
                        uint32_t* d_crc, void* stream) {
  if (!ensure_device()) return SZ_ERROR_FAIL;
  if (n > 0xFFFFFFFFull || n_chunks > 0xFFFFFFFFull) return SZ_ERROR_PARAM;
  if (lzgpu_launch_crc_decoded(d_descs, d_results, d_dst, uint32_t(n), d_chunk_base,
                               d_chunk_range, uint32_t(n_chunks), d_chunk_crc, d_crc,
                               static_cast<hipStream_t>(stream)) != 0) {
    set_error("CRC kernel launch failed");
    return SZ_ERROR_FAIL;
  }
  return SZ_OK;
}

// 7zCrc.h drop-ins over host buffers (upload + the batch kernels, n = 1).
// They cannot report errors; without a device they print once and return 0.
void CrcGenerateTable(void) {}  // tables are compile-time constants on the device

static uint32_t crc_host_one(uint32_t init, const void* data, size_t size, uint32_t xorout) {
  if (!ensure_device()) return 0;
  if (size == 0) return init ^ xorout;
  lzgpu_host::CallScratch* S = lzgpu_host::scratch_acquire();
  if (!S) return 0;
  const uint64_t cap = size;
  const size_t nch = CrcGpu_PlanChunks(&cap, 1, nullptr, nullptr);
  // one upload: [offset, length | chunk base | chunk ranges]
  std::vector<uint32_t> meta(4 + 1 + nch, 0);
  meta[2] = uint32_t(cap);
  meta[3] = uint32_t(cap >> 32);
  CrcGpu_PlanChunks(&cap, 1, meta.data() + 4, meta.data() + 5);
  uint8_t* d_data = static_cast<uint8_t*>(S->buf[0].get(size));
  uint8_t* d_meta = static_cast<uint8_t*>(S->buf[1].get(4 * meta.size() + 8));
  uint32_t* d_chunks = static_cast<uint32_t*>(S->buf[2].get(4 * (nch + 1)));
  uint32_t out = 0;
  const hipStream_t st = S->stream;
  if (!d_data || !d_meta || !d_chunks) {
    set_error("CRC: device allocation failed");
  } else {
    uint64_t* d_ol = reinterpret_cast<uint64_t*>(d_meta);
    uint32_t* d_base = reinterpret_cast<uint32_t*>(d_meta + 16);
    uint32_t* d_crc = reinterpret_cast<uint32_t*>(d_meta + 4 * meta.size());
    if (hip_ok(hipMemcpyAsync(d_data, data, size, hipMemcpyHostToDevice, st), "CRC H2D") &&
        hip_ok(hipMemcpyAsync(d_meta, meta.data(), 4 * meta.size(), hipMemcpyHostToDevice, st),
               "CRC H2D") &&
        lzgpu_launch_crc_arrays(d_data, d_ol, d_ol + 1, 1, d_base, d_base + 1, uint32_t(nch), init,
                                xorout, d_chunks, d_crc, st) == 0 &&
        hip_ok(hipMemcpyAsync(&out, d_crc, 4, hipMemcpyDeviceToHost, st), "CRC D2H") &&
        hip_ok(hipStreamSynchronize(st), "CRC kernel")) {
    } else {
      out = 0;
    }
  }
  (void)hipStreamSynchronize(st);  // host buffers are reused after return
  lzgpu_host::scratch_release(S);
  return out;
}

UInt32 CrcUpdate(UInt32 v, const void* data, size_t size) { return crc_host_one(v, data, size, 0); }

UInt32 CrcCalc(const void* data, size_t size) {
  return crc_host_one(0xFFFFFFFFu, data, size, 0xFFFFFFFFu);
}

int LzmaGpu_DeviceCount(void) { return device_count(); }

const char* LzmaGpu_LastError(void) { return g_last_error.c_str(); }

const char* LzmaGpu_Version(void) { return "liblzmagpu 0.1 (gfx950, LZMA SDK 9.20 decoder contract)"; }

}  // extern "C"

namespace lzgpu_host {
bool ensure_device() { return ::ensure_device(); }
void set_error(const char* what) { ::set_error(what); }
bool hip_ok(hipError_t e, const char* what) { return ::hip_ok(e, what); }
uint32_t device_cus() { return ::device_cus(); }

namespace {
struct ScratchPool {
  std::mutex mu;
  std::vector<CallScratch*> free_sets[kLzgpuMaxDevices];
};
ScratchPool& scratch_pool() {
  static ScratchPool* p = new ScratchPool();  // process lifetime (HIP teardown order)
  return *p;
}
}  // namespace

CallScratch* scratch_acquire() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kLzgpuMaxDevices) {
    ::set_error("scratch: no current device");
    return nullptr;
  }
  ScratchPool& P = scratch_pool();
  {
    std::lock_guard<std::mutex> g(P.mu);
    if (!P.free_sets[dev].empty()) {
      CallScratch* s = P.free_sets[dev].back();
      P.free_sets[dev].pop_back();
      return s;
    }
  }
  CallScratch* s = new (std::nothrow) CallScratch();
  if (!s) {
    ::set_error("scratch: host allocation failed");
    return nullptr;
  }
  s->dev = dev;
  if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) {
    (void)hipGetLastError();
    ::set_error("scratch: stream creation failed");
    delete s;
    return nullptr;
  }
  return s;
}

uint8_t* scratch_pinned(CallScratch* s, size_t n) {
  if (!s || n > kPinnedStageMax) return nullptr;
  if (s->pin_cap >= n) return s->pin;
  const size_t want = std::min(kPinnedStageMax, std::max({n, s->pin_cap * 2, size_t(256) << 10}));
  if (s->pin) (void)hipHostFree(s->pin);
  s->pin = nullptr;
  s->pin_cap = 0;
  if (hipHostMalloc(reinterpret_cast<void**>(&s->pin), want, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    s->pin = nullptr;
    return nullptr;
  }
  s->pin_cap = want;
  return s->pin;
}

void scratch_release(CallScratch* s) {
  if (!s) return;
  ScratchPool& P = scratch_pool();
  std::lock_guard<std::mutex> g(P.mu);
  try {
    P.free_sets[s->dev].push_back(s);
  } catch (const std::exception&) {
    (void)hipStreamDestroy(s->stream);
    if (s->pin) (void)hipHostFree(s->pin);
    delete s;
  }
}
}  // namespace lzgpu_host

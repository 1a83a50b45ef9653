// dropin_capi.hip -- the drop-in decoder symbols of LzmaDec.h, LzmaLib.h and
// Lzma2Dec.h (include/lzma_gpu.h part 1).
//
// Every decode runs on the GPU.  What stays on the host is what the reference
// keeps outside its decoder loop: property parsing (LzmaDec.c:898-922),
// ISzAlloc bookkeeping (LzmaDec.c:880-970) and the LZMA2 chunk-header walk of
// the streaming interface (Lzma2Dec.c:170-328), whose LZMA chunks are decoded by
// the GPU LzmaDec_DecodeToDic.
//
// One-call decodes (LzmaDecode, LzmaUncompress, Lzma2Decode) are one-item
// batches planned onto the wave-cooperative kernel (whole table in LDS where it
// fits): upload the compressed bytes, decode, download the output.
//
// The dictionary interface keeps a DEVICE MIRROR per decoder object (keyed by
// the CLzmaDec address, its dic / dicBufSize / probs and the device): the
// dictionary, the probability table and the session state stay on the GPU
// between calls, so a call uploads only its input (plus, once per mirror, the
// history a continuing decoder needs) and downloads only the bytes it decoded,
// the ~200-byte state and the table.  The 7zDec pattern (16 KiB look windows over
// a whole-folder dic, 7zDec.c:133-171) is therefore linear in the folder size;
// round 2 re-uploaded the whole dicBufSize every call.  DecodeToBuf runs its
// whole ring loop (LzmaDec.c:840-878) in ONE launch on the device ring and
// downloads the caller's output once; the host ring is rebuilt from it.
//
// Coherence with a caller that writes `dic` itself (round 4): the reference's
// dictionary IS the caller's buffer, and its own LZMA2 walker copies stored
// chunks into it and advances dicPos / processedPos between decoder calls
// (Lzma2Dec.c:159-166, 234).  Every call therefore compares the decoder's
// positions on entry with the ones the previous call left behind: equal (or
// dicPos wrapped from dicBufSize to 0, LzmaDec.c:849) -- nothing to do; both
// advanced by the same amount -- the host wrote exactly those bytes, which are
// uploaded (ring-wrapped spans in two pieces); anything else -- the mirror's
// history is dropped and the whole dictionary is uploaded again when the call
// reads history.  The table is checked the same way (a 64-bit hash of the host
// cells against the one recorded after the previous call).  What stays out of
// reach is a caller rewriting bytes it already handed to the decoder without
// moving the positions; no caller in the reference does that
// (INTEGRATION.md §2).  A decoder used on another device drops its mirrors on
// every other device, so switching devices back and forth never decodes on a
// stale table or dictionary.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <memory>
#include <mutex>
#include <new>
#include <vector>

#include "lzma_device.h"
#include "lzma_gpu_internal.h"

using lzgpu_host::CallScratch;
using lzgpu_host::DevBuf;
using lzgpu_host::ensure_device;
using lzgpu_host::hip_ok;
using lzgpu_host::set_error;

namespace {

uint32_t probs_for(uint32_t lc, uint32_t lp) { return lzgpu::num_probs(lc, lp); }

// PCIe bytes moved by the drop-in entry points (LzmaGpu_DropinTransferStats):
// the evidence that the dictionary interface uploads its input, not its
// dictionary, per call
std::atomic<uint64_t> g_h2d{0}, g_d2h{0}, g_calls{0};

hipError_t xfer(void* dst, const void* src, size_t n, hipMemcpyKind kind, hipStream_t st) {
  if (kind == hipMemcpyHostToDevice) g_h2d += n;
  if (kind == hipMemcpyDeviceToHost) g_d2h += n;
  return hipMemcpyAsync(dst, src, n, kind, st);
}

// RAII borrow of a pooled call scratch (buffers + its own stream)
struct ScratchLease {
  CallScratch* s = lzgpu_host::scratch_acquire();
  ~ScratchLease() {
    if (s) {
      (void)hipStreamSynchronize(s->stream);
      lzgpu_host::scratch_release(s);
    }
  }
};

// ------------------------------------------------------------------ one-call decodes

// ------------------------------------------------------------------ coalesced one-call decodes
//
// One-call decodes (LzmaDecode, LzmaUncompress, Lzma2Decode) made by several
// host threads at once share launches -- group commit: a call joins its
// device's pending list; if one of the device's batch sets is free it takes
// the whole list and runs it as ONE batch (inputs packed into pinned staging,
// one upload, one plan + launch, one download of results and outputs),
// otherwise it waits, and the calls that arrive while the sets are busy form
// the next batch.  An
// unchanged multi-threaded caller (the reference's LzmaDecode / LzmaUncompress
// are reentrant, LzmaDec.c:972-1002, LzmaLib.c:41-46) therefore reaches the
// batch planner and its throughput / latency kernels; a lone caller pays
// nothing extra (its batch has one item, planned onto the wave-cooperative
// kernel as before, and starts at once).  LZGPU_COALESCE=0 gives every call its
// own launch.
struct OneCall {
  uint8_t kind = 0;
  const Byte* src = nullptr;
  SizeT in_size = 0;
  Byte* dest = nullptr;
  SizeT out_size = 0;
  Byte props[LZMA_PROPS_SIZE] = {};
  uint8_t props_size = 0;
  uint8_t finish = 0;
  LzmaGpuResult r = {};
  SRes err = SZ_OK;       // infrastructure failure of the batch (else r.res)
  const char* msg = "";   // its message (static text)
  bool taken = false;     // in a batch (running or done)
  bool done = false;
  std::condition_variable cv;  // its caller sleeps here (group_commit)
};

// The resources of one batch in flight: pinned staging (inputs | descriptors +
// order | results | outputs), device buffers and a stream of its own.
struct BatchSet {
  uint8_t* pin = nullptr;
  size_t pin_cap = 0;
  DevBuf io, ws, meta;
  hipStream_t stream = nullptr;
  bool busy = false;
  bool broken = false;  // its stream could not be created: not picked (group_commit)
};

// Batches in flight per device at once (LZGPU_COALESCE_INFLIGHT=1..8, default
// 4: GPU_MAX_HW_QUEUES is 4).  A lone 4 KiB call is one wave's serial decode
// (2.3 ms of its 2.4, profiles/r05_coalesce/), so with one batch at a time the
// callers that arrive during it all wait for it to end; with several sets the
// next leader launches at once and the batches share the chip (a one-wave
// batch leaves the rest of every CU idle).
constexpr int kMaxInFlight = 8;
int in_flight_limit() {
  static const int n = [] {
    const char* e = getenv("LZGPU_COALESCE_INFLIGHT");
    const int v = e ? atoi(e) : 4;
    return v < 1 ? 1 : (v > kMaxInFlight ? kMaxInFlight : v);
  }();
  return n;
}

struct Coalescer {
  std::mutex mu;
  std::vector<OneCall*> pending;
  BatchSet sets[kMaxInFlight];
  uint32_t in_flight = 0;  // calls in running batches
  std::atomic<uint32_t> callers{0};  // threads inside a call (ActiveCall)
  std::atomic<uint64_t> batches{0}, items{0}, max_items{0};
};

// Counts a thread as inside a drop-in call for its whole duration, host work
// before and after its launch included (the concurrency gate of free_set).
struct ActiveCall {
  std::atomic<uint32_t>* n;
  explicit ActiveCall(std::atomic<uint32_t>* c) : n(c) {
    if (n) ++*n;
  }
  ~ActiveCall() {
    if (n) --*n;
  }
  ActiveCall(const ActiveCall&) = delete;
  ActiveCall& operator=(const ActiveCall&) = delete;
};

// Group commit, shared by the one-call and the session coalescers (C: mu,
// pending, sets[], in_flight and the counters; Call: taken, done, cv).  A
// pending call leads when a batch set is free and no batch runs, or fewer
// than budget / 2 calls are active -- threads inside a call, whether pending,
// running or in their own host work around it (budget: one call per CU; a
// lone call's stream is one wave, so small batches leave the chip idle and
// run side by side, while a large one already fills it); it takes the
// pending calls in arrival order, up to budget minus those in flight, runs them
// (run(set, batch)) and marks them done.  Every caller sleeps on its own
// condition variable: a finished batch wakes its own callers and, when calls
// are pending, the oldest one to lead next -- not all the threads (256
// callers on 16 host cores: the wake-up storm alone cost milliseconds per
// batch).
bool coalesce_on();

template <class Set, class Coal>
Set* free_set(Coal& C, uint32_t budget) {
  // a second batch only while the active calls (threads inside a call, or
  // running + pending if more) are fewer than half the budget (a finished
  // batch wakes the oldest pending call, so a call refused here is retried
  // when the running batches end): with many callers one batch at a time holds them
  // all, while concurrent sets split them into small batches -- 256 callers
  // 124 vs 86 MB/s, DecodeToBuf loops 21 vs 12 MB/s; with few callers the
  // sets run side by side -- 16 callers 12.9 vs 19.3 MB/s
  // (profiles/r05_coalesce/)
  const size_t active = std::max<size_t>(C.in_flight + C.pending.size(), C.callers.load());
  if (C.in_flight != 0 && active >= budget / 2) return nullptr;
  for (int i = 0; i < in_flight_limit(); ++i)
    if (!C.sets[i].busy && !C.sets[i].broken) return &C.sets[i];
  return nullptr;
}
template <class Coal>
bool all_sets_broken(const Coal& C) {
  for (int i = 0; i < in_flight_limit(); ++i)
    if (!C.sets[i].broken) return false;
  return true;
}
// A batch set's stream.  LZGPU_FAULT_STREAM_CREATE=N (fault injection for
// tests/test_coalesce.py only) makes the first N creations in the process fail.
bool create_set_stream(hipStream_t* st) {
  static std::atomic<int> fail_left{[] {
    const char* e = getenv("LZGPU_FAULT_STREAM_CREATE");
    return e ? atoi(e) : 0;
  }()};
  if (fail_left.load() > 0 && fail_left.fetch_sub(1) > 0) return false;
  if (hipStreamCreateWithFlags(st, hipStreamNonBlocking) != hipSuccess) {
    (void)hipGetLastError();
    *st = nullptr;
    return false;
  }
  return true;
}
template <class Coal, class Set>
void wake_next(Coal& C, uint32_t budget) {
  if (!C.pending.empty() && free_set<Set>(C, budget))
    C.pending.front()->cv.notify_one();
}
template <class Coal, class Set, class Call, class Run, class Fail>
void group_commit(Coal& C, Call& me, uint32_t budget, Run run, Fail stream_failed) {
  std::unique_lock<std::mutex> lk(C.mu);
  C.pending.push_back(&me);
  while (!me.done) {
    Set* R = me.taken ? nullptr : free_set<Set>(C, budget);
    if (!R) {
      if (!me.taken && C.in_flight == 0 && all_sets_broken(C)) {
        // no set has a stream and no batch runs: fail this call
        // and wake every pending one, which fails the same way -- nobody
        // waits for a batch that cannot come; the last one clears the marks,
        // so later calls try to create the streams again
        C.pending.erase(std::find(C.pending.begin(), C.pending.end(), &me));
        stream_failed(me);
        me.taken = me.done = true;
        for (Call* c : C.pending) c->cv.notify_one();
        if (C.pending.empty())
          for (auto& x : C.sets) x.broken = false;
        return;
      }
      me.cv.wait(lk);
      continue;
    }
    if (!R->stream && !create_set_stream(&R->stream)) {
      // this set cannot run batches: leave it out and try again -- another
      // set, the end of a running batch (which wakes the next pending call),
      // or the failure above when no set is left
      R->broken = true;
      continue;
    }
    std::vector<Call*> batch;
    if (!coalesce_on()) {  // one launch per call: this one now
      C.pending.erase(std::find(C.pending.begin(), C.pending.end(), &me));
      batch.assign(1, &me);
    } else {
      const size_t room = budget > C.in_flight ? budget - C.in_flight : 1;
      const size_t take = std::min(C.pending.size(), room);
      batch.assign(C.pending.begin(), C.pending.begin() + take);
      C.pending.erase(C.pending.begin(), C.pending.begin() + take);
    }
    for (Call* c : batch) c->taken = true;
    R->busy = true;
    C.in_flight += uint32_t(batch.size());
    wake_next<Coal, Set>(C, budget);  // more pending and room: a concurrent batch
    lk.unlock();
    run(*R, batch);
    C.batches++;
    C.items += batch.size();
    uint64_t mx = C.max_items.load();
    while (batch.size() > mx && !C.max_items.compare_exchange_weak(mx, batch.size())) {
    }
    lk.lock();
    for (Call* c : batch) {
      c->done = true;
      if (c != &me) c->cv.notify_one();
    }
    R->busy = false;
    C.in_flight -= uint32_t(batch.size());
    wake_next<Coal, Set>(C, budget);
  }
}

std::atomic<Coalescer*> g_coal[kLzgpuMaxDevices];
Coalescer* coalescer(int dev) {
  static std::mutex mu;
  if (dev < 0 || dev >= kLzgpuMaxDevices) return nullptr;
  std::lock_guard<std::mutex> g(mu);
  if (!g_coal[dev].load()) g_coal[dev].store(new (std::nothrow) Coalescer());  // process lifetime
  return g_coal[dev].load();
}
Coalescer* coalescer_if(int dev) { return g_coal[dev].load(); }

bool coalesce_on() {
  static const bool on = [] {
    const char* e = getenv("LZGPU_COALESCE");
    return !(e && e[0] == '0');
  }();
  return on;
}

size_t align16(size_t v) { return (v + 15) & ~size_t(15); }

// Host time of the one-call batches by phase (LzmaGpu_CoalesceTimes; VERDICT
// r04 item 4: where a lone 4 KiB LzmaDecode's time goes): plan, staging
// (pinned / device buffers, packing), upload enqueue, launch enqueue, waiting
// for the kernel and the results, downloading the outputs; the whole batch;
// and every call from entry to return (queueing behind a running batch
// included).
enum { kTPlan, kTStage, kTUpload, kTLaunch, kTWait, kTDownload, kTBatch, kTCall, kTPhases };
std::atomic<uint64_t> g_tns[kTPhases], g_tbatches{0};
uint64_t now_ns() {
  return uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(
                      std::chrono::steady_clock::now().time_since_epoch())
                      .count());
}
struct PhaseClock {
  uint64_t t0 = now_ns(), t = t0;
  void mark(int k) {
    const uint64_t n = now_ns();
    g_tns[k] += n - t;
    t = n;
  }
  ~PhaseClock() {
    g_tns[kTBatch] += now_ns() - t0;
    ++g_tbatches;
  }
};

// Outputs of a batch up to this many bytes of capacity come back in one
// transfer into the pinned staging and are copied to the callers' buffers on
// the host; a larger batch downloads each call's decoded bytes on its own
// (one pageable transfer per call: ~7 us each, 1.9 ms of a 255-call batch).
constexpr size_t kBulkOutMax = size_t(64) << 20;
// First allocation of a batch set's pinned staging and device I/O buffer (the
// workspace and metadata take a quarter): 256 coalesced 4 KiB calls need
// ~1.6 MB, so steady traffic never regrows them.
constexpr size_t kSetFloor = size_t(4) << 20;
// Largest pinned staging a batch set keeps: the doubling stops
// here, and a batch that would need more -- an oversized call run alone, up to
// 256 MiB of input -- stages through pageable memory instead of leaving every
// set holding that much pinned memory for the life of the process.
constexpr size_t kSetPinMax = kBulkOutMax + (size_t(32) << 20);

// One batch of calls on the current device (the leader, C.mu not held).
void run_batch(BatchSet& C, const std::vector<OneCall*>& b) {
  PhaseClock pc;
  const size_t k = b.size();
  auto fail_all = [&](SRes e, const char* what) {
    for (OneCall* c : b) {
      c->err = e;
      c->msg = what;
    }
  };
  std::vector<LzmaGpuStreamDesc> d(k);
  std::vector<uint32_t> order(k);
  size_t in_total = 0, out_total = 0;
  for (size_t i = 0; i < k; ++i) {
    const OneCall& c = *b[i];
    LzmaGpuStreamDesc& x = d[i];
    memset(&x, 0, sizeof x);
    x.src_off = in_total;
    x.src_len = c.in_size;
    x.dst_off = out_total;
    x.dst_cap = c.out_size;
    memcpy(x.props, c.props, sizeof c.props);
    x.props_size = c.props_size;
    x.finish_mode = c.finish;
    x.kind = c.kind;
    in_total += align16(c.in_size);
    out_total += align16(c.out_size);
  }
  LzmaGpuPlan plan;
  LzmaGpuPlanOptions o;
  memset(&o, 0, sizeof o);
  // one item: one 32-lane wave with the whole table in LDS (the round-3
  // single-call path); several: the planner's choice for the batch
  o.kernel = k == 1 ? LZMA_GPU_KERNEL_COOP : LZMA_GPU_KERNEL_AUTO;
  {
    const SRes pr = LzmaGpu_PlanBatchOpt(d.data(), k, order.data(), &plan, &o);
    if (pr != SZ_OK) return fail_all(pr, "LzmaDecode: batch plan failed");
  }
  pc.mark(kTPlan);
  const size_t meta_bytes = align16(k * sizeof(LzmaGpuStreamDesc)) + align16(k * sizeof(uint32_t));
  const size_t res_bytes = align16(k * sizeof(LzmaGpuResult));
  bool bulk_out = out_total <= kBulkOutMax;
  size_t pin_need = in_total + meta_bytes + res_bytes + (bulk_out ? out_total : 0) + 64;
  // over kSetPinMax: inputs uploaded and outputs downloaded per call from the
  // callers' own (pageable) buffers, descriptors and results in host memory
  const bool pageable = pin_need > kSetPinMax;
  std::vector<uint8_t> host_meta;
  if (pageable) {
    bulk_out = false;
    host_meta.resize(meta_bytes + res_bytes + 64);
  }
  if (!pageable && C.pin_cap < pin_need) {
    // grow geometrically from 4 MiB up to kSetPinMax: a run of slightly
    // larger batches reallocates (and synchronises the device, hipHostFree /
    // hipHostMalloc, stalling the other sets' batches) O(log) times
    const size_t want = std::max({pin_need, std::min(C.pin_cap * 2, kSetPinMax), kSetFloor});
    if (C.pin) (void)hipHostFree(C.pin);
    C.pin = nullptr;
    C.pin_cap = 0;
    if (hipHostMalloc(reinterpret_cast<void**>(&C.pin), want, hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      C.pin = nullptr;
      return fail_all(SZ_ERROR_MEM, "LzmaDecode: pinned staging allocation failed");
    }
    C.pin_cap = want;
  }
  uint8_t* d_io = static_cast<uint8_t*>(C.io.get(std::max(in_total + out_total + 16, kSetFloor)));
  void* d_ws = C.ws.get(std::max(size_t(plan.workspace_bytes), kSetFloor / 4));
  uint8_t* d_meta = static_cast<uint8_t*>(C.meta.get(std::max(meta_bytes + res_bytes + 16, kSetFloor / 4)));
  if (!d_io || !d_ws || !d_meta) return fail_all(SZ_ERROR_MEM, "LzmaDecode: device allocation failed");
  // pack inputs and metadata, one upload each
  uint8_t* pin_meta = pageable ? host_meta.data() : C.pin + in_total;
  if (!pageable)
    for (size_t i = 0; i < k; ++i)
      if (b[i]->in_size) memcpy(C.pin + d[i].src_off, b[i]->src, b[i]->in_size);
  memcpy(pin_meta, d.data(), k * sizeof(LzmaGpuStreamDesc));
  memcpy(pin_meta + align16(k * sizeof(LzmaGpuStreamDesc)), order.data(), k * sizeof(uint32_t));
  const hipStream_t st = C.stream;
  LzmaGpuResult* pin_res = reinterpret_cast<LzmaGpuResult*>(pin_meta + meta_bytes);
  LzmaGpuResult* d_res = reinterpret_cast<LzmaGpuResult*>(d_meta + meta_bytes);
  pc.mark(kTStage);
  bool up_ok = true;
  if (pageable) {
    for (size_t i = 0; i < k && up_ok; ++i)
      up_ok = !b[i]->in_size || xfer(d_io + d[i].src_off, b[i]->src, b[i]->in_size,
                                     hipMemcpyHostToDevice, st) == hipSuccess;
  } else {
    up_ok = !in_total || xfer(d_io, C.pin, in_total, hipMemcpyHostToDevice, st) == hipSuccess;
  }
  if (!up_ok || xfer(d_meta, pin_meta, meta_bytes, hipMemcpyHostToDevice, st) != hipSuccess)
    return fail_all(SZ_ERROR_FAIL, "LzmaDecode: upload failed");
  pc.mark(kTUpload);
  if (LzmaGpu_DecodeBatchEx(&plan, reinterpret_cast<LzmaGpuStreamDesc*>(d_meta),
                            reinterpret_cast<uint32_t*>(d_meta + align16(k * sizeof(LzmaGpuStreamDesc))),
                            d_io, d_io + in_total, d_ws, d_res, st) != SZ_OK) {
    (void)hipStreamSynchronize(st);
    return fail_all(SZ_ERROR_FAIL, "LzmaDecode: batch launch failed");
  }
  pc.mark(kTLaunch);
  // results (and, for a bulk batch, every output) in one synchronisation
  uint8_t* pin_out = reinterpret_cast<uint8_t*>(pin_res) + align16(res_bytes);
  if (xfer(pin_res, d_res, res_bytes, hipMemcpyDeviceToHost, st) != hipSuccess ||
      (bulk_out && out_total &&
       xfer(pin_out, d_io + in_total, out_total, hipMemcpyDeviceToHost, st) != hipSuccess) ||
      hipStreamSynchronize(st) != hipSuccess)
    return fail_all(SZ_ERROR_FAIL, "LzmaDecode: decode kernel failed");
  pc.mark(kTWait);
  // outputs: only the bytes decoded, into each caller's buffer
  for (size_t i = 0; i < k; ++i) {
    OneCall& c = *b[i];
    c.r = pin_res[i];
    if (c.r.dest_len > c.out_size) {
      c.err = SZ_ERROR_FAIL;
      c.msg = "LzmaDecode: kernel reported more output than its capacity";
      continue;
    }
    if (!c.r.dest_len) continue;
    if (bulk_out) {
      memcpy(c.dest, pin_out + d[i].dst_off, size_t(c.r.dest_len));
    } else if (xfer(c.dest, d_io + in_total + d[i].dst_off, c.r.dest_len,
                    hipMemcpyDeviceToHost, st) != hipSuccess) {
      c.err = SZ_ERROR_FAIL;
      c.msg = "LzmaDecode: download output failed";
    }
  }
  if (!bulk_out && hipStreamSynchronize(st) != hipSuccess)
    fail_all(SZ_ERROR_FAIL, "LzmaDecode: download output");
  pc.mark(kTDownload);
}

// Calls whose input + output exceed this run in a batch of their own: one
// caller's multi-GB destination capacity must not set the device footprint of
// everyone else's batch, nor fail it when that allocation fails.
constexpr size_t kCoalesceItemMax = size_t(256) << 20;

// Run the leader's calls: the small ones as one batch, each big one alone; a
// batch of several calls that fails as a whole (an allocation, upload or
// launch of the batch) is retried call by call, so a call fails only when it
// would have failed alone.
void run_calls(BatchSet& C, const std::vector<OneCall*>& batch) {
  std::vector<OneCall*> small;
  std::vector<std::vector<OneCall*>> runs;
  for (OneCall* c : batch) {
    if (size_t(c->in_size) + size_t(c->out_size) > kCoalesceItemMax)
      runs.push_back({c});
    else
      small.push_back(c);
  }
  if (!small.empty()) runs.insert(runs.begin(), small);
  for (const auto& r : runs) {
    run_batch(C, r);
    if (r.size() < 2) continue;
    for (OneCall* c : r) {
      if (c->err == SZ_OK) continue;
      c->err = SZ_OK;
      c->msg = "";
      run_batch(C, {c});
    }
  }
}

// Submit one call; returns when its batch has run.
void coalesced(OneCall& me, int dev) {
  Coalescer* Cp = coalescer(dev);
  if (!Cp) {
    me.err = SZ_ERROR_MEM;
    me.msg = "LzmaDecode: host allocation failed";
    return;
  }
  group_commit<Coalescer, BatchSet>(
      *Cp, me, std::max(1u, lzgpu_host::device_cus()),
      [](BatchSet& R, std::vector<OneCall*>& batch) {
        try {
          run_calls(R, batch);
        } catch (const std::exception&) {
          for (OneCall* c : batch) {
            c->err = SZ_ERROR_MEM;
            c->msg = "LzmaDecode: host allocation failed";
          }
        }
      },
      [](OneCall& c) {
        c.err = SZ_ERROR_FAIL;
        c.msg = "LzmaDecode: stream creation failed";
      });
}

// LzmaDecode-style one call over host buffers through the device's coalescer.
SRes gpu_one_call(uint8_t kind, Byte* dest, SizeT* destLen, const Byte* src, SizeT* srcLen,
                  const Byte* props, unsigned propSize, ELzmaFinishMode finishMode,
                  int* status_out) {
  const SizeT in_size = *srcLen, out_size = *destLen;
  *srcLen = 0;
  *destLen = 0;
  if (!ensure_device()) return SZ_ERROR_FAIL;
  int dev = 0;
  if (!hip_ok(hipGetDevice(&dev), "current device")) return SZ_ERROR_FAIL;
  ++g_calls;
  Coalescer* Cp = coalescer(dev);
  ActiveCall active(Cp ? &Cp->callers : nullptr);
  const uint64_t t_call = now_ns();
  OneCall c;
  c.kind = kind;
  c.src = src;
  c.in_size = in_size;
  c.dest = dest;
  c.out_size = out_size;
  memcpy(c.props, props, std::min<unsigned>(propSize, LZMA_PROPS_SIZE));
  c.props_size = uint8_t(std::min<unsigned>(propSize, 255));
  c.finish = uint8_t(finishMode);
  coalesced(c, dev);
  g_tns[kTCall] += now_ns() - t_call;
  if (c.err != SZ_OK) {
    set_error(c.msg);
    return c.err;
  }
  *destLen = c.r.dest_len;
  *srcLen = c.r.src_len;
  *status_out = c.r.status;
  return c.r.res;
}

// ------------------------------------------------------------------ dictionary mirrors

// Device buffers of retired mirrors, kept for the next decoder instead of
// freed: hipFree synchronises the whole device, and a DecodeToBuf caller that
// creates and frees a decoder per stream (7zDec.c:567-648) would otherwise
// stall every other caller's launch once per stream.  Bounded; beyond it the
// oldest buffer is freed.
struct BufPool {
  struct Ent {
    void* p;
    size_t cap;
    int dev;
  };
  std::mutex mu;
  std::vector<Ent> v;
  size_t bytes = 0;
};
constexpr size_t kBufPoolMaxBytes = size_t(1) << 30;
constexpr size_t kBufPoolMaxCount = 512;
BufPool& buf_pool() {
  static BufPool* p = new BufPool();  // process lifetime (HIP teardown order)
  return *p;
}
void pool_put(DevBuf& b, int dev) {
  if (!b.p) return;
  std::vector<void*> drop;
  {
    BufPool& P = buf_pool();
    std::lock_guard<std::mutex> g(P.mu);
    try {
      P.v.push_back({b.p, b.cap, dev});
    } catch (const std::exception&) {
      drop.push_back(b.p);
    }
    if (drop.empty()) P.bytes += b.cap;
    while (P.v.size() > kBufPoolMaxCount || P.bytes > kBufPoolMaxBytes) {
      P.bytes -= P.v.front().cap;
      drop.push_back(P.v.front().p);
      P.v.erase(P.v.begin());
    }
  }
  b.p = nullptr;
  b.cap = 0;
  for (void* q : drop) (void)hipFree(q);  // outside the pool lock
}
// an empty DevBuf takes the smallest pooled buffer of at least n bytes
void pool_take(DevBuf& b, size_t n, int dev) {
  if (b.p) return;
  BufPool& P = buf_pool();
  std::lock_guard<std::mutex> g(P.mu);
  size_t best = P.v.size();
  for (size_t i = 0; i < P.v.size(); ++i)
    if (P.v[i].dev == dev && P.v[i].cap >= n && (best == P.v.size() || P.v[i].cap < P.v[best].cap))
      best = i;
  if (best == P.v.size()) return;
  b.p = P.v[best].p;
  b.cap = P.v[best].cap;
  P.bytes -= b.cap;
  P.v.erase(P.v.begin() + ptrdiff_t(best));
}

struct Mirror {
  ~Mirror() {
    pool_put(block, dev);
    pool_put(io, dev);
  }
  const CLzmaDec* key = nullptr;
  int dev = 0;
  const Byte* dic = nullptr;
  SizeT dic_buf_size = 0;
  const CLzmaProb* probs = nullptr;
  uint32_t num_probs = 0;
  DevBuf block;  // [session | probs | dic]
  DevBuf io;     // this call's input (+ DecodeToBuf output)
  bool history = false;    // device dic holds every byte the decoder wrote since its dic init
  bool probs_dev = false;  // device table == host table (downloaded after every call)
  // what the last successful call left in the host object: positions and a
  // hash of the table (the coherence check on entry)
  SizeT end_pos = 0;
  uint32_t end_total = 0;
  uint32_t probs_cells = 0;
  uint64_t probs_hash = 0;
  uint64_t tick = 0;
  std::mutex busy;  // one call at a time per decoder object (the reference's contract)
};

constexpr size_t kSessBytes = 256;  // LzgpuSession (192 B) rounded up
constexpr size_t kMirrorMaxCount = 256;
constexpr size_t kMirrorMaxBytes = size_t(16) << 30;

struct Registry {
  std::mutex mu;
  std::vector<std::shared_ptr<Mirror>> v;
  uint64_t tick = 0;
};
Registry& registry() {
  static Registry* r = new Registry();  // process lifetime (HIP teardown order)
  return *r;
}

size_t probs_area(uint32_t num_probs) { return (size_t(num_probs) * 2 + 255) & ~size_t(255); }

// The mirror of decoder p on device dev (created on first use).  A mirror whose
// dic / dicBufSize / probs allocation no longer match p is reset: its device
// copies no longer describe p.  p's mirrors on other devices are dropped (the
// host object moves on without them).  Least recently used mirrors nobody is
// using are evicted beyond kMirrorMaxCount or the byte budget, counting the
// `want` bytes this call's block will need (an evicted decoder's next call
// rebuilds its mirror: correctness never depends on one existing).  Dropped
// mirrors go to `dead`, released by the caller outside the registry lock.
size_t mirror_budget() {
  static const size_t b = [] {
    const char* e = getenv("LZGPU_MIRROR_BUDGET_MB");
    const long long mb = e ? atoll(e) : 0;
    return mb > 0 ? size_t(mb) << 20 : kMirrorMaxBytes;
  }();
  return b;
}
std::shared_ptr<Mirror> mirror_get(const CLzmaDec* p, int dev, size_t want,
                                   std::vector<std::shared_ptr<Mirror>>& dead) {
  Registry& R = registry();
  std::lock_guard<std::mutex> g(R.mu);
  std::shared_ptr<Mirror> m;
  for (size_t i = 0; i < R.v.size();) {
    auto& e = R.v[i];
    if (e->key == p && e->dev != dev) {
      dead.push_back(std::move(e));
      R.v.erase(R.v.begin() + ptrdiff_t(i));
      continue;
    }
    if (e->key == p) m = e;
    ++i;
  }
  if (!m) {
    m = std::make_shared<Mirror>();
    m->key = p;
    m->dev = dev;
    R.v.push_back(m);
  }
  if (m->dic != p->dic || m->dic_buf_size != p->dicBufSize || m->probs != p->probs ||
      m->num_probs != p->numProbs) {
    m->dic = p->dic;
    m->dic_buf_size = p->dicBufSize;
    m->probs = p->probs;
    m->num_probs = p->numProbs;
    m->history = false;
    m->probs_dev = false;
  }
  m->tick = ++R.tick;
  // eviction: oldest idle mirrors first
  size_t bytes = want > m->block.cap ? want - m->block.cap : 0;
  for (auto& e : R.v) bytes += e->block.cap + e->io.cap;
  while (R.v.size() > kMirrorMaxCount || bytes > mirror_budget()) {
    size_t victim = R.v.size();
    for (size_t i = 0; i < R.v.size(); ++i)
      if (R.v[i].use_count() == 1 && (victim == R.v.size() || R.v[i]->tick < R.v[victim]->tick))
        victim = i;
    if (victim == R.v.size()) break;  // all in use
    bytes -= R.v[victim]->block.cap + R.v[victim]->io.cap;
    dead.push_back(std::move(R.v[victim]));
    R.v.erase(R.v.begin() + ptrdiff_t(victim));
  }
  return m;
}

// FNV-1a over the table cells the decoder uses, four cells (one 64-bit word)
// per step: the coherence check of the host table, run twice per call (once
// on entry, once after the download).  Tables are table_cells() cells: 14.6 KB
// at lc3, up to 6 MiB at lc + lp = 12.
uint64_t probs_hash(const CLzmaProb* t, uint32_t cells) {
  const uint8_t* b = reinterpret_cast<const uint8_t*>(t);
  const size_t n = size_t(cells) * sizeof(CLzmaProb);
  uint64_t h = 1469598103934665603ull;
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    memcpy(&w, b + i, 8);
    h = (h ^ w) * 1099511628211ull;
  }
  for (; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
  return h;
}

void mirror_drop(const CLzmaDec* p) {
  std::vector<std::shared_ptr<Mirror>> dead;  // released after the registry lock
  Registry& R = registry();
  std::lock_guard<std::mutex> g(R.mu);
  for (size_t i = 0; i < R.v.size();) {
    if (R.v[i]->key == p) {
      dead.push_back(std::move(R.v[i]));
      R.v.erase(R.v.begin() + ptrdiff_t(i));
    } else {
      ++i;
    }
  }
}

// ------------------------------------------------------------------ coalesced session calls
//
// Dictionary-interface calls (LzmaDec_DecodeToDic / LzmaDec_DecodeToBuf) made
// by several host threads at once, each on its own decoder, share launches the
// same way one-call decodes do: each call prepares its mirror (uploads its
// input, table and history on its own stream) and hands the device session
// state to its device's session queue; a call that finds a free session set
// (up to in_flight_limit() launches at once) takes the whole queue as ONE
// launch of the session kernels (one 32-lane wave per decoder) and every
// caller then downloads its own table and bytes.
struct SessCall {
  LzgpuSession q;  // in: the call; out: the state after it
  uint32_t cells = 0;
  int err = 0;     // launch failure
  bool taken = false;  // in a launch (running or done)
  bool done = false;
  std::condition_variable cv;  // its caller sleeps here (group_commit)
};

// One session launch in flight: its LzgpuSession array, host copy and stream.
struct SessSet {
  DevBuf arr;                   // the batch's LzgpuSession array
  std::vector<LzgpuSession> h;  // its host copy
  hipStream_t stream = nullptr;
  bool busy = false;
  bool broken = false;  // its stream could not be created: not picked (group_commit)
};

struct SessCoalescer {
  std::mutex mu;
  std::vector<SessCall*> pending;
  SessSet sets[kMaxInFlight];  // up to in_flight_limit() launches at once
  uint32_t in_flight = 0;      // calls in running launches
  std::atomic<uint32_t> callers{0};  // threads inside a session call (ActiveCall)
  std::atomic<uint64_t> batches{0}, items{0}, max_items{0};
};

std::atomic<SessCoalescer*> g_scoal[kLzgpuMaxDevices];
SessCoalescer* sess_coalescer(int dev) {
  static std::mutex mu;
  if (dev < 0 || dev >= kLzgpuMaxDevices) return nullptr;
  std::lock_guard<std::mutex> g(mu);
  if (!g_scoal[dev].load()) g_scoal[dev].store(new (std::nothrow) SessCoalescer());
  return g_scoal[dev].load();
}

// One launch for a batch of session calls (the leader, C.mu not held):
// wave-cooperative sessions in one launch, tables wider than 64 KiB on the
// one-lane global session kernel.
void run_sess_batch(SessSet& C, const std::vector<SessCall*>& b) {
  const size_t k = b.size();
  std::vector<size_t> coop, glob;
  uint32_t lds_cells = 0;
  for (size_t i = 0; i < k; ++i) {
    if (b[i]->cells <= kSessCoopMaxCells) {
      coop.push_back(i);
      lds_cells = std::max(lds_cells, b[i]->cells);
    } else {
      glob.push_back(i);
    }
  }
  C.h.resize(k);
  size_t j = 0;
  for (size_t i : coop) C.h[j++] = b[i]->q;
  for (size_t i : glob) C.h[j++] = b[i]->q;
  LzgpuSession* d = static_cast<LzgpuSession*>(C.arr.get(std::max(k * sizeof(LzgpuSession), kSetFloor / 4)));
  const hipStream_t st = C.stream;
  int e = (d && xfer(d, C.h.data(), k * sizeof(LzgpuSession), hipMemcpyHostToDevice, st) ==
                    hipSuccess) ? 0 : 1;
  if (!e && !coop.empty() &&
      lzgpu_launch_session_coop(d, uint32_t(coop.size()), lds_cells, 0, st) != 0)
    e = 1;
  if (!e && !glob.empty() && lzgpu_launch_session(d + coop.size(), uint32_t(glob.size()), st) != 0)
    e = 1;
  if (!e && (xfer(C.h.data(), d, k * sizeof(LzgpuSession), hipMemcpyDeviceToHost, st) !=
                 hipSuccess ||
             hipStreamSynchronize(st) != hipSuccess))
    e = 1;
  if (e) (void)hipStreamSynchronize(st);
  j = 0;
  for (size_t i : coop) b[i]->q = C.h[j++];
  for (size_t i : glob) b[i]->q = C.h[j++];
  for (SessCall* c : b) c->err = e;
}

// Run one prepared session call through the device's queue; returns when
// its launch has finished (c.err set on a launch failure).
void sess_coalesced(SessCall& me, int dev) {
  SessCoalescer* Cp = sess_coalescer(dev);
  if (!Cp) {
    me.err = 1;
    return;
  }
  group_commit<SessCoalescer, SessSet>(
      *Cp, me, std::max(1u, lzgpu_host::device_cus()),
      [](SessSet& R, std::vector<SessCall*>& batch) {
        try {
          run_sess_batch(R, batch);
        } catch (const std::exception&) {
          for (SessCall* c : batch) c->err = 1;
        }
      },
      [](SessCall& c) { c.err = 1; });
}

// One LzmaDec_DecodeToDic (mode 0) or LzmaDec_DecodeToBuf (mode 1) call on the
// GPU over a host CLzmaDec, through its mirror.
SRes gpu_session_call(CLzmaDec* p, int mode, SizeT dicLimit, const Byte* src, SizeT in_size,
                      SizeT* in_used, Byte* dest, SizeT* destLen, ELzmaFinishMode finishMode,
                      ELzmaStatus* status) {
  int dev = 0;
  if (!hip_ok(hipGetDevice(&dev), "current device")) return SZ_ERROR_FAIL;
  ++g_calls;
  SessCoalescer* SCp = sess_coalescer(dev);
  ActiveCall active(SCp ? &SCp->callers : nullptr);
  const uint32_t cells = lzgpu::table_cells(p->prop.lc, p->prop.lp, p->prop.pb);
  if (p->probs == nullptr || cells > p->numProbs) {
    set_error("LzmaDec: probabilities not allocated for the current props");
    return SZ_ERROR_PARAM;
  }
  const size_t pa = probs_area(p->numProbs);
  std::shared_ptr<Mirror> m;
  {
    std::vector<std::shared_ptr<Mirror>> dead;  // released after the registry lock
    try {
      m = mirror_get(p, dev, kSessBytes + pa + p->dicBufSize + 16, dead);
    } catch (const std::exception&) {
      set_error("LzmaDec: host allocation failed");
      return SZ_ERROR_MEM;
    }
  }
  std::lock_guard<std::mutex> busy(m->busy);
  ScratchLease L;
  if (!L.s) return SZ_ERROR_FAIL;
  const hipStream_t st = L.s->stream;
  const size_t out_room = mode == 1 ? size_t(*destLen) : 0;
  const void* blk_before = m->block.p;
  pool_take(m->block, kSessBytes + pa + p->dicBufSize + 16, dev);
  uint8_t* blk = static_cast<uint8_t*>(m->block.get(kSessBytes + pa + p->dicBufSize + 16));
  const size_t in_pad = (size_t(in_size) + 15) & ~size_t(15);
  pool_take(m->io, in_pad + out_room + 16, dev);
  uint8_t* d_io = static_cast<uint8_t*>(m->io.get(in_pad + out_room + 16));
  if (!blk || !d_io) {
    m->history = m->probs_dev = false;
    set_error("LzmaDec: device allocation failed");
    return SZ_ERROR_MEM;
  }
  if (blk != blk_before) m->history = m->probs_dev = false;  // fresh or regrown: nothing held
  LzgpuSession* d_sess = reinterpret_cast<LzgpuSession*>(blk);
  uint16_t* d_probs = reinterpret_cast<uint16_t*>(blk + kSessBytes);
  uint8_t* d_dic = blk + kSessBytes + pa;

  auto fail = [&](const char* what) {
    (void)hipStreamSynchronize(st);
    m->history = m->probs_dev = false;  // device state unknown; the host object is untouched
    set_error(what);
    return SZ_ERROR_FAIL;
  };
  // coherence with host-side writes since the previous call (file header)
  if (m->history) {
    const SizeT np = p->dicPos, op = m->end_pos, B = p->dicBufSize;
    const uint32_t dt = p->processedPos - m->end_total;
    bool ok = false;
    if (dt == 0) {
      ok = np == op || (op == B && np == 0);  // untouched, or the ring wrapped
    } else if (np <= B && op <= B) {
      const SizeT o = op == B ? 0 : op;
      if (np >= o && np - o == dt) {  // the host wrote dic[o, np)
        ok = xfer(d_dic + o, p->dic + o, np - o, hipMemcpyHostToDevice, st) == hipSuccess;
      } else if (np < o && (B - o) + np == dt) {  // ... across the ring end
        ok = xfer(d_dic + o, p->dic + o, B - o, hipMemcpyHostToDevice, st) == hipSuccess &&
             (np == 0 || xfer(d_dic, p->dic, np, hipMemcpyHostToDevice, st) == hipSuccess);
      }
    }
    if (!ok) m->history = false;
  }
  if (m->probs_dev && (m->probs_cells != cells || probs_hash(p->probs, cells) != m->probs_hash))
    m->probs_dev = false;
  // small transfers go through the scratch's pinned staging (layout: input |
  // table up; after the launch: table down | decoded bytes)
  const size_t tab_bytes = size_t(cells) * 2, tab_pad = (tab_bytes + 15) & ~size_t(15);
  // (DecodeToDic downloads at most dic[dicPos, dicLimit), not the whole ring:
  // ADVICE r05, many callers on multi-MiB dictionaries)
  const size_t dic_room = dicLimit > p->dicPos ? size_t(dicLimit - p->dicPos) : 0;
  const size_t down_max = tab_pad + (mode == 1 ? out_room : dic_room);
  uint8_t* pin = lzgpu_host::scratch_pinned(L.s, std::max(in_pad + tab_pad, down_max));
  // the table: the device copy is current after every successful call
  if (!m->probs_dev) {
    const void* from = p->probs;
    if (pin) {
      memcpy(pin + in_pad, p->probs, tab_bytes);
      from = pin + in_pad;
    }
    if (xfer(d_probs, from, tab_bytes, hipMemcpyHostToDevice, st) != hipSuccess)
      return fail("LzmaDec: upload probs");
  }
  // history: only a decoder continuing a dictionary reads bytes it did not
  // write in this call (LzmaDec.c:165-166,176,216,376-408 read dic only when
  // processedPos or checkDicSize is non-zero); uploaded once per mirror
  const bool need_hist = p->processedPos != 0 || p->checkDicSize != 0;
  if (need_hist && !m->history && p->dicBufSize &&
      xfer(d_dic, p->dic, p->dicBufSize, hipMemcpyHostToDevice, st) != hipSuccess)
    return fail("LzmaDec: upload dictionary");
  if (in_size && pin) memcpy(pin, src, in_size);
  if (in_size && xfer(d_io, pin ? pin : src, in_size, hipMemcpyHostToDevice, st) != hipSuccess)
    return fail("LzmaDec: upload src");

  LzgpuSession q;
  memset(&q, 0, sizeof q);
  q.lc = p->prop.lc;
  q.lp = p->prop.lp;
  q.pb = p->prop.pb;
  q.dict_size = p->prop.dicSize;
  q.probs = d_probs;
  q.dic = d_dic;
  q.in = d_io;
  q.dic_buf_size = p->dicBufSize;
  q.dic_pos = p->dicPos;
  q.dic_limit = dicLimit;
  q.in_len = in_size;
  q.range = p->range;
  q.code = p->code;
  q.processed_pos = p->processedPos;
  q.check_dic_size = p->checkDicSize;
  q.state = p->state;
  for (int i = 0; i < 4; ++i) q.reps[i] = p->reps[i];
  q.remain_len = p->remainLen;
  q.need_flush = p->needFlush ? 1 : 0;
  q.need_init_state = p->needInitState ? 1 : 0;
  q.temp_buf_size = p->tempBufSize;
  memcpy(q.temp_buf, p->tempBuf, LZMA_REQUIRED_INPUT_MAX);
  q.finish_mode = finishMode;
  q.mode = mode;
  q.out = d_io + in_pad;
  q.out_len = out_room;
  const SizeT pos0 = p->dicPos;
  (void)d_sess;
  // this call's uploads are complete before it joins the device's session
  // queue; the launch (shared with concurrent calls on other decoders) runs
  // on the queue's stream
  if (hipStreamSynchronize(st) != hipSuccess) return fail("LzmaDec: uploads");
  SessCall call;
  call.q = q;
  call.cells = cells;
  sess_coalesced(call, dev);
  if (call.err) return fail("LzmaDec: session kernel");
  q = call.q;
  // the table back (the kernel wrote it to the mirror's device copy) and the
  // decoded bytes (DecodeToDic's new dictionary bytes, DecodeToBuf's output),
  // in one synchronisation, into the pinned staging when there is one
  if (mode == 0) {
    if (q.dic_pos < pos0 || q.dic_pos > p->dicBufSize || q.dic_pos > std::max<SizeT>(dicLimit, pos0))
      return fail("LzmaDec: bad session state");
  } else if (q.out_len > out_room || q.dic_pos > p->dicBufSize) {
    return fail("LzmaDec: bad session state");
  }
  const size_t nbytes = mode == 0 ? size_t(q.dic_pos - pos0) : size_t(q.out_len);
  const uint8_t* d_bytes = mode == 0 ? d_dic + pos0 : d_io + in_pad;
  Byte* h_bytes = mode == 0 ? p->dic + pos0 : dest;
  std::vector<uint8_t> back;
  uint8_t* tab_to = pin;
  if (!pin) {
    try {
      back.resize(tab_bytes);
    } catch (const std::exception&) {
      m->history = m->probs_dev = false;
      set_error("LzmaDec: host allocation failed");
      return SZ_ERROR_MEM;
    }
    tab_to = back.data();
  }
  if (xfer(tab_to, d_probs, tab_bytes, hipMemcpyDeviceToHost, st) != hipSuccess ||
      (nbytes && xfer(pin ? pin + tab_pad : h_bytes, d_bytes, nbytes, hipMemcpyDeviceToHost, st) !=
                     hipSuccess) ||
      hipStreamSynchronize(st) != hipSuccess)
    return fail("LzmaDec: download probs / decoded bytes");
  if (pin && nbytes) memcpy(h_bytes, pin + tab_pad, nbytes);
  if (mode == 1) {
    // the host ring gets the same bytes the device ring got (LzmaDec.c:849-866:
    // each pass writes from dicPos, wrapping to 0 at dicBufSize)
    SizeT pos = pos0, left = q.out_len;
    const Byte* from = dest;
    while (left) {
      if (pos == p->dicBufSize) pos = 0;
      const SizeT k = std::min<SizeT>(left, p->dicBufSize - pos);
      memcpy(p->dic + pos, from, k);
      pos += k;
      from += k;
      left -= k;
    }
    *destLen = q.out_len;
  }
  memcpy(p->probs, tab_to, tab_bytes);
  p->dicPos = q.dic_pos;
  p->range = q.range;
  p->code = q.code;
  p->processedPos = q.processed_pos;
  p->checkDicSize = q.check_dic_size;
  p->state = q.state;
  for (int i = 0; i < 4; ++i) p->reps[i] = q.reps[i];
  p->remainLen = q.remain_len;
  p->needFlush = int(q.need_flush);
  p->needInitState = int(q.need_init_state);
  p->tempBufSize = q.temp_buf_size;
  memcpy(p->tempBuf, q.temp_buf, LZMA_REQUIRED_INPUT_MAX);
  p->buf = src + q.in_used;
  m->history = true;
  m->probs_dev = true;
  m->end_pos = p->dicPos;
  m->end_total = p->processedPos;
  m->probs_cells = cells;
  m->probs_hash = probs_hash(p->probs, cells);
  *in_used = q.in_used;
  *status = ELzmaStatus(q.status);
  return q.res;
}

}  // namespace

extern "C" {

// ------------------------------------------------------------------ props + allocation

SRes LzmaProps_Decode(CLzmaProps* p, const Byte* data, unsigned size) {
  uint32_t lc, lp, pb, dict;
  if (size < LZMA_PROPS_SIZE) return SZ_ERROR_UNSUPPORTED;
  int r = lzgpu::lz_props_parse(data, size, lc, lp, pb, dict);
  // the reference stores dicSize before rejecting a bad lc/lp/pb byte
  p->dicSize = dict;
  if (r != SZ_OK) return r;
  p->lc = lc;
  p->lp = lp;
  p->pb = pb;
  return SZ_OK;
}

void LzmaDec_FreeProbs(CLzmaDec* p, ISzAlloc* alloc) {
  mirror_drop(p);
  alloc->Free(alloc, p->probs);
  p->probs = nullptr;
}

static void free_dict(CLzmaDec* p, ISzAlloc* alloc) {
  alloc->Free(alloc, p->dic);
  p->dic = nullptr;
}

void LzmaDec_Free(CLzmaDec* p, ISzAlloc* alloc) {
  LzmaDec_FreeProbs(p, alloc);
  free_dict(p, alloc);
}

static SRes alloc_probs(CLzmaDec* p, const CLzmaProps* np, ISzAlloc* alloc) {
  const uint32_t n = probs_for(np->lc, np->lp);
  if (p->probs == nullptr || n != p->numProbs) {
    LzmaDec_FreeProbs(p, alloc);
    p->probs = static_cast<CLzmaProb*>(alloc->Alloc(alloc, size_t(n) * sizeof(CLzmaProb)));
    p->numProbs = n;
    if (p->probs == nullptr) return SZ_ERROR_MEM;
  }
  return SZ_OK;
}

SRes LzmaDec_AllocateProbs(CLzmaDec* p, const Byte* props, unsigned propsSize, ISzAlloc* alloc) {
  CLzmaProps np;
  SRes r = LzmaProps_Decode(&np, props, propsSize);
  if (r != SZ_OK) return r;
  r = alloc_probs(p, &np, alloc);
  if (r != SZ_OK) return r;
  p->prop = np;
  return SZ_OK;
}

SRes LzmaDec_Allocate(CLzmaDec* p, const Byte* props, unsigned propsSize, ISzAlloc* alloc) {
  CLzmaProps np;
  SRes r = LzmaProps_Decode(&np, props, propsSize);
  if (r != SZ_OK) return r;
  r = alloc_probs(p, &np, alloc);
  if (r != SZ_OK) return r;
  const SizeT dsz = np.dicSize;
  if (p->dic == nullptr || dsz != p->dicBufSize) {
    free_dict(p, alloc);
    p->dic = static_cast<Byte*>(alloc->Alloc(alloc, dsz));
    if (p->dic == nullptr) {
      LzmaDec_FreeProbs(p, alloc);
      return SZ_ERROR_MEM;
    }
  }
  p->dicBufSize = dsz;
  p->prop = np;
  return SZ_OK;
}

void LzmaDec_InitDicAndState(CLzmaDec* p, Bool initDic, Bool initState) {
  p->needFlush = 1;
  p->remainLen = 0;
  p->tempBufSize = 0;
  if (initDic) {
    p->processedPos = 0;
    p->checkDicSize = 0;
    p->needInitState = 1;
  }
  if (initState) p->needInitState = 1;
}

void LzmaDec_Init(CLzmaDec* p) {
  p->dicPos = 0;
  LzmaDec_InitDicAndState(p, 1, 1);
}

void LzmaGpu_DecoderRelease(const CLzmaDec* p) { mirror_drop(p); }

void LzmaGpu_DropinTransferStats(uint64_t* h2d_bytes, uint64_t* d2h_bytes, uint64_t* calls,
                                 int reset) {
  if (h2d_bytes) *h2d_bytes = reset ? g_h2d.exchange(0) : g_h2d.load();
  if (d2h_bytes) *d2h_bytes = reset ? g_d2h.exchange(0) : g_d2h.load();
  if (calls) *calls = reset ? g_calls.exchange(0) : g_calls.load();
}

void LzmaGpu_CoalesceStats(uint64_t* batches, uint64_t* calls, uint64_t* max_batch, int reset) {
  uint64_t b = 0, c = 0, m = 0;
  for (int dev = 0; dev < kLzgpuMaxDevices; ++dev) {
    Coalescer* C = coalescer_if(dev);
    if (!C) continue;
    b += reset ? C->batches.exchange(0) : C->batches.load();
    c += reset ? C->items.exchange(0) : C->items.load();
    m = std::max<uint64_t>(m, reset ? C->max_items.exchange(0) : C->max_items.load());
  }
  for (int dev = 0; dev < kLzgpuMaxDevices; ++dev) {
    SessCoalescer* C = g_scoal[dev].load();
    if (!C) continue;
    b += reset ? C->batches.exchange(0) : C->batches.load();
    c += reset ? C->items.exchange(0) : C->items.load();
    m = std::max<uint64_t>(m, reset ? C->max_items.exchange(0) : C->max_items.load());
  }
  if (batches) *batches = b;
  if (calls) *calls = c;
  if (max_batch) *max_batch = m;
}

void LzmaGpu_CoalesceTimes(uint64_t* ns, uint64_t* batches, int reset) {
  for (int k = 0; k < kTPhases; ++k)
    if (ns) ns[k] = reset ? g_tns[k].exchange(0) : g_tns[k].load();
  const uint64_t b = reset ? g_tbatches.exchange(0) : g_tbatches.load();
  if (batches) *batches = b;
}

// ------------------------------------------------------------------ decode entry points

SRes LzmaDec_DecodeToDic(CLzmaDec* p, SizeT dicLimit, const Byte* src, SizeT* srcLen,
                         ELzmaFinishMode finishMode, ELzmaStatus* status) {
  const SizeT in_size = *srcLen;
  *srcLen = 0;
  *status = LZMA_STATUS_NOT_SPECIFIED;
  if (!ensure_device()) return SZ_ERROR_FAIL;
  if (dicLimit > p->dicBufSize || (p->dic == nullptr && p->dicBufSize != 0)) {
    set_error("LzmaDec_DecodeToDic: dicLimit beyond dicBufSize");
    return SZ_ERROR_PARAM;
  }
  return gpu_session_call(p, 0, dicLimit, src, in_size, srcLen, nullptr, nullptr, finishMode,
                          status);
}

SRes LzmaDec_DecodeToBuf(CLzmaDec* p, Byte* dest, SizeT* destLen, const Byte* src, SizeT* srcLen,
                         ELzmaFinishMode finishMode, ELzmaStatus* status) {
  const SizeT in_size = *srcLen;
  *srcLen = 0;
  if (!ensure_device()) {
    *destLen = 0;
    return SZ_ERROR_FAIL;
  }
  if (p->dic == nullptr || p->dicBufSize == 0 || p->dicPos > p->dicBufSize) {
    *destLen = 0;
    set_error("LzmaDec_DecodeToBuf: no dictionary ring");
    return SZ_ERROR_PARAM;
  }
  SizeT out = *destLen;
  const SRes r = gpu_session_call(p, 1, 0, src, in_size, srcLen, dest, &out, finishMode, status);
  *destLen = r == SZ_ERROR_FAIL || r == SZ_ERROR_MEM || r == SZ_ERROR_PARAM ? 0 : out;
  return r;
}

SRes LzmaDecode(Byte* dest, SizeT* destLen, const Byte* src, SizeT* srcLen, const Byte* propData,
                unsigned propSize, ELzmaFinishMode finishMode, ELzmaStatus* status,
                ISzAlloc* alloc) {
  const SizeT in_size = *srcLen, out_size = *destLen;
  *srcLen = 0;
  *destLen = 0;
  if (in_size < 5) return SZ_ERROR_INPUT_EOF;
  CLzmaProps np;
  SRes r = LzmaProps_Decode(&np, propData, propSize);
  if (r != SZ_OK) return r;
  // honour the caller's allocator contract: the reference allocates the
  // probability table through it and reports SZ_ERROR_MEM when that fails
  void* host_probs = alloc->Alloc(alloc, size_t(probs_for(np.lc, np.lp)) * sizeof(CLzmaProb));
  if (host_probs == nullptr) return SZ_ERROR_MEM;
  SizeT sl = in_size, dl = out_size;
  int st = -1;
  r = gpu_one_call(LZMA_GPU_KIND_LZMA, dest, &dl, src, &sl, propData, propSize, finishMode, &st);
  alloc->Free(alloc, host_probs);
  *srcLen = sl;
  *destLen = dl;
  if (st >= 0) *status = ELzmaStatus(st);
  return r;
}

static void* lib_alloc(void*, size_t n) { return malloc(n ? n : 1); }
static void lib_free(void*, void* a) { free(a); }
static ISzAlloc g_lib_alloc = {lib_alloc, lib_free};

int LzmaUncompress(unsigned char* dest, size_t* destLen, const unsigned char* src, SizeT* srcLen,
                   const unsigned char* props, size_t propsSize) {
  ELzmaStatus status;
  return LzmaDecode(dest, destLen, src, srcLen, props, unsigned(propsSize), LZMA_FINISH_ANY,
                    &status, &g_lib_alloc);
}

// ------------------------------------------------------------------ LZMA2

enum {
  S2_CONTROL, S2_UNPACK0, S2_UNPACK1, S2_PACK0, S2_PACK1, S2_PROP, S2_DATA, S2_DATA_CONT,
  S2_FINISHED, S2_ERROR
};

static SRes lzma2_props(Byte prop, Byte* props) {
  if (prop > 40) return SZ_ERROR_UNSUPPORTED;
  const UInt32 dict = (prop == 40) ? 0xFFFFFFFFu : ((2u | (prop & 1u)) << (prop / 2 + 11));
  props[0] = 4;  // lc+lp budget of LZMA2 (Lzma2Dec.c:36,67)
  props[1] = Byte(dict);
  props[2] = Byte(dict >> 8);
  props[3] = Byte(dict >> 16);
  props[4] = Byte(dict >> 24);
  return SZ_OK;
}

SRes Lzma2Dec_AllocateProbs(CLzma2Dec* p, Byte prop, ISzAlloc* alloc) {
  Byte props[LZMA_PROPS_SIZE];
  SRes r = lzma2_props(prop, props);
  if (r != SZ_OK) return r;
  return LzmaDec_AllocateProbs(&p->decoder, props, LZMA_PROPS_SIZE, alloc);
}

SRes Lzma2Dec_Allocate(CLzma2Dec* p, Byte prop, ISzAlloc* alloc) {
  Byte props[LZMA_PROPS_SIZE];
  SRes r = lzma2_props(prop, props);
  if (r != SZ_OK) return r;
  return LzmaDec_Allocate(&p->decoder, props, LZMA_PROPS_SIZE, alloc);
}

void Lzma2Dec_Init(CLzma2Dec* p) {
  p->state = S2_CONTROL;
  p->needInitDic = 1;
  p->needInitState = 1;
  p->needInitProp = 1;
  LzmaDec_Init(&p->decoder);
}

static int lzma2_header(CLzma2Dec* p, Byte b) {
  const bool copy = (p->control & 0x80) == 0;
  switch (p->state) {
    case S2_CONTROL:
      p->control = b;
      if (b == 0) return S2_FINISHED;
      if ((b & 0x80) == 0) {
        if ((b & 0x7F) > 2) return S2_ERROR;
        p->unpackSize = 0;
      } else {
        p->unpackSize = UInt32(b & 0x1F) << 16;
      }
      return S2_UNPACK0;
    case S2_UNPACK0:
      p->unpackSize |= UInt32(b) << 8;
      return S2_UNPACK1;
    case S2_UNPACK1:
      p->unpackSize |= b;
      p->unpackSize++;
      return copy ? S2_DATA : S2_PACK0;
    case S2_PACK0:
      p->packSize = UInt32(b) << 8;
      return S2_PACK1;
    case S2_PACK1:
      p->packSize |= b;
      p->packSize++;
      if (((p->control >> 5) & 3) >= 2) return S2_PROP;
      return p->needInitProp ? S2_ERROR : S2_DATA;
    case S2_PROP: {
      if (b >= 225) return S2_ERROR;
      unsigned lc = b % 9;
      b /= 9;
      unsigned pb = b / 5, lp = b % 5;
      if (lc + lp > 4) return S2_ERROR;
      p->decoder.prop.lc = lc;
      p->decoder.prop.lp = lp;
      p->decoder.prop.pb = pb;
      p->needInitProp = 0;
      return S2_DATA;
    }
  }
  return S2_ERROR;
}

SRes Lzma2Dec_DecodeToDic(CLzma2Dec* p, SizeT dicLimit, const Byte* src, SizeT* srcLen,
                          ELzmaFinishMode finishMode, ELzmaStatus* status) {
  const SizeT in_size = *srcLen;
  *srcLen = 0;
  *status = LZMA_STATUS_NOT_SPECIFIED;
  if (!ensure_device()) return SZ_ERROR_FAIL;
  while (p->state != S2_FINISHED) {
    const SizeT pos0 = p->decoder.dicPos;
    if (p->state == S2_ERROR) return SZ_ERROR_DATA;
    if (pos0 == dicLimit && finishMode == LZMA_FINISH_ANY) {
      *status = LZMA_STATUS_NOT_FINISHED;
      return SZ_OK;
    }
    if (p->state != S2_DATA && p->state != S2_DATA_CONT) {
      if (*srcLen == in_size) {
        *status = LZMA_STATUS_NEEDS_MORE_INPUT;
        return SZ_OK;
      }
      (*srcLen)++;
      p->state = lzma2_header(p, *src++);
      continue;
    }
    SizeT out_cur = dicLimit - pos0, in_cur = in_size - *srcLen;
    ELzmaFinishMode fin_cur = LZMA_FINISH_ANY;
    if (p->unpackSize <= out_cur) {
      out_cur = p->unpackSize;
      fin_cur = LZMA_FINISH_END;
    }
    if ((p->control & 0x80) == 0) {
      if (*srcLen == in_size) {
        *status = LZMA_STATUS_NEEDS_MORE_INPUT;
        return SZ_OK;
      }
      if (p->state == S2_DATA) {
        const bool reset = (p->control == 1);
        if (reset)
          p->needInitProp = p->needInitState = 1;
        else if (p->needInitDic)
          return SZ_ERROR_DATA;
        p->needInitDic = 0;
        LzmaDec_InitDicAndState(&p->decoder, reset, 0);
      }
      if (in_cur > out_cur) in_cur = out_cur;
      if (in_cur == 0) return SZ_ERROR_DATA;
      // stored chunk: a plain copy into the dictionary (Lzma2Dec.c:159-166);
      // the next LzmaDec_DecodeToDic uploads it (the mirror's coherence check)
      CLzmaDec* d = &p->decoder;
      memcpy(d->dic + d->dicPos, src, in_cur);
      d->dicPos += in_cur;
      if (d->checkDicSize == 0 && d->prop.dicSize - d->processedPos <= in_cur)
        d->checkDicSize = d->prop.dicSize;
      d->processedPos += UInt32(in_cur);
      src += in_cur;
      *srcLen += in_cur;
      p->unpackSize -= UInt32(in_cur);
      p->state = (p->unpackSize == 0) ? S2_CONTROL : S2_DATA_CONT;
    } else {
      if (p->state == S2_DATA) {
        const int mode = (p->control >> 5) & 3;
        const bool init_dic = (mode == 3), init_state = (mode > 0);
        if ((!init_dic && p->needInitDic) || (!init_state && p->needInitState))
          return SZ_ERROR_DATA;
        LzmaDec_InitDicAndState(&p->decoder, init_dic, init_state);
        p->needInitDic = 0;
        p->needInitState = 0;
        p->state = S2_DATA_CONT;
      }
      if (in_cur > p->packSize) in_cur = p->packSize;
      SRes r = LzmaDec_DecodeToDic(&p->decoder, pos0 + out_cur, src, &in_cur, fin_cur, status);
      src += in_cur;
      *srcLen += in_cur;
      p->packSize -= UInt32(in_cur);
      const SizeT produced = p->decoder.dicPos - pos0;
      p->unpackSize -= UInt32(produced);
      if (r != SZ_OK) return r;
      if (*status == LZMA_STATUS_NEEDS_MORE_INPUT) return r;
      if (in_cur == 0 && produced == 0) {
        if (*status != LZMA_STATUS_MAYBE_FINISHED_WITHOUT_MARK || p->unpackSize != 0 ||
            p->packSize != 0)
          return SZ_ERROR_DATA;
        p->state = S2_CONTROL;
      }
      if (*status == LZMA_STATUS_MAYBE_FINISHED_WITHOUT_MARK) *status = LZMA_STATUS_NOT_FINISHED;
    }
  }
  *status = LZMA_STATUS_FINISHED_WITH_MARK;
  return SZ_OK;
}

SRes Lzma2Dec_DecodeToBuf(CLzma2Dec* p, Byte* dest, SizeT* destLen, const Byte* src,
                          SizeT* srcLen, ELzmaFinishMode finishMode, ELzmaStatus* status) {
  SizeT out_left = *destLen, in_left = *srcLen;
  *srcLen = 0;
  *destLen = 0;
  for (;;) {
    SizeT in_cur = in_left, lim, start;
    ELzmaFinishMode fin_cur;
    CLzmaDec* d = &p->decoder;
    if (d->dicPos == d->dicBufSize) d->dicPos = 0;
    start = d->dicPos;
    if (out_left > d->dicBufSize - start) {
      lim = d->dicBufSize;
      fin_cur = LZMA_FINISH_ANY;
    } else {
      lim = start + out_left;
      fin_cur = finishMode;
    }
    SRes r = Lzma2Dec_DecodeToDic(p, lim, src, &in_cur, fin_cur, status);
    src += in_cur;
    in_left -= in_cur;
    *srcLen += in_cur;
    const SizeT produced = d->dicPos - start;
    memcpy(dest, d->dic + start, produced);
    dest += produced;
    out_left -= produced;
    *destLen += produced;
    if (r != SZ_OK) return r;
    if (produced == 0 || out_left == 0) return SZ_OK;
  }
}

SRes Lzma2Decode(Byte* dest, SizeT* destLen, const Byte* src, SizeT* srcLen, Byte prop,
                 ELzmaFinishMode finishMode, ELzmaStatus* status, ISzAlloc* alloc) {
  const SizeT in_size = *srcLen, out_size = *destLen;
  *destLen = 0;
  *srcLen = 0;
  *status = LZMA_STATUS_NOT_SPECIFIED;
  Byte props[LZMA_PROPS_SIZE];
  SRes r = lzma2_props(prop, props);
  if (r != SZ_OK) return r;
  void* host_probs = alloc->Alloc(alloc, size_t(probs_for(4, 0)) * sizeof(CLzmaProb));
  if (host_probs == nullptr) return SZ_ERROR_MEM;
  SizeT sl = in_size, dl = out_size;
  int st = -1;
  r = gpu_one_call(LZMA_GPU_KIND_LZMA2, dest, &dl, src, &sl, &prop, 1, finishMode, &st);
  if (r == SZ_OK && st == LZMA_STATUS_NEEDS_MORE_INPUT) r = SZ_ERROR_INPUT_EOF;  // Lzma2Dec.c:350
  alloc->Free(alloc, host_probs);
  *srcLen = sl;
  *destLen = dl;
  if (st >= 0) *status = ELzmaStatus(st);
  return r;
}

}  // extern "C"

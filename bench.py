"""bench.py -- batch LZMA decode throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scaling weak|strong]
                    [--config cfg3|cfg1|cfg2|cfg4|cfg5|xz|7z] [--streams S]

One "step" = one launch of the batch decode kernel over the whole per-GPU
batch (inputs already resident in HBM, outputs written to HBM).  Default
workload = BASELINE config 3, the 64K-stream batch: 65,536 independent
streams x 4,096 B of synthetic English-like text, lc0/lp0/pb0, 4 KiB dict.

Multi-GPU: one process per GPU.  Under torch.distributed.run the ranks come
from the environment; `bench.py --gpus N` started on its own spawns the N
rank processes itself (before anything touches a GPU) on 127.0.0.1.  Streams
are sharded with no data-path collective: --scaling weak (default) gives
every rank its own 65,536-stream batch, --scaling strong splits one fixed
65,536-stream batch over the ranks.  Timing is barrier + synchronize
bracketed, MAX over ranks; value = all ranks' decompressed bytes / that time.

Rank 0 prints ONE JSON line.  It carries the live roofline of the decode
kernel (HIP events on the launch stream), the issue-side counters of the
committed rocprof profile, an end-to-end (H2D + decode + D2H, pinned host
buffers) rate, and the CPU baseline: the reference's own LzmaDecode
(oracle/_ref/libref_lzma.so, LzmaDec.c compiled in place, "kind": "reference";
the oracle restatement oracle/liboracle.so, "kind": "port", where that library
is absent) timed on every host core this job may use over the same batch, on
rank 0 after the timed region at any world size.  The output is poisoned and
every timed step writes its own poisoned results array, so `verified` covers
each timed launch (bit-exact output, exact per-stream results).

--config cfg4: 1 MiB LZMA2 dict-reset blocks, 1024
per GPU, one compressed file on rank 0 scattered to the peers over RCCL
(grouped point-to-point, the only data exchange of the path), one block per
lane; the scatter is timed and reported separately.
--dry-run: the launcher, sharding and reductions on CPU (gloo), no decode --
the multi-rank plumbing test (tests/test_dist.py).
"""
import argparse
import ctypes
import hashlib
import json
import lzma
import multiprocessing as mp
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "lzma-sdk-zliblike_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

CONFIGS = {
    # name: (streams, stream_bytes, lc, lp, pb, dict, description)
    "cfg3": (65536, 4096, 0, 0, 0, 4096,
             "65536 x 4096 B streams, lc0/lp0/pb0, 4 KiB dict (BASELINE config 3, 64K-stream batch)"),
    "cfg2": (4096, 65536, 3, 0, 2, 65536,
             "4096 x 65536 B streams, lc3/lp0/pb2, 64 KiB dict (BASELINE config 2)"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def pool_map(fn, jobs, workers, chunksize=1):
    """imap_unordered over a fork pool that is closed and joined when done,
    never terminated: `with Pool()` calls terminate() on exit, which SIGTERMs
    the workers -- forked under rocprofv3 they carry its signal handler, and
    the profile record then shows an abort."""
    pool = mp.get_context("fork").Pool(workers)
    try:
        for r in pool.imap_unordered(fn, jobs, chunksize=chunksize):
            yield r
    finally:
        pool.close()
        pool.join()


def _compress_range(args):
    plain_path, n, lc, lp, pb, dsz, lo, hi = args
    mm = np.memmap(plain_path, dtype=np.uint8, mode="r")
    filt = [{"id": lzma.FILTER_LZMA1, "dict_size": dsz, "lc": lc, "lp": lp, "pb": pb, "preset": 6}]
    out = []
    for i in range(lo, hi):
        out.append(lzma.compress(mm[i * n:(i + 1) * n].tobytes(), format=lzma.FORMAT_RAW,
                                 filters=filt))
    return lo, out


def build_workload(cfg, first, count, workers):
    """Streams [first, first + count) of config `cfg`'s global stream sequence
    (stream i: plaintext from the C generator seeded by its global index i,
    liblzma-encoded).  Cached under $TMPDIR keyed by config + range."""
    _, n, lc, lp, pb, dsz, _ = CONFIGS[cfg]
    tmp = os.environ.get("TMPDIR", "/tmp")
    key = f"lzgpu_{cfg}_{first}_{count}_v2"
    plain_path = os.path.join(tmp, key + ".plain")
    comp_path = os.path.join(tmp, key + ".comp.npz")
    import native
    if not os.path.exists(plain_path):
        plain = np.zeros(count * n, dtype=np.uint8)
        native.synth().synth_batch(0, first, plain.ctypes.data, n, count, max(1, workers))
        plain.tofile(plain_path)
    plain = np.fromfile(plain_path, dtype=np.uint8)
    if os.path.exists(comp_path):
        z = np.load(comp_path)
        comp, lens = z["comp"], z["lens"]
    else:
        t0 = time.time()
        chunk = max(64, count // (workers * 8))
        jobs = [(plain_path, n, lc, lp, pb, dsz, lo, min(lo + chunk, count))
                for lo in range(0, count, chunk)]
        parts = [None] * count
        for lo, out in pool_map(_compress_range, jobs, workers):
            for k, c in enumerate(out):
                parts[lo + k] = c
        lens = np.array([len(c) for c in parts], dtype=np.uint64)
        comp = np.frombuffer(b"".join(parts), dtype=np.uint8)
        np.savez(comp_path, comp=comp, lens=lens)
        log(f"[{cfg}] compressed streams {first}..{first + count - 1} in {time.time() - t0:.1f}s "
            f"with {workers} workers")
    props = bytes([(pb * 5 + lp) * 9 + lc]) + dsz.to_bytes(4, "little")
    return plain, comp, lens, props


def rank_streams(count, world, rank, scaling):
    """This rank's [first, first + n) of the stream sequence: weak = its own
    `count`-stream batch, strong = its shard of one `count`-stream batch."""
    import dist_bench as D
    if scaling == "strong":
        return D.shard(count, world, rank)
    return rank * count, count


def cpu_info():
    """Host CPUs this job may use: affinity mask, cgroup CPU quota, model."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    usable = min(aff, quota) if quota else aff
    return {"model": model, "host_cpus": os.cpu_count(), "affinity_cpus": aff,
            "cgroup_quota_cpus": quota, "usable": usable}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(nranks):
    """bench.py --gpus N run without torch.distributed.run: start N fresh rank
    processes (this parent never touches a GPU, so nothing is re-executed
    after a GPU init), each with RANK / LOCAL_RANK / WORLD_SIZE and a
    127.0.0.1 rendezvous; rank 0 prints the JSON line.  Returns the worst
    exit code."""
    port = _free_port()
    procs = []
    for r in range(nranks):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nranks),
                   LOCAL_WORLD_SIZE=str(nranks), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   LZGPU_BENCH_CHILD="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rcs = [p.wait() for p in procs]
    return max(rcs, key=abs)


def gather_ranks(obj):
    """Every rank's `obj`, in rank order (all_gather_object; [obj] at world 1)."""
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def run_dry(args):
    """--dry-run: launcher + sharding + reductions on the gloo backend, no GPU
    and no decode (the CPU test of the multi-rank plumbing).  Prints the line
    shape the GPU run prints, with value null."""
    import dist_bench as D
    import torch.distributed as dist
    world, rank, _ = D.world_info()
    if world > 1:
        dist.init_process_group("gloo")
    count = CONFIGS[args.config][0] if args.config in CONFIGS else 0
    first, mine = rank_streams(count, world, rank, args.scaling)
    D.barrier()
    elapsed = D.reduce_max(0.001 * (rank + 1))
    ranks = gather_ranks({"rank": rank, "first": first, "streams": mine})
    total = int(D.reduce_sum(float(mine)))
    cpu = None
    if rank == 0 and not args.no_cpu_baseline and args.config in CONFIGS:
        # the same object shape the GPU run emits at any world size, on a small
        # sample (the plumbing test: rank 0, after the timed region)
        import native
        _, n, lc, lp, pb, dsz, _ = CONFIGS[args.config]
        ci = cpu_info()
        m = 64
        plain, comp, lens, props = build_workload(args.config, 0, m, 1)
        offs = np.zeros(m, dtype=np.uint64)
        offs[1:] = np.cumsum(lens)[:-1]
        kind = "reference" if native.have_ref() else "port"
        v, dt, mm, errs = cpu_baseline(comp, lens, offs, n, props, ci["usable"], m, kind)
        cpu = {"value": round(v, 2), "unit": "MB/s", "cores": ci["usable"], "kind": kind,
               "sample": f"{mm} streams of {args.config} (dry run), {dt:.3f}s", "cpu": ci,
               "errors": int(errs)}
    if rank == 0:
        print(json.dumps({
            "metric": "decompressed MB/s (whole node), 64K-stream batch; bit-exact vs CPU LzmaDec",
            "value": None, "unit": "MB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "scaling": args.scaling, "dry_run": True,
            "world": dist.get_world_size() if dist.is_initialized() else 1,
            "backend": dist.get_backend() if dist.is_initialized() else None,
            "streams_total": total, "elapsed_max_s": elapsed, "ranks": ranks,
            "cpu_baseline": cpu}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


RES_DT = np.dtype([("res", "<i4"), ("status", "<i4"), ("dest_len", "<u8"), ("src_len", "<u8")])


def poison(torch, t):
    """Overwrite a device output buffer with seeded random bytes (outside any
    timed region).  Not a constant: a buffer filled with one byte value (0xA5)
    made the next decode into it 15 % slower on MI355X (config 4: 412 vs 357 ms;
    other real data or random bytes in the buffer: 357 ms) -- uniform lines are
    handled differently by the memory system, and output buffers in use hold
    earlier, non-uniform data.  LZGPU_BENCH_POISON=const
    restores the constant fill (diagnostic)."""
    if os.environ.get("LZGPU_BENCH_POISON") == "const":
        t.fill_(0xA5)
        return
    g = torch.Generator(device=t.device)
    g.manual_seed(0xA5)
    flat = t.view(-1)
    step = 1 << 28  # in pieces: no 1 GiB temporary beside a 1 GiB output
    for a in range(0, flat.numel(), step):
        piece = flat[a:a + step]
        piece.copy_(torch.randint(0, 256, piece.shape, dtype=torch.uint8, device=t.device,
                                  generator=g))


def timed_buffers(torch, dev, d_dst, count, steps):
    """Poison for the timed loop (outside its events): the output is filled with
    random bytes (poison()) and every timed step gets its OWN results array
    filled with 0xFF (res = -1).  Afterwards the output must equal the
    plaintext and every step's array must hold every stream's exact answer, so
    `verified` covers each timed launch: one that decoded nothing leaves its
    array poisoned."""
    poison(torch, d_dst)
    r = torch.full((max(steps, 1), count * 24), 0xFF, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    return r


def step_results(d_res_steps):
    """Every timed step's results, as a (steps, count) structured array."""
    raw = d_res_steps.cpu().numpy()
    return np.stack([np.frombuffer(raw[k].tobytes(), dtype=RES_DT) for k in range(raw.shape[0])])


def plan_kernels(plan):
    """Names of the kernels a plan launches (one per LDS class, + the generic one)."""
    names = []
    for c in list(plan.classes)[:int(plan.n_classes)]:
        if int(c.n) == 0:
            continue
        m = int(c.lds_mask)
        dup = int(os.environ.get("LZGPU_DUP", "32") or 0)  # lzma_kernels.hip kLaneDup
        if m & 0x80000000:
            k = "lzgpu_decode_coop_kernel"
        elif m in (0x1BF, 0x19F) and int(c.lanes_per_group) == 1 and 1 < dup <= 64:
            k = "lzgpu_decode_dup_kernel"  # one-stream waves on all 32 lanes
        else:
            k = "lzgpu_decode_lds_kernel"
        if k not in names:
            names.append(k)
    if int(plan.n) > int(plan.n_lds):
        names.append("lzgpu_decode_batch_kernel")
    return " + ".join(names) if names else None


def make_descs(lens, n, props, finish=1):
    import lzmagpu as L
    count = len(lens)
    descs = (L.StreamDesc * count)()
    arr = np.frombuffer(descs, dtype=np.uint8).reshape(count, 48)
    offs = np.zeros(count, dtype=np.uint64)
    offs[1:] = np.cumsum(lens)[:-1]
    u64 = arr[:, :40].view(np.uint64)
    u64[:, 0] = offs
    u64[:, 1] = lens
    u64[:, 2] = np.arange(count, dtype=np.uint64) * n
    u64[:, 3] = n
    arr[:, 40:45] = np.frombuffer(props, dtype=np.uint8)
    arr[:, 45] = 5
    arr[:, 46] = finish
    arr[:, 47] = L.KIND_LZMA
    plan, order = L.plan_ex(descs)
    return descs, order, plan, offs


def measure_crc(L, torch, descs, d_desc, d_res, d_dst, plain, count, n, stream, dev, steps):
    """CRC-32 of every decoded stream straight from the decode's device buffers
    (LzmaGpu_Crc32Batch), timed apart from the decode with
    HIP events on the same stream; checked against zlib.crc32 (same CRC-32)."""
    import zlib
    base, crange, total = L.crc32_plan_decoded(descs)
    d_base = torch.frombuffer(bytearray(base), dtype=torch.uint8).to(dev)
    d_range = torch.frombuffer(bytearray(crange), dtype=torch.uint8).to(dev)
    d_chunks = torch.empty(max(total, 1) * 4, dtype=torch.uint8, device=dev)
    d_crc = torch.empty(count * 4, dtype=torch.uint8, device=dev)
    sh = stream.cuda_stream

    def run():
        r = L.crc32_batch_decoded(d_desc.data_ptr(), d_res.data_ptr(), count, d_dst.data_ptr(),
                                  d_base.data_ptr(), d_range.data_ptr(), total,
                                  d_chunks.data_ptr(), d_crc.data_ptr(), sh)
        if r != 0:
            raise RuntimeError("LzmaGpu_Crc32Batch failed: " + L.last_error())

    run()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(steps)]
    for a, b in evs:
        a.record(stream)
        run()
        b.record(stream)
    torch.cuda.synchronize()
    ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    got = np.frombuffer(d_crc.cpu().numpy().tobytes(), dtype="<u4")
    rows = plain.reshape(count, n)
    want = np.array([zlib.crc32(rows[i].tobytes()) for i in range(count)], dtype=np.uint32)
    # bytes per launch: decoded output read once + chunk registers written and re-read
    alg = count * n
    moved = alg + 8 * total + count * (8 + 8 + 4)
    gbs = moved / (ms * 1e-3) / 1e9
    return {"kernels": "lzgpu_crc_chunk_kernel + lzgpu_crc_fold_kernel",
            "value": round(alg / (ms * 1e-3) / 1e6, 2), "unit": "MB/s", "avg_ms": round(ms, 4),
            "chunks": int(total),
            "roofline": {"bound": "hbm", "achieved": round(gbs, 3), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                         "alg_bytes_per_launch": int(moved)},
            "verified": bool(np.array_equal(got, want))}


# ---------------------------------------------------------------- config 1

def run_cfg1(args):
    """Config 1: ONE 1 MiB stream (lc3/lp0/pb2, 64 KiB dict) --
    plumbing and bit-exactness of the single-stream path, timed beside the
    reference's own LzmaDecode on one host core.  The stream is the committed
    reference-encoded golden (tests/golden/cfg1_blob.bin; enwik8 is not
    available offline: synthetic text).

    value: the device-resident decode (the stream already in HBM, one launch of
    the batch API with n = 1 on the wave-cooperative kernel, output left in
    HBM), K steps between barrier + synchronize.  Beside it, over host buffers
    (PCIe-inclusive, never `value`): the drop-in LzmaDecode, the fork's
    DecodeToBuf loop (512 KiB in / 1 MiB out, 7zDec.c:567-648) and the
    7zDec.c:127-171 DecodeToDic loop (16 KiB look windows over a whole-output
    dictionary, the device mirror), each checked against the reference's
    recorded answers.  One stream is one serial range-decoder chain: a GPU wave
    decides it far slower than a CPU core does; the batch configs are where the
    GPU's throughput is."""
    import hashlib
    import dist_bench as D
    world, rank, local_rank = D.world_info()
    gold = os.path.join(ROOT, "tests", "golden")
    doc = json.load(open(os.path.join(gold, "cfg1_cases.json")))
    comp = open(os.path.join(gold, "cfg1_blob.bin"), "rb").read()
    props = bytes.fromhex(doc["props"])
    n = doc["plaintext"]["bytes"]
    want_sha = doc["plaintext"]["sha256"]
    exp = {(c["kind"], c.get("dest_cap"), c.get("finish"), c.get("in_chunk"), c.get("win")):
           c["expect"] for c in doc["cases"]}
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    import lzmagpu as L

    def sha(b):
        return hashlib.sha256(b).hexdigest()

    # ---- device-resident: one stream, batch API n = 1 (cooperative plan)
    descs = L.make_descs([dict(src_off=0, src_len=len(comp), dst_off=0, dst_cap=n, props=props,
                               finish=1, kind=L.KIND_LZMA)])
    plan, order = L.plan_ex(descs, L.plan_options("coop"))
    d_src = torch.frombuffer(bytearray(comp + bytes(16)), dtype=torch.uint8).to(dev)
    d_dst = torch.empty(n + 16, dtype=torch.uint8, device=dev)
    d_ws = torch.empty(max(int(plan.workspace_bytes), 16), dtype=torch.uint8, device=dev)
    d_desc = torch.frombuffer(bytearray(bytes(descs)), dtype=torch.uint8).to(dev)
    d_order = torch.frombuffer(bytearray(bytes(order)), dtype=torch.uint8).to(dev)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream

    def step(res):
        if L.decode_batch_device_ex(plan, d_desc.data_ptr(), d_order.data_ptr(), d_src.data_ptr(),
                                    d_dst.data_ptr(), d_ws.data_ptr(), res.data_ptr(), sh):
            raise RuntimeError("LzmaGpu_DecodeBatchEx failed: " + L.last_error())

    d_res0 = torch.empty(24, dtype=torch.uint8, device=dev)
    for _ in range(args.warmup):
        step(d_res0)
    torch.cuda.synchronize()
    d_res_steps = timed_buffers(torch, dev, d_dst, 1, args.steps)
    D.barrier()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k, (a, b) in enumerate(evs):
        a.record(stream)
        step(d_res_steps[k])
        b.record(stream)
    torch.cuda.synchronize()
    D.barrier()
    torch.cuda.synchronize()
    elapsed = D.reduce_max(time.perf_counter() - t0, dev)
    dec_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    e_end = exp[("lzma", n, 1, None, None)]
    allres = step_results(d_res_steps)
    ok = bool((allres["res"] == e_end["res"]).all() and (allres["status"] == e_end["status"]).all()
              and (allres["dest_len"] == e_end["dest_len"]).all()
              and (allres["src_len"] == e_end["src_len"]).all())
    ok = ok and sha(d_dst[:n].cpu().numpy().tobytes()) == want_sha

    # ---- host buffers through the drop-in API (PCIe-inclusive)
    dropin = {}
    t0 = time.perf_counter()
    k_calls = max(1, min(args.steps, 5))
    for _ in range(k_calls):
        r = L.LzmaDecode(comp, props, n, 1)
        ok = ok and (r[0], r[1], r[2], r[3], sha(r[4])) == (
            e_end["res"], e_end["status"], e_end["dest_len"], e_end["src_len"], e_end["sha256"])
    dt = (time.perf_counter() - t0) / k_calls
    dropin["LzmaDecode"] = {"MBps": round(n / dt / 1e6, 3), "ms_per_call": round(dt * 1e3, 3)}
    t0 = time.perf_counter()
    r = L.LzmaUncompress(comp, props, n)
    dt = time.perf_counter() - t0
    e_any = exp[("lzma", n, 0, None, None)]
    ok = ok and (r[0], r[1], r[2], sha(r[3])) == (e_any["res"], e_any["dest_len"],
                                                  e_any["src_len"], e_any["sha256"])
    dropin["LzmaUncompress"] = {"MBps": round(n / dt / 1e6, 3), "ms_per_call": round(dt * 1e3, 3)}
    L.transfer_stats(reset=True)
    t0 = time.perf_counter()
    calls, trace, out, used = L.stream_decode(comp, props, n, 1 << 19, 1 << 20, 0)
    dt = time.perf_counter() - t0
    h2d, d2h, _ = L.transfer_stats(reset=True)
    e_st = exp[("stream", None, 0, 1 << 19, None)]
    ok = ok and [list(t) for t in trace] == e_st["trace"] and sha(out) == e_st["sha256"]
    dropin["DecodeToBuf_512K_in_1M_out"] = {"MBps": round(n / dt / 1e6, 3), "calls": calls,
                                            "h2d_bytes": h2d, "d2h_bytes": d2h}
    t0 = time.perf_counter()
    calls, trace, out, used = L.dic_decode(comp, props, n, 1 << 14)
    dt = time.perf_counter() - t0
    h2d, d2h, _ = L.transfer_stats(reset=True)
    e_dic = exp[("dic", None, None, None, 1 << 14)]
    ok = ok and [list(t) for t in trace] == e_dic["trace"] and sha(out) == e_dic["sha256"]
    dropin["DecodeToDic_16K_windows"] = {"MBps": round(n / dt / 1e6, 3), "calls": calls,
                                         "h2d_bytes": h2d, "d2h_bytes": d2h,
                                         "compressed_bytes": len(comp),
                                         "note": "device dictionary mirror: each call uploads "
                                                 "its input window + the 192-byte state"}
    # the 7zDec pattern over a dictionary far larger than the stream: a 64 MiB
    # dic (a whole folder's output buffer) decoded through 16 KiB windows --
    # round 2 uploaded dicBufSize on every call (quadratic); the mirror uploads
    # the windows.  Per-call parity against the oracle's identical loop.
    import native
    big = 64 << 20
    L.transfer_stats(reset=True)
    t0 = time.perf_counter()
    calls, trace, out, used = L.dic_decode(comp, props, big, 1 << 14)
    dt = time.perf_counter() - t0
    h2d, d2h, _ = L.transfer_stats(reset=True)
    w = native.dic_decode(native.oracle(), "orc", comp, props, big, 1 << 14)
    ok = ok and [tuple(t) for t in trace] == [tuple(t) for t in w[1]] and out == w[2] \
        and sha(out) == want_sha
    dropin["DecodeToDic_16K_windows_64MiB_dic"] = {
        "MBps": round(len(out) / dt / 1e6, 3), "calls": calls, "h2d_bytes": h2d,
        "d2h_bytes": d2h, "round2_h2d_bytes_would_be": calls * big,
        "note": "dicBufSize 64 MiB, the 1 MiB stream decoded into its start; trace equal "
                "to the oracle's loop"}
    ok = D.all_true(ok, dev)

    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        if native.have_ref():
            lib, pre, kind = native.ref(), "ref", "reference"
        else:
            lib, pre, kind = native.oracle(), "orc", "port"
        reps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < 3.0 or reps < 3:
            r = native.decode(lib, pre, comp, props, n, 1)
            reps += 1
        dt = (time.perf_counter() - t0) / reps
        cpu = {"value": round(n / dt / 1e6, 2), "unit": "MB/s", "cores": 1, "kind": kind,
               "impl": "the reference's LzmaDecode (LzmaDec.c:972, oracle/_ref/libref_lzma.so, "
                       "gcc -O2, compiled in place)" if kind == "reference" else
                       "oracle/lzma_oracle.c restatement",
               "sample": f"the same 1 MiB stream decoded {reps} times on one core, "
                         f"{dt * 1e3:.2f} ms per call",
               "verified": sha(r[4]) == want_sha}
        if kind == "reference":
            _, _, out, _, ns = native.dic_decode(lib, pre, comp, props, n, 1 << 14)
            cpu["DecodeToDic_16K_windows_MBps"] = round(n / (ns * 1e-9) / 1e6, 2)
    value = world * n * args.steps / elapsed / 1e6
    alg = len(comp) + 5 + n
    achieved = alg / (dec_ms * 1e-3) / 1e9
    if rank == 0:
        print(json.dumps({
            "metric": "decompressed MB/s, config 1: one 1 MiB stream (single-stream path)",
            "value": round(value, 3), "unit": "MB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic text (1 MiB, seed 1), reference-encoded (tests/golden/cfg1_blob.bin)",
            "config": {"workload": "1 stream x 1 MiB, lc3/lp0/pb2, 64 KiB dict (BASELINE config 1)",
                       "compressed_bytes": len(comp),
                       "kernel_plan": {"kernel": plan_kernels(plan),
                                       "placement": hex(plan.classes[0].lds_mask)
                                       if plan.n_classes else None}},
            "roofline": {"bound": "issue", "priced_against": "hbm", "achieved": round(achieved, 4),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 8), "traffic": None,
                         "kernel": plan_kernels(plan), "kernel_avg_ms": round(dec_ms, 4),
                         "alg_bytes_per_launch": alg},
            "dropin_host_buffers": dropin,
            "cpu_baseline": cpu, "verified": ok}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


# ---------------------------------------------------------------- config 4

CFG4_BLOCK = 1 << 20     # 1 MiB dict-reset blocks (Lzma2Enc.c MT layout)
CFG4_PROP = 16           # LZMA2 dict prop: 1 MiB
CFG4_UNIQUE = 1024       # distinct blocks generated (one GPU's worth); larger files repeat them


def _compress_lzma2_block(i):
    import native
    data = native.gen("text", 50000 + i, CFG4_BLOCK)
    f = [{"id": lzma.FILTER_LZMA2, "dict_size": CFG4_BLOCK, "lc": 3, "lp": 0, "pb": 2,
          "preset": 6}]
    c = lzma.compress(data, format=lzma.FORMAT_RAW, filters=f)
    assert c[-1] == 0
    return i, c[:-1], zlib_crc(data)


def zlib_crc(b):
    import zlib
    return zlib.crc32(b)


def build_cfg4_unique(workers):
    tmp = os.environ.get("TMPDIR", "/tmp")
    path = os.path.join(tmp, f"lzgpu_cfg4_u{CFG4_UNIQUE}_v1.npz")
    if os.path.exists(path):
        z = np.load(path)
        comp, lens, crcs = z["comp"], z["lens"], z["crcs"]
        parts, o = [], 0
        for ln in lens:
            parts.append(comp[o:o + int(ln)].tobytes())
            o += int(ln)
        return parts, [int(c) for c in crcs]
    t0 = time.time()
    parts, crcs = [None] * CFG4_UNIQUE, [0] * CFG4_UNIQUE
    for i, c, crc in pool_map(_compress_lzma2_block, range(CFG4_UNIQUE), workers):
        parts[i], crcs[i] = c, crc
    np.savez(path, comp=np.frombuffer(b"".join(parts), dtype=np.uint8),
             lens=np.array([len(c) for c in parts], dtype=np.uint64),
             crcs=np.array(crcs, dtype=np.uint64))
    log(f"[rank 0] compressed {CFG4_UNIQUE} LZMA2 blocks in {time.time() - t0:.1f}s")
    return parts, crcs


def print_prof(L):
    """Region cycles and counters of a profiling build (LZGPU_PROF), else nothing."""
    if hasattr(L.lib, "LzmaGpu_ProfileRead"):  # profiling variant builds only
        buf = (ctypes.c_ulonglong * 40)()
        L.lib.LzmaGpu_ProfileRead(buf, 0)
        lanes = max(1, buf[23])
        if buf[22] == 3:
            # wait attribution (lzma_device.h LZGPU_PROF=3): cycles per stream the
            # wave spent in forced vmcnt(0) waits, by class, and the stream's total
            w = ("drain_stores", "matched_literal", "rep", "length", "slot", "specpos", "align",
                 "lenhigh", "copy_region", "matched_byte", "input", "prev_probe")
            prof = {k: buf[24 + i] / lanes for i, k in enumerate(w)}
            prof["stream_total"] = buf[3] / lanes
            prof["bytes"] = buf[12] / lanes
            log("PROF3 per stream (cycles, wave time per lane): " + json.dumps(
                {k: round(v) for k, v in prof.items()}))
            return
        # "a|b|c": the counter's meaning in the per-lane (PROF=2) / global-slot /
        # LDS-slot (cooperative, round 4) builds
        names = ("literal_batches", "match_decode", "copy_tail", "decode_to_dic_total",
                 "refills", "batch_iters|slot_sub3_a|cyc_slot",
                 "lit_lanes|slot_sub3_b|cyc_direct", "mlit_lanes|n_slot|cyc_align",
                 "mixed_iters|cyc_rep_bits", "match_entries|cyc_len", "match_lanes|cyc_dist",
                 "live_lanes|n_dist", "bytes", "matches|cyc_drain|cyc_specpos",
                 "cyc_ismatch", "cyc_literal", "cyc_lit_tail", "cyc_iterations",
                 "cyc_input_tail", "tail_passes", "cyc_table_init")
        prof = {k: buf[i] / lanes for i, k in enumerate(names)}
        prof["other_in_decode_to_dic"] = prof["decode_to_dic_total"] - sum(
            prof[k] for k in names[:3])  # refills overlap the first three regions
        log("PROF per stream (cycles: lane-summed wave time; counts: wave-level "
            "seen by each lane): " + json.dumps(
            {k: round(v) for k, v in prof.items()}))


def run_cfg4(args):
    import dist_bench as D
    world, rank, local_rank = D.world_info()
    cpus = cpu_info()["usable"]
    workers = max(1, min(16, cpus // max(1, world)))
    B = args.blocks
    parts = crcs = None
    if rank == 0:
        parts, crcs = build_cfg4_unique(workers)  # before the GPU is touched (fork pool)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    import lzmagpu as L
    # rank 0: the whole file (world x B blocks + EOS) and its block table
    meta = [None]
    if rank == 0:
        seq = [b % CFG4_UNIQUE for b in range(world * B)]
        blob = b"".join(parts[u] for u in seq) + b"\0"
        blocks = L.split_lzma2_blocks(blob)  # host header walk, O(#chunks)
        assert len(blocks) == world * B
        ranges = [(int(blocks[r * B][0]), int(blocks[(r + 1) * B - 1][0] + blocks[(r + 1) * B - 1][1]))
                  for r in range(world)]
        table = [[(int(o), int(ln), int(u)) for o, ln, u in blocks[r * B:(r + 1) * B]]
                 for r in range(world)]
        meta = [(ranges, table, [crcs[u] for u in seq], len(blob))]
        d_file = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
    if world > 1:
        dist.broadcast_object_list(meta, src=0)
    ranges, table, crc_seq, file_bytes = meta[0]
    lo, hi = ranges[rank]
    mine = table[rank]
    d_src = torch.empty(max(hi - lo, 16) + 16, dtype=torch.uint8, device=dev)
    if world == 1:
        d_src[:hi - lo].copy_(d_file[lo:hi])
    items, doff = [], 0
    for o, ln, u in mine:
        items.append(dict(src_off=o - lo, src_len=ln, dst_off=doff, dst_cap=u,
                          props=bytes([CFG4_PROP]), finish=0, kind=L.KIND_LZMA2))
        doff += u
    descs = L.make_descs(items)
    plan, order = L.plan_ex(descs)
    d_dst = torch.empty(doff + 16, dtype=torch.uint8, device=dev)
    d_ws = torch.empty(max(int(plan.workspace_bytes), 16), dtype=torch.uint8, device=dev)
    d_desc = torch.frombuffer(bytearray(bytes(descs)), dtype=torch.uint8).to(dev)
    d_order = torch.frombuffer(bytearray(bytes(order)), dtype=torch.uint8).to(dev)
    d_res = torch.empty(B * 24, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    out_view = d_src[:hi - lo]

    def scatter():
        if world > 1:
            D.scatter_ranges(d_file if rank == 0 else None, ranges, out_view, rank, world)

    def decode(res=None):
        res = d_res if res is None else res
        r = L.decode_batch_device_ex(plan, d_desc.data_ptr(), d_order.data_ptr(), d_src.data_ptr(),
                                     d_dst.data_ptr(), d_ws.data_ptr(), res.data_ptr(), sh)
        if r != 0:
            raise RuntimeError("LzmaGpu_DecodeBatchEx failed: " + L.last_error())

    for _ in range(args.warmup):
        scatter()
        decode()
    torch.cuda.synchronize()
    d_res_steps = timed_buffers(torch, dev, d_dst, B, args.steps)
    if world > 1:
        poison(torch, out_view)  # the scatter must deliver this rank's bytes again
        torch.cuda.synchronize()
    D.barrier()
    torch.cuda.synchronize()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        scatter()
        ev[i][1].record(stream)
        decode(d_res_steps[i])
        ev[i][2].record(stream)
    torch.cuda.synchronize()
    D.barrier()
    torch.cuda.synchronize()
    elapsed = D.reduce_max(time.perf_counter() - t0, dev)
    print_prof(L)
    scat_ms = float(np.mean([a.elapsed_time(b) for a, b, _ in ev]))
    dec_steps = [b.elapsed_time(c) for _, b, c in ev]
    dec_ms = float(np.mean(dec_steps))
    scat_ms = D.reduce_max(scat_ms, dev)

    # optional last exchange: every rank's decoded blocks
    # gathered on rank 0 by grouped point-to-point receives; timed on its own
    gather = None
    if world > 1 and not args.no_gather:
        sizes = [int(sum(u for _, _, u in table[r])) for r in range(world)]
        whole = torch.empty(sum(sizes), dtype=torch.uint8, device=dev) if rank == 0 else None
        D.barrier()
        g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        g0.record(stream)
        D.gather_ranges(d_dst, sizes, whole, rank, world)
        g1.record(stream)
        torch.cuda.synchronize()
        g_ms = D.reduce_max(float(g0.elapsed_time(g1)), dev)
        g_ok = True
        if rank == 0:  # each rank's first and last block, by their CRC-32, where they belong
            import zlib
            off = 0
            for r in range(world):
                us = [u for _, _, u in table[r]]
                for j in (0, len(us) - 1):
                    a = off + sum(us[:j])
                    blk = whole[a:a + us[j]].cpu().numpy().tobytes()
                    g_ok = g_ok and zlib.crc32(blk) == crc_seq[r * B + j]
                off += sizes[r]
        gather = {"gather_ms": round(g_ms, 4), "bytes_to_rank0": int(sum(sizes[1:])),
                  "GBps_into_rank0": round(sum(sizes[1:]) / (g_ms * 1e-3) / 1e9, 2),
                  "verified": D.all_true(g_ok, dev)}
        del whole

    # verify every timed launch: per-block results of each step, and the CRC of
    # every decoded block (on the GPU) of the poisoned-then-decoded output
    res = step_results(d_res_steps)
    d_res = d_res_steps[args.steps - 1]
    ok = bool((res["res"] == 0).all() and (res["status"] == 2).all() and
              (res["dest_len"] == np.array([u for _, _, u in mine])[None, :]).all() and
              (res["src_len"] == np.array([ln for _, ln, _ in mine])[None, :]).all())
    base, crange, total = L.crc32_plan_decoded(descs)
    d_base = torch.frombuffer(bytearray(base), dtype=torch.uint8).to(dev)
    d_range = torch.frombuffer(bytearray(crange), dtype=torch.uint8).to(dev)
    d_chunks = torch.empty(max(total, 1) * 4, dtype=torch.uint8, device=dev)
    d_crc = torch.empty(B * 4, dtype=torch.uint8, device=dev)
    assert L.crc32_batch_decoded(d_desc.data_ptr(), d_res.data_ptr(), B, d_dst.data_ptr(),
                                 d_base.data_ptr(), d_range.data_ptr(), total,
                                 d_chunks.data_ptr(), d_crc.data_ptr(), sh) == 0
    got = np.frombuffer(d_crc.cpu().numpy().tobytes(), dtype="<u4")
    ok = ok and bool(np.array_equal(got, np.array(crc_seq[rank * B:(rank + 1) * B],
                                                  dtype=np.uint32)))
    ok = D.all_true(ok, dev)

    cpu = None
    if rank == 0 and not args.no_cpu_baseline:  # after the timed region, any world size
        cpu = cfg4_cpu_baseline(parts, cpus)
    total_bytes = world * B * CFG4_BLOCK * args.steps
    value = total_bytes / elapsed / 1e6
    comp_bytes = hi - lo
    alg = comp_bytes + B * CFG4_BLOCK
    achieved = alg / (dec_ms * 1e-3) / 1e9
    if rank == 0:
        print(json.dumps({
            "metric": "decompressed MB/s (whole node), config 4: 1 MiB LZMA2 dict-reset blocks",
            "value": round(value, 2), "unit": "MB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": f"synthetic text, {CFG4_UNIQUE} distinct liblzma LZMA2 blocks repeated",
            "config": {"workload": f"{B} x 1 MiB LZMA2 blocks per GPU (lc3/lp0/pb2, dict 1 MiB), "
                                   "one file on rank 0 scattered over RCCL",
                       "blocks_per_gpu": B, "compressed_bytes_per_gpu": comp_bytes,
                       "file_bytes": file_bytes,
                       "kernel_plan": {"lds_streams": int(plan.n_lds),
                                       "streams_per_workgroup": int(plan.lanes_per_group),
                                       "workgroups_per_cu": int(plan.groups_per_cu)},
                       "exchange": {"collective": "grouped P2P isend/irecv from rank 0"
                                    if world > 1 else "none (1 GPU)",
                                    "scatter_ms": round(scat_ms, 4),
                                    "bytes_per_peer": comp_bytes,
                                    "gather": gather}},
            "roofline": {"bound": "issue", "priced_against": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6),
                         "traffic": pmc_traffic("cfg4"), "traffic_source": "profiles/pmc_cfg4.json",
                         "binary": lib_sha256(), "kernel": plan_kernels(plan),
                         "kernel_avg_ms": round(dec_ms, 4), "alg_bytes_per_launch": alg,
                         "kernel_ms_steps": [round(x, 3) for x in dec_steps]},
            "cpu_baseline": cpu, "verified": ok}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


# ---------------------------------------------------------------- config 5

CFG5_STREAMS = 32768


def _cfg5_stream(i):
    """Stream i of config 5: tests/workloads.py cfg5_stream --
    props, dict, length and finish mode seeded by (5, i), liblzma-encoded text."""
    import workloads as W
    data, c, props, fin = W.cfg5_stream(i)
    return i, c, props, len(data), fin, zlib_crc(data)


def build_cfg5(workers, first, count):
    tmp = os.environ.get("TMPDIR", "/tmp")
    path = os.path.join(tmp, f"lzgpu_cfg5_{first}_{count}_v1.npz")
    if os.path.exists(path):
        z = np.load(path)
        return (z["comp"], z["lens"], z["props"], z["n"], z["fin"], z["crc"])
    t0 = time.time()
    out = [None] * count
    for i, c, props, n, fin, crc in pool_map(_cfg5_stream, range(first, first + count),
                                             workers, chunksize=64):
        out[i - first] = (c, props, n, fin, crc)
    comp = np.frombuffer(b"".join(o[0] for o in out), dtype=np.uint8)
    lens = np.array([len(o[0]) for o in out], dtype=np.uint64)
    props = np.frombuffer(b"".join(o[1] for o in out), dtype=np.uint8).reshape(count, 5)
    n = np.array([o[2] for o in out], dtype=np.uint64)
    fin = np.array([o[3] for o in out], dtype=np.uint8)
    crc = np.array([o[4] for o in out], dtype=np.uint32)
    np.savez(path, comp=comp, lens=lens, props=props, n=n, fin=fin, crc=crc)
    log(f"[cfg5] compressed {count} mixed streams in {time.time() - t0:.1f}s")
    return comp, lens, props, n, fin, crc


def run_cfg5(args):
    """Config 5: 32,768 streams of mixed lc/lp/pb, dictionaries and lengths per
    GPU (weak scaling), one batch launch set per step (one LDS launch per
    table-width class), verified by per-stream results and GPU CRC-32."""
    import dist_bench as D
    world, rank, local_rank = D.world_info()
    cpus = cpu_info()["usable"]
    workers = max(1, min(16, cpus // max(1, world)))
    count = args.streams or CFG5_STREAMS
    comp, lens, props, nout, fin, crcs = build_cfg5(workers, rank * count, count)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    import lzmagpu as L
    descs = (L.StreamDesc * count)()
    arr = np.frombuffer(descs, dtype=np.uint8).reshape(count, 48)
    u64 = arr[:, :40].view(np.uint64)
    src_off = np.zeros(count, dtype=np.uint64)
    src_off[1:] = np.cumsum(lens)[:-1]
    dst_off = np.zeros(count, dtype=np.uint64)
    dst_off[1:] = np.cumsum(nout)[:-1]
    u64[:, 0], u64[:, 1], u64[:, 2], u64[:, 3] = src_off, lens, dst_off, nout
    arr[:, 40:45] = props
    arr[:, 45] = 5
    arr[:, 46] = fin
    arr[:, 47] = L.KIND_LZMA
    plan, order = L.plan_ex(descs)
    total_out = int(nout.sum())
    d_src = torch.from_numpy(np.concatenate([comp, np.zeros(16, np.uint8)])).to(dev)
    d_dst = torch.empty(total_out + 16, dtype=torch.uint8, device=dev)
    d_ws = torch.empty(max(int(plan.workspace_bytes), 16), dtype=torch.uint8, device=dev)
    d_desc = torch.frombuffer(bytearray(bytes(descs)), dtype=torch.uint8).to(dev)
    d_order = torch.frombuffer(bytearray(bytes(order)), dtype=torch.uint8).to(dev)
    d_res = torch.empty(count * 24, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream

    def step(res=None):
        res = d_res if res is None else res
        r = L.decode_batch_device_ex(plan, d_desc.data_ptr(), d_order.data_ptr(), d_src.data_ptr(),
                                     d_dst.data_ptr(), d_ws.data_ptr(), res.data_ptr(), sh)
        if r != 0:
            raise RuntimeError("LzmaGpu_DecodeBatchEx failed: " + L.last_error())

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    d_res_steps = timed_buffers(torch, dev, d_dst, count, args.steps)
    D.barrier()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k, (a, b) in enumerate(evs):
        a.record(stream)
        step(d_res_steps[k])
        b.record(stream)
    torch.cuda.synchronize()
    D.barrier()
    torch.cuda.synchronize()
    elapsed = D.reduce_max(time.perf_counter() - t0, dev)
    dec_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    res = step_results(d_res_steps)
    d_res = d_res_steps[args.steps - 1]
    want_status = np.where(fin == 1, 1, 2)[None, :]
    ok = bool((res["res"] == 0).all() and (res["status"] == want_status).all() and
              (res["dest_len"] == nout[None, :]).all() and
              (res["src_len"][:, fin == 1] == lens[None, fin == 1]).all())
    base, crange, total = L.crc32_plan_decoded(descs)
    d_base = torch.frombuffer(bytearray(base), dtype=torch.uint8).to(dev)
    d_range = torch.frombuffer(bytearray(crange), dtype=torch.uint8).to(dev)
    d_chunks = torch.empty(max(total, 1) * 4, dtype=torch.uint8, device=dev)
    d_crc = torch.empty(count * 4, dtype=torch.uint8, device=dev)
    assert L.crc32_batch_decoded(d_desc.data_ptr(), d_res.data_ptr(), count, d_dst.data_ptr(),
                                 d_base.data_ptr(), d_range.data_ptr(), total,
                                 d_chunks.data_ptr(), d_crc.data_ptr(), sh) == 0
    got = np.frombuffer(d_crc.cpu().numpy().tobytes(), dtype="<u4")
    ok = D.all_true(ok and bool(np.array_equal(got, crcs)), dev)
    sliced = None
    if args.sliced:
        def check(rr):
            return bool((rr["res"] == 0).all() and (rr["status"] == want_status[0]).all() and
                        (rr["dest_len"] == nout).all() and
                        (rr["src_len"][fin == 1] == lens[fin == 1]).all())
        sliced = measure_sliced(L, torch, descs, count, d_src, d_dst, dev, args.sliced,
                                min(args.steps, 3), dec_ms, check)
        ok = D.all_true(ok and sliced["verified"], dev)
    value = world * total_out * args.steps / elapsed / 1e6
    alg = int(lens.sum()) + 5 * count + total_out
    achieved = alg / (dec_ms * 1e-3) / 1e9
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:  # after the timed region, any world size
        thr = cpus
        m = min(count, 2048)
        orc_n = nout[:m]
        v, dt, mm, errs = cpu_baseline_mixed(comp, lens, src_off, orc_n, props, fin, thr, m)
        cpu = {"value": round(v, 2), "unit": "MB/s", "cores": thr, "kind": "port",
               "sample": f"first {mm} streams of the batch, {thr} threads, {dt:.2f}s",
               "errors": int(errs)}
    if rank == 0:
        cls = [{"streams": int(c.n), "streams_per_workgroup": int(c.lanes_per_group),
                "lds_bytes_per_stream": int(c.lds_cells_per_lane) * 2,
                "workgroups_per_cu": int(c.groups_per_cu)}
               for c in list(plan.classes)[:int(plan.n_classes)]]
        print(json.dumps({
            "metric": "decompressed MB/s (whole node), config 5: 32K mixed-props streams",
            "value": round(value, 2), "unit": "MB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic text, liblzma-encoded (lc 0-4, lp 0-2, pb 0-4, dict 4K-1M)",
            "config": {"workload": f"{count} streams, log-uniform 1 KiB-256 KiB, mixed props, "
                                   "half FINISH_END / half FINISH_ANY",
                       "decompressed_bytes_per_gpu": total_out,
                       "compressed_bytes_per_gpu": int(lens.sum()),
                       "kernel_plan": {"lds_streams": int(plan.n_lds), "classes": cls}},
            "roofline": {"bound": "issue", "priced_against": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6),
                         "traffic": pmc_traffic("cfg5"), "traffic_source": "profiles/pmc_cfg5.json",
                         "binary": lib_sha256(), "kernel": plan_kernels(plan),
                         "kernel_avg_ms": round(dec_ms, 4), "alg_bytes_per_launch": alg},
            "sliced": sliced, "cpu_baseline": cpu, "verified": ok}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


def cpu_baseline_mixed(comp, lens, offs, nout, props, fin, threads, m):
    """The oracle restatement over the first m streams of a mixed batch."""
    import native
    orc = native.oracle()
    src_off = np.ascontiguousarray(offs[:m], dtype=np.uint64)
    src_len = np.ascontiguousarray(lens[:m], dtype=np.uint64)
    dst_cap = np.ascontiguousarray(nout[:m], dtype=np.uint64)
    dst_off = np.zeros(m, dtype=np.uint64)
    dst_off[1:] = np.cumsum(dst_cap)[:-1]
    dst = np.zeros(int(dst_cap.sum()) + 1, dtype=np.uint8)
    res = np.zeros(m, np.int32)
    st = np.zeros(m, np.int32)
    dl = np.zeros(m, np.uint64)
    sl = np.zeros(m, np.uint64)
    errs = 0
    t0 = time.perf_counter()
    for f in (0, 1):  # the oracle batch helper takes one finish mode per call
        sel = np.nonzero(fin[:m] == f)[0]
        if len(sel) == 0:
            continue
        # keep every argument array referenced until the call returns
        so, sn, do, dc = (np.ascontiguousarray(x[sel]) for x in (src_off, src_len, dst_off,
                                                                 dst_cap))
        pp = np.ascontiguousarray(props[:m][sel]).reshape(-1)
        errs += orc.orc_lzma_decode_batch(
            comp.ctypes.data, so.ctypes.data, sn.ctypes.data, pp.ctypes.data, dst.ctypes.data,
            do.ctypes.data, dc.ctypes.data, f, res.ctypes.data, st.ctypes.data,
            dl.ctypes.data, sl.ctypes.data, len(sel), threads)
    dt = time.perf_counter() - t0
    return float(dst_cap.sum()) / dt / 1e6, dt, m, errs


def cfg4_cpu_baseline(parts, threads):
    """LZMA2 decode of distinct blocks on host threads: the reference's own
    Lzma2Dec_DecodeToDic (oracle/_ref, compiled in place; threads in C, stdout
    silenced once for the batch) when present, else the oracle restatement on a
    thread pool (ctypes drops the GIL); plus a one-thread figure."""
    import native
    from concurrent.futures import ThreadPoolExecutor
    kind = "reference" if native.have_ref() else "port"
    sample = parts[:min(len(parts), 16 * threads)]

    def run(blocks, thr):
        if kind == "reference":
            lib = native.ref()
            m = len(blocks)
            src = np.frombuffer(b"".join(blocks), dtype=np.uint8)
            lens = np.array([len(c) for c in blocks], dtype=np.uint64)
            offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
            dst_off = np.arange(m, dtype=np.uint64) * CFG4_BLOCK
            cap = np.full(m, CFG4_BLOCK, dtype=np.uint64)
            dst = np.ones(m * CFG4_BLOCK, dtype=np.uint8)  # pages touched before the clock
            res = np.zeros(m, dtype=np.int32)
            dl = np.zeros(m, dtype=np.uint64)
            t0 = time.perf_counter()
            lib.ref_lzma2_decode_batch(src.ctypes.data, offs.ctypes.data, lens.ctypes.data,
                                       CFG4_PROP, dst.ctypes.data, dst_off.ctypes.data,
                                       cap.ctypes.data, 0, res.ctypes.data, dl.ctypes.data, m, thr)
            dt = time.perf_counter() - t0
            return dt, int(((res != 0) | (dl != CFG4_BLOCK)).sum())
        orc = native.oracle()

        def one(c):
            r = native.lzma2_decode(orc, "orc", c, CFG4_PROP, CFG4_BLOCK, 0)
            return r[0] == 0 and r[2] == CFG4_BLOCK

        t0 = time.perf_counter()
        with ThreadPoolExecutor(thr) as ex:
            oks = list(ex.map(one, blocks))
        return time.perf_counter() - t0, int(len(oks) - sum(oks))

    dt, errs = run(sample, threads)
    dt1, _ = run(sample[:8], 1)
    return {"value": round(len(sample) * CFG4_BLOCK / dt / 1e6, 2), "unit": "MB/s",
            "cores": threads, "kind": kind,
            "impl": "oracle/_ref/libref_lzma.so: the reference's Lzma2Dec.c + LzmaDec.c compiled in "
                    "place" if kind == "reference" else "oracle/lzma_oracle.c restatement",
            "sample": f"{len(sample)} distinct 1 MiB blocks, {threads} threads, {dt:.2f}s; "
                      f"1-core: 8 blocks in {dt1:.2f}s",
            "one_core_MBps": round(8 * CFG4_BLOCK / dt1 / 1e6, 2), "errors": errs}


def cpu_baseline(comp, lens, offs, n, props, threads, sample_streams, impl="port"):
    """A CPU LzmaDecode over a bounded sample: impl "reference" = the reference's
    own LzmaDec.c (oracle/_ref/libref_lzma.so, compiled in place with gcc -O2),
    "port" = the oracle restatement (oracle/liboracle.so)."""
    import native
    m = min(sample_streams, len(lens))
    if impl == "reference":
        ref = native.ref()
        src_off = np.ascontiguousarray(offs[:m], dtype=np.uint64)
        src_len = np.ascontiguousarray(lens[:m], dtype=np.uint64)
        dst_off = np.arange(m, dtype=np.uint64) * n
        dst_cap = np.full(m, n, dtype=np.uint64)
        p5 = np.tile(np.frombuffer(props, dtype=np.uint8), m)
        dst = np.ones(m * n, dtype=np.uint8)  # pages touched before the clock
        res = np.zeros(m, dtype=np.int32)
        dl = np.zeros(m, dtype=np.uint64)
        t0 = time.perf_counter()
        errs = ref.ref_lzma_decode_batch(comp.ctypes.data, src_off.ctypes.data, src_len.ctypes.data,
                                         p5.ctypes.data, dst.ctypes.data, dst_off.ctypes.data,
                                         dst_cap.ctypes.data, 1, res.ctypes.data, dl.ctypes.data,
                                         m, threads)
        dt = time.perf_counter() - t0
        errs += int((dl != n).sum())
        return m * n / dt / 1e6, dt, m, errs
    orc = native.oracle()
    src_off = np.ascontiguousarray(offs[:m], dtype=np.uint64)
    src_len = np.ascontiguousarray(lens[:m], dtype=np.uint64)
    dst_off = np.arange(m, dtype=np.uint64) * n
    dst_cap = np.full(m, n, dtype=np.uint64)
    p5 = np.tile(np.frombuffer(props, dtype=np.uint8), m)
    dst = np.zeros(m * n, dtype=np.uint8)
    res = np.zeros(m, dtype=np.int32)
    t0 = time.perf_counter()
    errs = orc.orc_lzma_decode_batch(comp.ctypes.data, src_off.ctypes.data, src_len.ctypes.data,
                                     p5.ctypes.data, dst.ctypes.data, dst_off.ctypes.data,
                                     dst_cap.ctypes.data, 1, res.ctypes.data, None, None, None,
                                     m, threads)
    dt = time.perf_counter() - t0
    return m * n / dt / 1e6, dt, m, errs


# --config xz: one xz file per GPU of XZ_BLOCKS blocks of
# XZ_BLOCK bytes, filter chain [x86 BCJ, LZMA2], CRC-64 checks.  Timed per step on the
# device: the LZMA2 batch over all blocks, the BCJ kernel, the CRC-64 kernels.
XZ_BLOCK = 256 * 1024
XZ_UNIQUE = 64


def _xz_unique_block(i):
    import native
    import xzwrite
    data = native.gen("text", 60000 + i, XZ_BLOCK)
    blk, unpadded, n = xzwrite.make_block(data, 4, dict_size=XZ_BLOCK, x86=0)
    return i, blk, unpadded, n


def build_xz_file(workers, nblocks):
    """The xz file: XZ_UNIQUE encoded blocks repeated to nblocks (encoding time)."""
    import struct
    import zlib
    import xzwrite
    tmp = os.environ.get("TMPDIR", "/tmp")
    path = os.path.join(tmp, f"lzgpu_xz_u{XZ_UNIQUE}_b{XZ_BLOCK}_v1.npz")
    if os.path.exists(path):
        z = np.load(path)
        blob, meta = z["blob"].tobytes(), z["meta"]
        parts, o = [], 0
        for ln, unp, n in meta:
            parts.append((blob[o:o + int(ln)], int(unp), int(n)))
            o += int(ln)
    else:
        t0 = time.time()
        parts = [None] * XZ_UNIQUE
        for i, blk, unp, n in pool_map(_xz_unique_block, range(XZ_UNIQUE), workers):
            parts[i] = (blk, unp, n)
        np.savez(path, blob=np.frombuffer(b"".join(p[0] for p in parts), dtype=np.uint8),
                 meta=np.array([(len(p[0]), p[1], p[2]) for p in parts], dtype=np.uint64))
        log(f"[xz] encoded {XZ_UNIQUE} blocks in {time.time() - t0:.1f}s")
    flags = bytes([0, 4])
    out = [b"\xfd7zXZ\0" + flags + struct.pack("<I", zlib.crc32(flags))]
    recs = []
    for b in range(nblocks):
        blk, unp, n = parts[b % XZ_UNIQUE]
        out.append(blk)
        recs.append((unp, n))
    idx = b"\0" + xzwrite.varint(len(recs)) + b"".join(xzwrite.varint(u) + xzwrite.varint(n)
                                                       for u, n in recs)
    idx += b"\0" * ((-len(idx)) % 4)
    idx += struct.pack("<I", zlib.crc32(idx))
    back = struct.pack("<I", len(idx) // 4 - 1) + flags
    out += [idx, struct.pack("<I", zlib.crc32(back)) + back + b"YZ"]
    return b"".join(out)


def run_xz(args):
    import dist_bench as D
    world, rank, local_rank = D.world_info()
    cpus = cpu_info()["usable"]
    workers = max(1, min(16, cpus // max(1, world)))
    nblocks = args.blocks
    xz = build_xz_file(workers, nblocks)  # before the GPU is touched (fork pool)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    import lzmagpu as L
    r, blocks, total = L.xz_index(xz)
    assert r == 0 and len(blocks) == nblocks, r
    n = nblocks
    items = [dict(src_off=b.data_off, src_len=b.pack_size, dst_off=b.dst_off,
                  dst_cap=b.unpack_size, props=bytes([b.lzma2_prop]), finish=1,
                  kind=L.KIND_LZMA2) for b in blocks]
    descs = L.make_descs(items)
    plan, order = L.plan_ex(descs)
    offs = [b.dst_off for b in blocks]
    lens = [b.unpack_size for b in blocks]
    base, rng, nch = L.crc_plan(lens)

    def dev_bytes(b):
        return torch.frombuffer(bytearray(bytes(b)), dtype=torch.uint8).to(dev)

    d_src = dev_bytes(xz)
    d_dst = torch.empty(total + 16, dtype=torch.uint8, device=dev)
    d_ws = torch.empty(max(int(plan.workspace_bytes), 16), dtype=torch.uint8, device=dev)
    d_desc, d_order = dev_bytes(descs), dev_bytes(order)
    d_res = torch.empty(n * 24, dtype=torch.uint8, device=dev)
    d_off = torch.tensor(offs, dtype=torch.int64, device=dev)
    d_len = torch.tensor(lens, dtype=torch.int64, device=dev)
    d_ip = torch.tensor([b.x86_ip for b in blocks], dtype=torch.int32, device=dev)
    d_state = torch.zeros(n, dtype=torch.int32, device=dev)
    d_done = torch.zeros(n, dtype=torch.int64, device=dev)
    d_base, d_rng = dev_bytes(base), dev_bytes(rng)
    d_chunks = torch.empty(max(nch, 1), dtype=torch.int64, device=dev)
    d_crc = torch.empty(n, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream

    def step(ev=None, res=None):
        res = d_res if res is None else res
        if ev:
            ev[0].record(stream)
        if L.decode_batch_device_ex(plan, d_desc.data_ptr(), d_order.data_ptr(), d_src.data_ptr(),
                                    d_dst.data_ptr(), d_ws.data_ptr(), res.data_ptr(), sh):
            raise RuntimeError(L.last_error())
        if ev:
            ev[1].record(stream)
        d_state.zero_()
        if L.bcj_x86_batch_device(d_dst.data_ptr(), d_off.data_ptr(), d_len.data_ptr(),
                                  d_ip.data_ptr(), d_state.data_ptr(), d_done.data_ptr(), n, 0, sh):
            raise RuntimeError(L.last_error())
        if ev:
            ev[2].record(stream)
        if L.crc64_batch_device(d_dst.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n,
                                d_base.data_ptr(), d_rng.data_ptr(), nch, 2**64 - 1, 2**64 - 1,
                                d_chunks.data_ptr(), d_crc.data_ptr(), sh):
            raise RuntimeError(L.last_error())
        if ev:
            ev[3].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    d_res_steps = timed_buffers(torch, dev, d_dst, n, args.steps)
    d_crc.fill_(-1)
    D.barrier()
    torch.cuda.synchronize()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(evs[i], d_res_steps[i])
    torch.cuda.synchronize()
    D.barrier()
    torch.cuda.synchronize()
    elapsed = D.reduce_max(time.perf_counter() - t0, dev)
    ms = [float(np.mean([e[k].elapsed_time(e[k + 1]) for e in evs])) for k in range(3)]
    # verify every timed launch: each step's block results, and the CRC-64 of
    # every block of the poisoned-then-decoded output equals the stored check
    allres = step_results(d_res_steps)
    crc = d_crc.cpu().numpy().astype(np.uint64)
    want = np.array([int.from_bytes(xz[b.check_off:b.check_off + 8], "little") for b in blocks],
                    dtype=np.uint64)
    ok = bool((allres["res"] == 0).all() and (allres["status"] == 1).all() and
              (allres["dest_len"] == np.array(lens)[None, :]).all() and (crc == want).all())
    ok = D.all_true(ok, dev)
    comp_bytes = len(xz)
    value = total * world * args.steps / elapsed / 1e6
    alg_dec = comp_bytes + total  # read the file once, write the output once
    dec_gbps = alg_dec / (ms[0] * 1e-3) / 1e9
    if rank == 0:
        line = {
            "metric": "decompressed MB/s (whole node), xz multi-block file ([x86 BCJ, LZMA2], CRC-64)",
            "value": round(value, 2), "unit": "MB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic text, liblzma-encoded blocks written into one xz stream per GPU",
            "config": {"workload": f"{n} blocks x {XZ_BLOCK} B, x86 BCJ + LZMA2 "
                                   f"(dict {XZ_BLOCK}), CRC-64 (SURVEY 8(f) rows 3-4)",
                       "file_bytes": comp_bytes, "unpack_bytes": total,
                       "kernel_ms": {"lzma2_batch": round(ms[0], 4), "bcj_x86": round(ms[1], 4),
                                     "crc64": round(ms[2], 4)},
                       "parallelism": f"{world} rank(s), one xz file each, no collective"},
            "roofline": {"bound": "issue", "priced_against": "hbm", "kernel": f"{plan_kernels(plan)} (LZMA2 items)",
                         "achieved": round(dec_gbps, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(dec_gbps / HBM_PEAK_GBS, 6), "traffic": None,
                         "alg_bytes_per_launch": alg_dec},
            "bcj_x86": {"GBps": round(2 * total / (ms[1] * 1e-3) / 1e9, 2),
                        "alg_bytes_per_launch": 2 * total},
            "crc64": {"GBps": round(total / (ms[2] * 1e-3) / 1e9, 2),
                      "frac": round(total / (ms[2] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
            "verified": ok,
        }
        print(json.dumps(line), flush=True)
    return 0 if ok else 1


# --config 7z: one 7z archive per GPU of SZ_FOLDERS folders of
# SZ_FILES files x SZ_FILE bytes (LZMA lc3/lp0/pb2, 64 KiB dict: config 2's stream
# shape), an LZMA-packed header, a CRC-32 per file.  Timed per step on the device:
# the LZMA batch over all folders, the CRC-32 batch over all files.
SZ_FILE = 16 * 1024
SZ_FILES = 4
SZ_UNIQUE = 64


def build_7z_archive(nfolders):
    import lzma
    import native
    import sevenzwrite as W
    folders = []
    uniq = []
    for i in range(SZ_UNIQUE):
        files = [(f"u{i}/f{k}.txt", native.gen("text", 61000 + SZ_FILES * i + k, SZ_FILE))
                 for k in range(SZ_FILES)]
        uniq.append(W.Folder(files, method=W.M_LZMA, dict_size=1 << 16))
    for i in range(nfolders):
        u = uniq[i % SZ_UNIQUE]
        files = [(f"d{i}/" + n.split("/")[1], b) for n, b in u.files]
        folders.append(W.Folder(files, packed=u.packed, props=u.props))
    return W.archive(folders, encode_header=True)


def run_7z(args):
    import dist_bench as D
    world, rank, local_rank = D.world_info()
    nfolders = args.blocks if args.blocks != 1024 else 4096
    arc = build_7z_archive(nfolders)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    import lzmagpu as L
    t0 = time.perf_counter()
    r, folders, files, _, total = L.sz_open(arc)  # the packed header decodes on the GPU
    open_ms = (time.perf_counter() - t0) * 1e3
    assert r == 0 and len(folders) == nfolders, r
    n, nf = len(folders), len(files)
    items = [dict(src_off=f.pack_off, src_len=f.pack_size, dst_off=f.dst_off,
                  dst_cap=f.unpack_size, props=bytes(f.props[:5]), finish=1,
                  kind=L.KIND_LZMA) for f in folders]
    descs = L.make_descs(items)
    plan, order = L.plan_ex(descs)
    offs = [f.dst_off for f in files]
    lens = [f.size for f in files]
    base, rng, nch = L.crc_plan(lens)

    def dev_bytes(b):
        return torch.frombuffer(bytearray(bytes(b)), dtype=torch.uint8).to(dev)

    d_src = dev_bytes(arc)
    d_dst = torch.empty(total + 16, dtype=torch.uint8, device=dev)
    d_ws = torch.empty(max(int(plan.workspace_bytes), 16), dtype=torch.uint8, device=dev)
    d_desc, d_order = dev_bytes(descs), dev_bytes(order)
    d_res = torch.empty(n * 24, dtype=torch.uint8, device=dev)
    d_off = torch.tensor(offs, dtype=torch.int64, device=dev)
    d_len = torch.tensor(lens, dtype=torch.int64, device=dev)
    d_base, d_rng = dev_bytes(base), dev_bytes(rng)
    d_chunks = torch.empty(max(nch, 1), dtype=torch.int32, device=dev)
    d_crc = torch.empty(nf, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream

    def step(ev=None, res=None):
        res = d_res if res is None else res
        if ev:
            ev[0].record(stream)
        if L.decode_batch_device_ex(plan, d_desc.data_ptr(), d_order.data_ptr(), d_src.data_ptr(),
                                    d_dst.data_ptr(), d_ws.data_ptr(), res.data_ptr(), sh):
            raise RuntimeError(L.last_error())
        if ev:
            ev[1].record(stream)
        if L.crc_batch_device(d_dst.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), nf,
                              d_base.data_ptr(), d_rng.data_ptr(), nch, 0xFFFFFFFF, 0xFFFFFFFF,
                              d_chunks.data_ptr(), d_crc.data_ptr(), sh):
            raise RuntimeError(L.last_error())
        if ev:
            ev[2].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    d_res_steps = timed_buffers(torch, dev, d_dst, n, args.steps)
    d_crc.fill_(-1)
    D.barrier()
    torch.cuda.synchronize()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(evs[i], d_res_steps[i])
    torch.cuda.synchronize()
    D.barrier()
    torch.cuda.synchronize()
    elapsed = D.reduce_max(time.perf_counter() - t0, dev)
    ms = [float(np.mean([e[k].elapsed_time(e[k + 1]) for e in evs])) for k in range(2)]
    allres = step_results(d_res_steps)
    crc = d_crc.cpu().numpy().astype(np.uint32)
    want = np.array([f.crc for f in files], dtype=np.uint32)
    ok = bool((allres["res"] == 0).all()
              and (allres["dest_len"] == np.array([f.unpack_size for f in folders])[None, :]).all()
              and (allres["src_len"] == np.array([f.pack_size for f in folders])[None, :]).all()
              and (crc == want).all())
    # the C-ABI call end to end once (host buffers: upload, open, decode, CRCs, download)
    t0 = time.perf_counter()
    r2, out, fres = L.SzExtract(arc, total, max_files=nf)
    api_ms = (time.perf_counter() - t0) * 1e3
    ok = ok and r2 == 0 and not any(fres[:nf])
    ok = D.all_true(ok, dev)
    comp_bytes = len(arc)
    value = total * world * args.steps / elapsed / 1e6
    alg_dec = sum(f.pack_size for f in folders) + total
    dec_gbps = alg_dec / (ms[0] * 1e-3) / 1e9
    if rank == 0:
        line = {
            "metric": "decompressed MB/s (whole node), 7z archive (LZMA folders, CRC-32 per file)",
            "value": round(value, 2), "unit": "MB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic text, liblzma-encoded folders written into one 7z archive per GPU",
            "config": {"workload": f"{n} folders x {SZ_FILES} files x {SZ_FILE} B, LZMA lc3/lp0/pb2 "
                                   "dict 64 KiB, packed header, CRC-32 per file (SURVEY 8(f) row 3)",
                       "archive_bytes": comp_bytes, "unpack_bytes": total,
                       "kernel_ms": {"lzma_batch": round(ms[0], 4), "crc32_files": round(ms[1], 4)},
                       "open_ms_host": round(open_ms, 3),
                       "extract_api_ms_pcie_inclusive": round(api_ms, 3),
                       "parallelism": f"{world} rank(s), one archive each, no collective"},
            "roofline": {"bound": "issue", "priced_against": "hbm", "kernel": f"{plan_kernels(plan)} (7z LZMA folders)",
                         "achieved": round(dec_gbps, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(dec_gbps / HBM_PEAK_GBS, 6), "traffic": None,
                         "alg_bytes_per_launch": alg_dec},
            "crc32": {"GBps": round(total / (ms[1] * 1e-3) / 1e9, 2),
                      "frac": round(total / (ms[1] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
            "verified": ok,
        }
        print(json.dumps(line), flush=True)
    return 0 if ok else 1


def measure_e2e(L, torch, plan, d_desc, d_order, d_src, d_dst, d_ws, d_res, comp, count, n,
                stream, steps):
    """End to end over PCIe: H2D of the compressed batch from pinned host memory,
    the decode, D2H of the output into pinned host memory -- per step, on the
    launch stream (HIP events).  Not `value`: the headline is device-resident."""
    h_src = torch.from_numpy(np.ascontiguousarray(comp)).pin_memory()
    h_dst = torch.empty(count * n, dtype=torch.uint8).pin_memory()
    sh = stream.cuda_stream
    nb = int(h_src.numel())
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for e in ev:
        e[0].record(stream)
        d_src[:nb].copy_(h_src, non_blocking=True)
        e[1].record(stream)
        if L.decode_batch_device_ex(plan, d_desc.data_ptr(), d_order.data_ptr(), d_src.data_ptr(),
                                    d_dst.data_ptr(), d_ws.data_ptr(), d_res.data_ptr(), sh):
            raise RuntimeError(L.last_error())
        e[2].record(stream)
        h_dst.copy_(d_dst[:count * n], non_blocking=True)
        e[3].record(stream)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    ms = [float(np.mean([e[k].elapsed_time(e[k + 1]) for e in ev])) for k in range(3)]
    return {"value": round(count * n / wall / 1e6, 2), "unit": "MB/s",
            "h2d_ms": round(ms[0], 4), "decode_ms": round(ms[1], 4), "d2h_ms": round(ms[2], 4),
            "ms_per_step": round(wall * 1e3, 4), "steps": steps,
            "h2d_GBps": round(nb / (ms[0] * 1e-3) / 1e9, 2),
            "d2h_GBps": round(count * n / (ms[2] * 1e-3) / 1e9, 2),
            "note": "pinned host buffers, copies and decode serialised on one stream"}


def measure_e2e_pipelined(L, torch, plan, d_desc, d_order, d_ws, d_res, comp, plain, count, n,
                          dev, batches):
    """Serving shape: a stream of batches from pinned host memory, each batch
    H2D -> decode -> D2H, two device buffer sets, the copies on one copy stream
    and the decode on another.  Enqueue order per step is H2D(b+1), decode(b),
    D2H(b): the next batch's upload is queued ahead of this batch's download,
    so it runs while batch b decodes instead of waiting behind a download that
    waits for that decode (the order H2D(b), decode(b), D2H(b) held every upload
    behind the previous download: 18-19 ms per batch,
    profiles/r02_e2e/overlap_timeline.log; look-ahead order
    profiles/r02_e2e/overlap_ahead.log).  `value` = batches x bytes / wall time
    including the pipeline's fill and drain; `steady_ms_per_batch` = decode
    starts of the last and the second batch apart, over the batches between."""
    nb = int(comp.size)
    h_src = torch.from_numpy(np.array(comp)).pin_memory()
    h_dst = [torch.empty(count * n, dtype=torch.uint8).pin_memory() for _ in range(2)]
    d_src = [torch.empty(nb + 64, dtype=torch.uint8, device=dev) for _ in range(2)]
    d_dst = [torch.empty(count * n + 64, dtype=torch.uint8, device=dev) for _ in range(2)]
    s_copy, s_dec = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    h2d_done = [torch.cuda.Event() for _ in range(2)]
    dec_done = [torch.cuda.Event() for _ in range(2)]
    d2h_done = [torch.cuda.Event() for _ in range(2)]
    dec_start = [torch.cuda.Event(enable_timing=True) for _ in range(batches)]
    for e in dec_done + d2h_done:
        e.record(torch.cuda.current_stream(dev))
    torch.cuda.synchronize()

    def upload(b):
        k = b % 2
        s_copy.wait_event(dec_done[k])         # d_src[k] free (batch b-2 decoded)
        with torch.cuda.stream(s_copy):
            d_src[k][:nb].copy_(h_src, non_blocking=True)
        h2d_done[k].record(s_copy)

    t0 = time.perf_counter()
    upload(0)
    for b in range(batches):
        k = b % 2
        if b + 1 < batches:
            upload(b + 1)
        s_dec.wait_event(h2d_done[k])
        s_dec.wait_event(d2h_done[k])          # d_dst[k] free (batch b-2 copied out)
        dec_start[b].record(s_dec)
        if L.decode_batch_device_ex(plan, d_desc.data_ptr(), d_order.data_ptr(),
                                    d_src[k].data_ptr(), d_dst[k].data_ptr(), d_ws.data_ptr(),
                                    d_res.data_ptr(), s_dec.cuda_stream):
            raise RuntimeError(L.last_error())
        dec_done[k].record(s_dec)
        s_copy.wait_event(dec_done[k])
        with torch.cuda.stream(s_copy):
            h_dst[k].copy_(d_dst[k][:count * n], non_blocking=True)
        d2h_done[k].record(s_copy)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ok = all(bool(np.array_equal(h.numpy(), plain)) for h in h_dst)
    steady = dec_start[1].elapsed_time(dec_start[batches - 1]) / (batches - 2)
    return {"value": round(batches * count * n / wall / 1e6, 2), "unit": "MB/s",
            "batches": batches, "ms_per_batch": round(wall / batches * 1e3, 4),
            "steady_ms_per_batch": round(steady, 4),
            "steady_MBps": round(count * n / (steady * 1e-3) / 1e6, 2),
            "verified": ok,
            "note": "H2D(b+1) / decode(b) / D2H(b) from pinned host memory: one copy stream, "
                    "one decode stream, two device buffer sets; the copies of one batch "
                    "(H2D + D2H) hide under the next batch's decode"}


def measure_sliced(L, torch, descs, count, d_src, d_dst, dev, slice_bytes, steps, one_shot_ms,
                   check):
    """The same batch decoded time-sliced (LzmaGpu_DecodeBatchSliced): rounds of
    at most slice_bytes per stream, the decoder state spilled between rounds.
    Every step starts from a poisoned output and results array; its results
    must pass check(results) and its output equal the one-shot decode's
    (d_dst as the caller's verified timed steps left it, compared on the GPU)."""
    import ctypes
    sd = (L.StreamDesc * count)()
    ctypes.memmove(sd, descs, ctypes.sizeof(sd))
    plan, order = L.plan_sliced(sd, slice_bytes)
    ref = d_dst.clone()
    d_desc = torch.frombuffer(bytearray(bytes(sd)), dtype=torch.uint8).to(dev)
    d_order = torch.frombuffer(bytearray(bytes(order)[:4 * count]), dtype=torch.uint8).to(dev)
    d_ws = torch.empty(int(plan.workspace_bytes), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream

    def run(res):
        r = L.decode_batch_sliced_device(plan, d_desc.data_ptr(), d_order.data_ptr(),
                                         d_src.data_ptr(), d_dst.data_ptr(), d_ws.data_ptr(),
                                         res.data_ptr(), 0, 0, sh)
        if r != 0:
            raise RuntimeError("LzmaGpu_DecodeBatchSliced failed: " + L.last_error())

    warm = torch.empty(count * 24, dtype=torch.uint8, device=dev)
    run(warm)
    torch.cuda.synchronize()
    ms, ok = [], True
    for _ in range(steps):
        poison(torch, d_dst)
        res = torch.full((count * 24,), 0xFF, dtype=torch.uint8, device=dev)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record(stream)
        run(res)
        b.record(stream)
        torch.cuda.synchronize()
        ms.append(a.elapsed_time(b))
        ok = ok and check(np.frombuffer(res.cpu().numpy().tobytes(), dtype=RES_DT))
        ok = ok and bool(torch.equal(d_dst, ref))
    del ref
    avg = float(np.mean(ms))
    left = L.sliced_active(plan, d_ws.data_ptr(), plan.rounds, sh)
    kern = {1: "lzgpu_sliced_lane_kernel", 2: "lzgpu_sliced_coop_kernel",
            3: "lzgpu_sliced_global_kernel"}[plan.kernel]
    out_bytes = int(np.frombuffer(bytes(sd), dtype=np.uint8).reshape(count, 48)[:, 24:32]
                    .copy().view(np.uint64).sum())
    return {"slice_bytes": slice_bytes, "rounds": int(plan.rounds), "kernel": kern,
            "placement": hex(plan.lds_mask), "groups_per_cu": int(plan.groups_per_cu),
            "streams_in_place": int(plan.n_inplace), "ms": round(avg, 3),
            "MBps": round(out_bytes / (avg * 1e-3) / 1e6, 2),
            "vs_one_shot": round(one_shot_ms / avg, 3), "unfinished_after_last_round": int(left),
            "workspace_bytes": int(plan.workspace_bytes), "verified": ok and left == 0,
            "note": "the same streams in rounds of at most slice_bytes per stream, decoder "
                    "state spilled to device memory between rounds; no host round trip"}


def run_coalesce(args):
    """Concurrent single-stream callers: an UNCHANGED
    multi-threaded C caller of the reference's one-call API
    (tests/c_host/lzma_c_threads.c: THREADS pthreads, each LzmaDecode-ing its
    share of the config-3 stream set from host buffers) linked to this library
    -- whose coalescer turns the calls that arrive while a batch runs into the
    next batch launch -- and the same source linked to the reference's
    LzmaDec.c (oracle/_ref/lzma_c_threads_ref) on the same host cores.  1, 16
    and 256 callers; both builds' per-stream CRCs must agree.  Host buffers,
    PCIe-inclusive: never the headline `value` (this leg reports the 256-caller
    GPU rate as its own metric)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import tempfile
    import test_c_host as TC
    cpu = cpu_info()
    workers = max(1, min(16, cpu["usable"]))
    count = args.streams or 4096
    plain, comp, lens, props = build_workload("cfg3", 0, count, workers)
    n = CONFIGS["cfg3"][1]
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    comps = [comp[offs[i]:offs[i + 1]].tobytes() for i in range(count)]
    gpu_bin = TC.THREADS_BIN if os.path.exists(TC.THREADS_BIN) else TC.build_c_threads()
    ref_bin = TC.THREADS_REF
    rows = []
    with tempfile.TemporaryDirectory() as tmp:
        f = TC.write_stream_set(tmp, comps, [props] * count, [n] * count)
        # "one": LzmaDecode per stream; "buf": the fork's DecodeToBuf loop
        # (1 KiB in / 1 KiB out per call) on a decoder per thread
        for mode, threads in (("one", 1), ("one", 16), ("one", 256), ("buf", 16), ("buf", 256)):
            row = {"mode": mode, "threads": threads}
            for name, binary in (("gpu", gpu_bin), ("reference", ref_bin)):
                if not os.path.exists(binary):
                    row[name] = {"error": "not built"}
                    continue
                # size the run to ~1-4 s: a first pass of one repeat, then scale
                d = TC.run_c_threads(binary, threads, f, 1, timeout=600, mode=mode)
                rep = max(1, min(64, int(2.0 / max(d["seconds"], 1e-3))))
                if rep > 1:
                    d = TC.run_c_threads(binary, threads, f, rep, timeout=600, mode=mode)
                row[name] = d
                log(f"[coalesce] {name} {mode} threads={threads}: {d['MBps']} MB/s "
                    f"fails={d['fails']} batches={d.get('batches')} max={d.get('max_batch')}")
            g, r = row.get("gpu", {}), row.get("reference", {})
            row["crc_match"] = g.get("crc_xor") is not None and g.get("crc_xor") == r.get("crc_xor")
            if g.get("batches"):
                row["gpu_calls_per_launch"] = round(g["batched_calls"] / g["batches"], 2)
            rows.append(row)
    ok = all(r["crc_match"] and r["gpu"].get("fails") == 0 for r in rows)
    top = rows[2]["gpu"]  # LzmaDecode, 256 callers
    out = {"metric": "decompressed MB/s, concurrent LzmaDecode callers over host buffers "
                     "(drop-in, coalesced launches)",
           "value": top.get("MBps"), "unit": "MB/s", "n_gpus": 1, "higher_is_better": True,
           "verified": ok, "dtype": "u8", "data": "synthetic (config-3 streams)",
           "config": {"workload": f"{count} x {n} B streams (config 3 shape), 1/16/256 pthreads "
                                  "calling LzmaDecode (value: 256), and 16/256 running the "
                                  "DecodeToBuf loop",
                      "rows": rows, "cpu": cpu}}
    print(json.dumps(out))
    return 0 if ok else 1


def run_secondary(cfgs, steps=5, warmup=1, timeout=420):
    """The other BASELINE configs, each a short run of this script in a child
    process (started, not exec'd: this process has touched the GPU), so the
    default bench line also carries them.  Not `value`."""
    out = {}
    for c in cfgs:
        cmd = [sys.executable, os.path.abspath(__file__), "--config", c, "--steps", str(steps),
               "--warmup", str(warmup), "--no-cpu-baseline", "--no-e2e", "--no-crc",
               "--no-secondary"]
        if c == "cfg2":
            cmd += ["--sliced", "16384"]  # the time-sliced form of the same batch beside it
        t0 = time.perf_counter()
        try:
            r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                               timeout=timeout, env=os.environ.copy())
            lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            d = json.loads(lines[-1]) if lines else {}
        except (subprocess.TimeoutExpired, ValueError) as e:
            d, r = {"error": type(e).__name__}, None
        roof = d.get("roofline") or {}
        cfg_d = d.get("config") or {}
        out[c] = {"value": d.get("value"), "unit": d.get("unit"),
                  "ms_per_step": d.get("ms_per_step"),
                  "kernel_avg_ms": roof.get("kernel_avg_ms") or
                  (cfg_d.get("kernel_ms") or {}).get("lzma2_batch"),
                  "workload": cfg_d.get("workload"), "kernel_plan": cfg_d.get("kernel_plan"),
                  "verified": bool(d.get("verified")) and (r is not None and r.returncode == 0),
                  "sliced": d.get("sliced"),
                  "wall_s": round(time.perf_counter() - t0, 1)}
        log(f"[secondary] {c}: {out[c]['value']} MB/s verified={out[c]['verified']}")
    return out


ISSUE_PEAKS = os.path.join(ROOT, "profiles", "r05_issue", "issue_peaks.json")


def pmc_traffic(cfg):
    """L2<->fabric bytes per launch from the committed PMC summary of `cfg`."""
    try:
        return json.load(open(os.path.join(ROOT, "profiles", f"pmc_{cfg}.json"))).get(
            "hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def lib_sha256():
    """sha256 of the decode library this process loads (LZGPU_LIB or the
    in-tree build): the binary the bench line measured, to match against the
    profiles' binary.sha256."""
    import hashlib
    import lzmagpu as L
    try:
        return hashlib.sha256(open(L.LIB_PATH, "rb").read()).hexdigest()
    except OSError:
        return None


def issue_peaks():
    """Measured SIMD issue ceilings (scripts/ubench/simd_issue_ubench.hip, run
    on the box; summarized in profiles/r05_issue/issue_peaks.json): wave-
    instructions of any kind a SIMD sustains per cycle with W co-resident
    waves, timed over whole kernels (round 4 priced a SIMD
    at one VALU instruction per 4 cycles from per-wave s_memtime medians).
    Falls back to MI355X_MICROARCH.md's SIMD-32 figure, one wave64 VALU
    instruction per 2 cycles per SIMD."""
    try:
        return json.load(open(ISSUE_PEAKS))
    except (OSError, ValueError):
        return {"source": "MI355X_MICROARCH.md:53-54 (SIMD-32: one wave64 VALU per 2 cycles)",
                "valu_per_simd_cycle": 0.5, "simd_inst_per_cycle": {}, "wave_cycles_per_inst": 4.0}


def issue_roofline(cfg, kernel_ms, waves_per_simd=None):
    """Issue-side figures of the decode kernel from the committed rocprofv3 PMC
    summary for this config (profiles/pmc_<cfg>.json, written by
    scripts/pmc_summary.py from separate --pmc passes of this bench), priced
    against the measured SIMD issue ceilings (issue_peaks()): instructions of
    every kind issued per SIMD-cycle against the ceiling at the kernel's waves
    per SIMD, VALU instructions against the SIMD-32 VALU rate, lanes active per
    VALU instruction, and the shares of wave cycles issuing / parked on
    s_waitcnt / stalled for issue."""
    path = os.path.join(ROOT, "profiles", f"pmc_{cfg}.json")
    if not os.path.exists(path):
        return None
    try:
        p = json.load(open(path))
    except (OSError, ValueError):
        return None
    c = p.get("counters", {})
    pk = issue_peaks()
    out = {"source": os.path.relpath(path, ROOT), "binary": p.get("binary"),
           "peaks_source": pk.get("source")}
    clk = p.get("effective_clock_GHz") or 2.4
    simds = 256 * 4
    cyc = kernel_ms * 1e-3 * clk * 1e9  # shader cycles of one launch
    if "SQ_INSTS_VALU" in c:
        # SQ_INSTS_* are wave-instructions per launch (summed over XCD/SE instances)
        kinds = ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH",
                 "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SMEM")
        total = sum(c.get(k, 0.0) for k in kinds)
        per_simd = total / simds / cyc
        valu = c["SQ_INSTS_VALU"] / simds / cyc
        out.update({"valu_insts_per_launch": c["SQ_INSTS_VALU"],
                    "salu_insts_per_launch": c.get("SQ_INSTS_SALU"),
                    "insts_per_launch": total,
                    "insts_per_simd_cycle": round(per_simd, 4),
                    "valu_per_simd_cycle": round(valu, 4),
                    "valu_frac": round(valu / pk.get("valu_per_simd_cycle", 0.5), 4)})
        w = waves_per_simd
        ceil = (pk.get("simd_inst_per_cycle") or {}).get(str(w)) if w else None
        if ceil:
            out["issue_ceiling_per_simd_cycle"] = ceil
            out["issue_frac"] = round(per_simd / ceil, 4)
    if "SQ_THREAD_CYCLES_VALU" in c and "SQ_ACTIVE_INST_VALU" in c and c["SQ_ACTIVE_INST_VALU"]:
        out["lanes_active_per_valu"] = round(c["SQ_THREAD_CYCLES_VALU"] / c["SQ_ACTIVE_INST_VALU"], 2)
    if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
        # SQ_WAIT_ANY: wave-cycles parked on s_waitcnt (memory / LDS);
        # SQ_WAIT_INST_ANY: ready but not issued (arbitration, dependency)
        for k, name in (("SQ_WAIT_ANY", "wait_any_frac"), ("SQ_WAIT_INST_ANY", "wait_issue_frac"),
                        ("SQ_ACTIVE_INST_ANY", "issue_frac_of_wave_cycles")):
            if k in c:
                out[name] = round(c[k] / c["SQ_WAVE_CYCLES"], 4)
    for k in ("hbm_bytes_per_launch", "hbm_read_bytes_x2", "hbm_write_bytes", "kernel_avg_ns"):
        if k in p:
            out[k] = p[k]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak: a full batch per GPU; strong: one batch split over the GPUs")
    ap.add_argument("--config", default="cfg3",
                    choices=sorted(CONFIGS) + ["cfg1", "cfg4", "cfg5", "xz", "7z", "coalesce"])
    ap.add_argument("--streams", type=int, default=0,
                    help="streams per GPU: cfg5 (default 32768), or a share of cfg3 / cfg2's "
                         "batch (strong-scaling emulation on one GPU)")
    ap.add_argument("--blocks", type=int, default=1024, help="cfg4: LZMA2 blocks per GPU")
    ap.add_argument("--no-gather", action="store_true",
                    help="cfg4: skip the optional gather of decoded blocks on rank 0")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-crc", action="store_true", help="skip the CRC-32 (8(f) row 1) leg")
    ap.add_argument("--no-e2e", action="store_true", help="skip the H2D + decode + D2H leg")
    ap.add_argument("--sliced", type=int, default=0,
                    help="cfg2 / cfg3 / cfg5: also time the batch as a time-sliced decode "
                         "(LzmaGpu_DecodeBatchSliced) with this many output bytes per stream "
                         "and round (SURVEY 8(f) row 2)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher, sharding and reductions on CPU (gloo), no decode")
    ap.add_argument("--no-secondary", action="store_true",
                    help="config 3 at N = 1: skip the short runs of configs 2, 4 and 5 "
                         "reported under 'secondary'")
    args = ap.parse_args()
    if "RANK" not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus)  # spawns the ranks; touches no GPU here
    if args.dry_run:
        return run_dry(args)
    if args.config == "cfg1":
        return run_cfg1(args)
    if args.config == "cfg4":
        return run_cfg4(args)
    if args.config == "cfg5":
        return run_cfg5(args)
    if args.config == "xz":
        return run_xz(args)
    if args.config == "7z":
        return run_7z(args)
    if args.config == "coalesce":
        return run_coalesce(args)

    import dist_bench as D
    world, rank, local_rank = D.world_info()
    if world != args.gpus:
        log(f"[rank {rank}] note: --gpus {args.gpus} but WORLD_SIZE={world}; using {world}")
    cpu = cpu_info()
    workers = max(1, min(16, cpu["usable"] // max(1, world) if world > 1 else cpu["usable"]))

    count_cfg, n, lc, lp, pb, dsz, desc_txt = CONFIGS[args.config]
    if args.streams:
        # a per-GPU share of the config's batch on one GPU (strong-scaling
        # emulation: 65,536 / N streams of config 3, 4,096 / N of config 2)
        count_cfg = args.streams
        desc_txt = f"{count_cfg} of the {CONFIGS[args.config][0]} streams of " + desc_txt
    first, count = rank_streams(count_cfg, world, rank, args.scaling)
    # workload first: the compression pool forks before this process touches the GPU
    if args.streams and world == 1 and count <= CONFIGS[args.config][0]:
        # a share of the full batch: its first `count` streams (one cached encode
        # serves every share of the sweep)
        full = CONFIGS[args.config][0]
        plain, comp, lens, props = build_workload(args.config, 0, full, workers)
        plain = plain[:count * n]
        comp = comp[:int(lens[:count].sum())]
        lens = lens[:count]
    else:
        plain, comp, lens, props = build_workload(args.config, first, count, workers)

    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    import lzmagpu as L  # after torch: shares torch's HIP runtime
    descs, order, plan, offs = make_descs(lens, n, props)
    ws_bytes = int(plan.workspace_bytes)
    comp_bytes = int(lens.sum())
    dev = torch.device("cuda", local_rank)
    d_src = torch.from_numpy(np.concatenate([comp, np.zeros(16, np.uint8)])).to(dev)
    # LZGPU_SHADOW_BYTES: room behind the output for the attribution build's
    # repeated output stores (lzma_device.h LZGPU_SHADOW_OUT); 0 otherwise
    shadow = int(os.environ.get("LZGPU_SHADOW_BYTES", "0"))
    d_dst_full = torch.empty(count * n + shadow, dtype=torch.uint8, device=dev)
    d_dst = d_dst_full[:count * n]
    d_ws = torch.empty(max(ws_bytes, 16), dtype=torch.uint8, device=dev)
    d_desc = torch.frombuffer(bytearray(descs), dtype=torch.uint8).to(dev)
    d_order = torch.frombuffer(bytearray(order), dtype=torch.uint8).to(dev)
    d_res = torch.empty(count * 24, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream

    def step(res=None):
        res = d_res if res is None else res
        r = L.decode_batch_device_ex(plan, d_desc.data_ptr(), d_order.data_ptr(), d_src.data_ptr(),
                                     d_dst.data_ptr(), d_ws.data_ptr(), res.data_ptr(), sh)
        if r != 0:
            raise RuntimeError("LzmaGpu_DecodeBatch failed: " + L.last_error())

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    d_res_steps = timed_buffers(torch, dev, d_dst, count, args.steps)
    D.barrier()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        evs[i][0].record(stream)
        step(d_res_steps[i])
        evs[i][1].record(stream)
    torch.cuda.synchronize()
    D.barrier()
    torch.cuda.synchronize()
    elapsed_mine = time.perf_counter() - t0
    kern_ms = [a.elapsed_time(b) for a, b in evs]
    elapsed = D.reduce_max(elapsed_mine, dev)  # slowest rank sets the job time

    # ---- verify every timed launch (bit-exact vs plaintext + exact results)
    allres = step_results(d_res_steps)
    ok = bool((allres["res"] == 0).all() and (allres["status"] == 1).all() and
              (allres["dest_len"] == n).all() and (allres["src_len"] == lens[None, :]).all())
    out = d_dst.cpu().numpy()
    ok = ok and bool(np.array_equal(out, plain))
    ok = D.all_true(ok, dev)
    if not ok:
        log(f"[rank {rank}] VERIFY FAILED: res={np.unique(allres['res'])} "
            f"status={np.unique(allres['status'])}")
    d_res = d_res_steps[args.steps - 1]

    print_prof(L)
    crc = measure_crc(L, torch, descs, d_desc, d_res, d_dst, plain, count, n, stream, dev,
                      args.steps) if not args.no_crc else None
    if crc is not None:
        ok = D.all_true(ok and crc["verified"], dev)
    e2e = None
    if not args.no_e2e:
        e2e = measure_e2e(L, torch, plan, d_desc, d_order, d_src, d_dst, d_ws, d_res, comp, count,
                          n, stream, min(args.steps, 5))
        e2e["pipelined"] = measure_e2e_pipelined(L, torch, plan, d_desc, d_order, d_ws, d_res,
                                                 comp, plain, count, n, dev, 12)
        ok = D.all_true(ok and e2e["pipelined"]["verified"], dev)

    sliced = None
    if args.sliced:
        def check(rr):
            return bool((rr["res"] == 0).all() and (rr["status"] == 1).all() and
                        (rr["dest_len"] == n).all() and (rr["src_len"] == lens).all())
        sliced = measure_sliced(L, torch, descs, count, d_src, d_dst, dev, args.sliced,
                                min(args.steps, 5), float(np.mean(kern_ms)), check)
        ok = D.all_true(ok and sliced["verified"], dev)

    total_streams = int(D.reduce_sum(float(count), dev))
    total_bytes = total_streams * n * args.steps
    value = total_bytes / elapsed / 1e6
    avg_kern_ms = float(np.mean(kern_ms))
    alg_bytes = comp_bytes + 5 * count + count * n  # per launch
    achieved = alg_bytes / (avg_kern_ms * 1e-3) / 1e9
    ranks = gather_ranks({"rank": rank, "streams": count, "first_stream": first,
                          "kernel_avg_ms": round(avg_kern_ms, 4),
                          "elapsed_s": round(elapsed_mine, 5),
                          "MBps": round(count * n * args.steps / elapsed_mine / 1e6, 2),
                          "e2e_MBps": e2e["value"] if e2e else None})

    cpu_base = None
    if rank == 0 and not args.no_cpu_baseline:
        # rank 0 after the timed region at every world size (the
        # reference CPU path timed in the same run); the job's whole CPU quota
        import native
        thr = cpu["usable"]
        kind = "reference" if native.have_ref() else "port"
        v, dt, m, errs = cpu_baseline(comp, lens, offs, n, props, thr, count, kind)
        v1, dt1, m1, _ = cpu_baseline(comp, lens, offs, n, props, 1, max(64, count // 32), kind)
        impl = ("oracle/_ref/libref_lzma.so: the reference's own LzmaDec.c (LzmaDecode, "
                "LzmaDec.c:972) compiled in place with gcc -O2 by oracle/Makefile.ref"
                if kind == "reference" else
                "oracle/lzma_oracle.c: this build's C restatement of LzmaDec.c "
                "(pinned to the reference's outputs), not the reference binary")
        cpu_base = {"value": round(v, 2), "unit": "MB/s", "cores": thr, "kind": kind,
                    "impl": impl,
                    "sample": f"{m} streams ({m * n} B decompressed) of the same batch, "
                              f"{thr} threads, {dt:.2f}s; 1-core: {v1:.2f} MB/s over {m1} streams",
                    "one_core_MBps": round(v1, 2), "cpu": cpu, "errors": int(errs)}
        if kind == "reference":
            vp, dtp, mp_, _ = cpu_baseline(comp, lens, offs, n, props, thr, count, "port")
            cpu_base["port_MBps"] = round(vp, 2)

    # traffic and the issue figures from the same committed PMC summary
    # (profiles/pmc_<cfg>.json: scripts/profile.sh + scripts/pmc_summary.py on
    # the binary it names; `binary` below is the library this run loaded)
    issue = issue_roofline(args.config, avg_kern_ms, int(plan.waves_per_simd))
    traffic = issue.get("hbm_bytes_per_launch") if issue else None
    secondary = None
    if rank == 0 and world == 1 and args.config == "cfg3" and not args.no_secondary:
        # reported with their own `verified`; the headline's stands on config 3 alone
        secondary = run_secondary(("cfg1", "cfg2", "cfg4", "cfg5"))

    if rank == 0:
        line = {
            "metric": "decompressed MB/s (whole node), 64K-stream batch; bit-exact vs CPU LzmaDec",
            "value": round(value, 2), "unit": "MB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (C splitmix64 English-like text, liblzma-encoded)",
            "config": {"workload": desc_txt, "streams_per_gpu": count,
                       "streams_total": total_streams, "stream_bytes": n,
                       "props": props.hex(), "compressed_bytes_per_gpu": comp_bytes,
                       "ratio": round(comp_bytes / (count * n), 4),
                       "parallelism": f"{world} rank(s), streams sharded ({args.scaling} scaling), "
                                      "no data-path collective",
                       "world": dist.get_world_size() if dist.is_initialized() else 1,
                       "kernel_plan": {"lds_streams": int(plan.n_lds),
                                       "streams_per_workgroup": int(plan.lanes_per_group),
                                       "lds_bytes_per_stream": int(plan.lds_cells_per_lane) * 2,
                                       "workgroups_per_cu": int(plan.groups_per_cu),
                                       "waves_per_simd": int(plan.waves_per_simd),
                                       "placement": hex(plan.classes[0].lds_mask)
                                       if plan.n_classes else None}},
            "ranks": ranks,
            "roofline": {"bound": "issue", "priced_against": "hbm",
                         "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6),
                         "traffic": traffic,
                         "traffic_source": issue.get("source") if issue else None,
                         "binary": lib_sha256(),
                         "kernel": plan_kernels(plan),
                         "kernel_avg_ms": round(avg_kern_ms, 4),
                         "kernel_ms_steps": [round(x, 4) for x in kern_ms],
                         "alg_bytes_per_launch": alg_bytes,
                         "issue": issue,
                         "why": "each output byte needs ~5 serially dependent range-coder "
                                "decisions per stream: the kernel is bound by the latency of "
                                "that chain at 2 waves per SIMD (forced-wait attribution, "
                                "LZGPU_PROF=3: global-memory waits ~10 % of wave time), "
                                "not by HBM bytes"},
            "e2e": e2e,
            "sliced": sliced,
            "cpu_baseline": cpu_base,
            "crc32": crc,
            "secondary": secondary,
            "verified": ok,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


if __name__ == "__main__":
    sys.exit(main() or 0)

"""GPU parity per kernel instantiation and at every BASELINE config's full shape.

The planner picks a kernel by batch shape (LzmaGpu_PlanBatchEx): the
throughput placement 0x105 with 32 streams per wave for big narrow-table
batches (config 3), the latency placement 0x1BF with one stream per wave for
few streams per CU (configs 2 and 5), the wave-cooperative kernel at <= 8
streams per CU (config 4, xz), the generic kernel for tables too wide for LDS.
Small test batches would only ever reach the last two, so:

  * every golden vector (reference-decoded: KAT table, truncations, bit flips,
    capacities, both finish modes, 17 presets, LZMA2 ranges) and a 1,500-case
    seeded fuzz set (checked against the CPU restatement) run through EACH
    instantiation, forced per call with LzmaGpu_PlanBatchOpt;
  * configs 2, 3, 4 and 5 run at their full stream counts through the
    planner's own choice (asserted), checked by round trip to the plaintext
    and the per-stream result invariants.

Bit-exact throughout: output bytes and {res, status, destLen, srcLen}.
"""
import ctypes
import lzma
import os
import random
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import golden_cases as G
import native
import workloads as W

pytestmark = pytest.mark.gpu

COOP = 0x80000000
M_THR, M_LAT, M_ALL = 0x105, 0x1BF, 0x7FF
M_LAT_SG = 0x19F  # the latency placement with the slot trees global (kLdsMaskLatSlotG)
RES_DT = np.dtype([("res", "<i4"), ("status", "<i4"), ("dest_len", "<u8"), ("src_len", "<u8")])
# coop: the cooperative kernel, every table section in LDS where the table fits
# (placement 0x7FF); coop_lat: the same kernel on the latency placement 0x1BF
# (LZMA_GPU_PLAN_COOP_LAT)
# throughput_np: the throughput kernel without persistent lanes (one stream
# per lane, the grid covers the batch)
# throughput / throughput_np: the throughput kernel (global sections
# lane-interleaved in a slot area, the default) with and without persistent
# lanes; throughput_slices / throughput_slices_np: the same with per-stream
# global slices (LZMA_GPU_PLAN_NO_ILV, the round-2 layout)
ILV, PLAN_NO_ILV = 0x40000000, 16
# throughput_reuse: planned for one CU, so a persistent lane decodes several
# streams one after another in the same interleaved column (re-initialised per
# stream)
THR = ("throughput", "throughput_np", "throughput_slices", "throughput_slices_np",
       "throughput_reuse")
# (round 4's decision-level loop and scalar-register latency waves were
# measured slower and removed in round 5)
KERNELS = THR + ("latency", "coop", "coop_lat", "global")


@pytest.fixture(scope="module")
def L():
    import lzmagpu
    if lzmagpu.device_count() <= 0:
        pytest.fail("no HIP device visible: " + lzmagpu.last_error())
    return lzmagpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available()
    return t


def _check_plan(plan, kernel):
    """The forced instantiation is the one the plan launches."""
    cls = [plan.classes[k] for k in range(plan.n_classes)]
    if kernel == "global":
        assert plan.n_lds == 0 and plan.n_classes == 0
        return
    assert plan.n_lds > 0 and cls
    for c in cls:
        if kernel in THR:
            # interleaved rows for whole 32-lane groups, slices for narrower waves
            ilv = "slices" not in kernel and c.lanes_per_group in (32, 64)
            assert c.lds_mask == M_THR | (ILV if ilv else 0), (hex(c.lds_mask), c.lanes_per_group)
            if ilv:
                assert c.slot_cells > 0 and c.slot_groups > 0 and c.slot_off % 64 == 0
        elif kernel == "latency":
            # the slot trees go global where that fits more workgroups per CU
            assert c.lds_mask in (M_LAT, M_LAT_SG) and c.lanes_per_group == 1, hex(c.lds_mask)
        elif kernel == "coop":
            # all sections in LDS where the whole table fits the class's
            # streams per CU, else the latency placement
            assert c.lds_mask in (M_ALL | COOP, M_LAT | COOP) and c.lanes_per_group == 1, \
                hex(c.lds_mask)
        else:
            assert c.lds_mask == M_LAT | COOP, hex(c.lds_mask)
    if kernel == "coop":
        assert any(c.lds_mask == M_ALL | COOP for c in cls)
    if kernel in THR:
        # wave width follows table width: 32 streams per wave for lc+lp = 0
        # (config 3), 8 for lc+lp = 1, 2 for LZMA2 ranges (lc+lp <= 4 slices)
        assert all(c.lanes_per_group >= 2 for c in cls)
        if kernel == "throughput_np":
            # 32 lanes forced wherever the slices fit: interleaved rows for those
            assert any(c.lds_mask & ILV for c in cls)
        if kernel == "throughput_reuse":
            # fewer resident lanes than streams in every interleaved class
            ilv = [c for c in cls if c.lds_mask & ILV]
            assert ilv and any(c.n > c.slot_groups * c.lanes_per_group for c in ilv)
        assert plan.persistent == (0 if kernel.endswith("_np") else 1)


def _opts(L, kernel):
    # plan as if the batch were spread over a few CUs, so that the throughput
    # shape (>= 64 streams per CU) is what a real 64K batch gets
    if kernel == "coop_lat":
        return L.plan_options("coop", cus=8, flags=4)
    if kernel == "throughput_np":
        # 32 streams per wave wherever the slices fit: the interleaved rows
        # without persistent lanes on every batch, not only lc+lp = 0 classes
        return L.plan_options("throughput", cus=8, persistent=2, lanes_per_group=32)
    if kernel == "throughput_reuse":
        return L.plan_options("throughput", cus=1, groups_per_cu=1, lanes_per_group=32)
    if kernel == "throughput_slices":
        return L.plan_options("throughput", cus=8, flags=PLAN_NO_ILV)
    if kernel == "throughput_slices_np":
        return L.plan_options("throughput", cus=8, persistent=2, flags=PLAN_NO_ILV)
    return L.plan_options(kernel, cus=8)


# ---------------------------------------------------------------- goldens, every kernel

def _golden_batch():
    d = G.load()
    items, srcs, exp, off, doff = [], [], [], 0, 0
    for i, c in G.cases("lzma"):
        src = G.case_input(d, c)
        e = c["expect"]
        items.append(dict(src_off=off, src_len=len(src), dst_off=doff, dst_cap=c["dest_cap"],
                          props=bytes.fromhex(c["props"]), finish=c["finish"]))
        exp.append(((e["res"], e["status"], e["dest_len"], e["src_len"]), e["sha256"], c["note"]))
        srcs.append(src)
        off += len(src)
        doff += c["dest_cap"]
    for i, c in G.cases("lzma2"):
        src = G.case_input(d, c)
        e = c["expect"]
        # a batch LZMA2 item returns Lzma2Dec_DecodeToDic's own result over a flat
        # dictionary -- the 7zDec.c:181-202 pattern the golden vectors record
        items.append(dict(src_off=off, src_len=len(src), dst_off=doff, dst_cap=c["dest_cap"],
                          props=bytes([c["prop"]]), finish=c["finish"], kind=1))
        exp.append(((e["res"], e["status"], e["dest_len"], e["src_len"]), e["sha256"],
                    "lzma2 " + c["note"]))
        srcs.append(src)
        off += len(src)
        doff += c["dest_cap"]
    return items, b"".join(srcs), doff, exp


@pytest.mark.parametrize("kernel", KERNELS)
def test_goldens_through_each_kernel(L, kernel):
    items, src, dst_bytes, exp = _golden_batch()
    descs = L.make_descs(items)
    plan = L.Plan()
    r, res, dst = L.decode_batch_host(descs, src, dst_bytes, _opts(L, kernel), plan)
    assert r == 0, L.last_error()
    _check_plan(plan, kernel)
    if kernel in ("throughput", "throughput_slices"):
        # the lc0/lp0 goldens run the config-3 launch shape: 32 streams per wave
        assert max(plan.classes[k].lanes_per_group for k in range(plan.n_classes)) == 32
    bad = []
    for k, (want, sha, note) in enumerate(exp):
        got = (res[k].res, res[k].status, res[k].dest_len, res[k].src_len)
        out = dst[items[k]["dst_off"]:items[k]["dst_off"] + res[k].dest_len]
        if got != want or G.sha(out) != sha:
            bad.append((k, note, got, want))
    assert not bad, (kernel, len(bad), bad[:8])


# ---------------------------------------------------------------- the stream's last bytes

@pytest.mark.parametrize("kernel", KERNELS)
def test_tail_truncations_through_each_kernel(L, kernel):
    """The fast tail of one-shot decodes (lzma_device.h lz_decode_to_dic): the
    last < 20 input bytes in one bulk pass, checked afterwards against the
    reference's probe rule, a truncated end decoded again exactly.  Streams cut
    at every length in their last 26 bytes, with and without an end marker,
    exact / short / long capacities and both finish modes, against the oracle
    (LzmaDec.c:775-800: the probe decides where a truncated stream stops)."""
    import lzma
    orc = native.oracle()
    rng = random.Random(2605)
    items, srcs, exp, off, doff = [], [], [], 0, 0
    have_ref = os.path.exists(native.REF_SO)
    for it in range(12):
        n = rng.choice([300, 4096, 9000])
        data = native.gen(rng.choice(["text", "runs"]), 61_000 + it, n)
        if have_ref and it % 2:
            props, comp = native.ref_encode(data, level=5, dict_size=1 << 16, lc=3, lp=0, pb=2,
                                            end_mark=bool(it % 4 == 1))
        else:
            comp = lzma.compress(data, format=lzma.FORMAT_RAW, filters=[
                {"id": lzma.FILTER_LZMA1, "dict_size": 1 << 16, "lc": 3, "lp": 0, "pb": 2}])
            props = W.props_bytes(3, 0, 2, 1 << 16)
        for cut in range(0, 26):
            c = comp[:max(5, len(comp) - cut)]
            cap = n + rng.choice([0, 0, 7, -3])
            fin = rng.randrange(2)
            items.append(dict(src_off=off, src_len=len(c), dst_off=doff, dst_cap=cap, props=props,
                              finish=fin))
            srcs.append(c)
            exp.append(native.decode(orc, "orc", c, props, cap, fin))
            off += len(c)
            doff += cap
    descs = L.make_descs(items)
    plan = L.Plan()
    r, res, dst = L.decode_batch_host(descs, b"".join(srcs), doff, _opts(L, kernel), plan)
    assert r == 0, L.last_error()
    bad = []
    for k, e in enumerate(exp):
        got = (res[k].res, res[k].status, res[k].dest_len, res[k].src_len)
        out = dst[items[k]["dst_off"]:items[k]["dst_off"] + res[k].dest_len]
        if got != tuple(e[:4]) or out != e[4]:
            bad.append((k, got, e[:4]))
    assert not bad, (kernel, len(bad), bad[:6])


# ---------------------------------------------------------------- fuzz, every kernel

_FUZZ = {}


def _fuzz_set():
    """1,500 seeded cases: random presets, sizes, bit flips, truncations,
    capacities and finish modes, liblzma-encoded; expectations from the oracle
    (the CPU restatement, pinned to the reference's vectors)."""
    if "v" in _FUZZ:
        return _FUZZ["v"]
    # a bigger campaign: LZGPU_FUZZ_CASES / LZGPU_FUZZ_SEED (profiles/r02_tests/)
    cases = int(os.environ.get("LZGPU_FUZZ_CASES", "1500"))
    rng = random.Random(int(os.environ.get("LZGPU_FUZZ_SEED", "7331")))
    orc = native.oracle()
    items, srcs, exp, off, doff = [], [], [], 0, 0
    for it in range(cases):
        lc, lp, pb = rng.randrange(5), rng.randrange(3), rng.randrange(5)
        if lc + lp > 4:
            lp = 0
        dsz = rng.choice([4096, 1 << 14, 1 << 16])
        n = rng.choice([0, 1, 2, 60, 700, 4096, 9000, 20000])
        kind = rng.choice(["text", "text", "random", "runs"])
        data = native.gen(kind, 91_000 + it, n)
        filt = [{"id": lzma.FILTER_LZMA1, "dict_size": dsz, "lc": lc, "lp": lp, "pb": pb,
                 "preset": rng.choice([0, 6, 9])}]
        comp = bytearray(lzma.compress(data, format=lzma.FORMAT_RAW, filters=filt))
        props = W.props_bytes(lc, lp, pb, dsz)
        mode = rng.randrange(5)
        if mode == 1 and len(comp) > 6:
            for _ in range(rng.randrange(1, 4)):
                comp[rng.randrange(5, len(comp))] ^= 1 << rng.randrange(8)
        elif mode == 2:
            comp = comp[:rng.randrange(len(comp) + 1)]
        cap = max(0, n + rng.choice([0, 0, 0, 1, -1, 50, -50, -3000]))
        fin = rng.randrange(2)
        comp = bytes(comp)
        items.append(dict(src_off=off, src_len=len(comp), dst_off=doff, dst_cap=cap, props=props,
                          finish=fin))
        srcs.append(comp)
        exp.append(native.decode(orc, "orc", comp, props, cap, fin))
        off += len(comp)
        doff += cap
    _FUZZ["v"] = (items, b"".join(srcs), doff, exp)
    return _FUZZ["v"]


@pytest.mark.parametrize("kernel", KERNELS)
def test_fuzz_vs_oracle_each_kernel(L, kernel):
    items, src, dst_bytes, exp = _fuzz_set()
    descs = L.make_descs(items)
    plan = L.Plan()
    r, res, dst = L.decode_batch_host(descs, src, dst_bytes, _opts(L, kernel), plan)
    assert r == 0, L.last_error()
    _check_plan(plan, kernel)
    bad = []
    for k in range(len(items)):
        got = (res[k].res, res[k].status, res[k].dest_len, res[k].src_len)
        out = dst[items[k]["dst_off"]:items[k]["dst_off"] + res[k].dest_len]
        if got != exp[k][:4] or out != exp[k][4]:
            bad.append((k, got, exp[k][:4]))
    assert not bad, (kernel, len(bad), bad[:8])


# ---------------------------------------------------------------- LZMA2 fuzz, every kernel

_FUZZ2 = {}


def _fuzz2_set():
    """Seeded LZMA2 items (600 by default; LZGPU_FUZZ2_CASES / LZGPU_FUZZ2_SEED):
    random lc/lp/pb and dictionary props, 0-300 KB of text / random / runs (so
    several chunks, stored chunks for random data), with or without the end
    byte, bit flips, truncations, capacities, both finish modes and a few bad
    dictionary props; expectations from the oracle's Lzma2Dec_DecodeToDic
    restatement (the 7zDec.c:181-202 pattern the golden LZMA2 vectors pin)."""
    if "v" in _FUZZ2:
        return _FUZZ2["v"]
    cases = int(os.environ.get("LZGPU_FUZZ2_CASES", "600"))
    rng = random.Random(int(os.environ.get("LZGPU_FUZZ2_SEED", "2718")))
    orc = native.oracle()
    items, srcs, exp, off, doff = [], [], [], 0, 0
    for it in range(cases):
        lc = rng.randrange(5)
        lp = rng.randrange(5 - lc)
        pb = rng.randrange(5)
        prop = rng.choice([0, 8, 16, 18])        # dict 4 KiB, 64 KiB, 1 MiB, 2 MiB
        dsz = (2 | (prop & 1)) << (prop // 2 + 11)
        n = rng.choice([0, 1, 100, 5000, 70000, 140000, 300000])
        kind = rng.choice(["text", "text", "random", "runs"])
        data = native.gen(kind, 97_000 + it, n)
        filt = [{"id": lzma.FILTER_LZMA2, "dict_size": dsz, "lc": lc, "lp": lp, "pb": pb,
                 "preset": rng.choice([0, 6])}]
        comp = bytearray(lzma.compress(data, format=lzma.FORMAT_RAW, filters=filt))
        mode = rng.randrange(6)
        if mode == 1 and len(comp) > 8:
            for _ in range(rng.randrange(1, 4)):
                comp[rng.randrange(len(comp))] ^= 1 << rng.randrange(8)
        elif mode == 2:
            comp = comp[:rng.randrange(len(comp) + 1)]
        elif mode == 3 and comp:
            comp = comp[:-1]                      # no end byte
        if rng.random() < 0.02:
            prop = rng.choice([41, 60, 255])      # bad dictionary prop
        cap = max(0, n + rng.choice([0, 0, 0, 1, -1, 100, -100, -20000]))
        fin = rng.randrange(2)
        comp = bytes(comp)
        items.append(dict(src_off=off, src_len=len(comp), dst_off=doff, dst_cap=cap,
                          props=bytes([prop]), finish=fin, kind=1))
        srcs.append(comp)
        exp.append(native.lzma2_decode(orc, "orc", comp, prop, cap, fin))
        off += len(comp)
        doff += cap
    _FUZZ2["v"] = (items, b"".join(srcs), doff, exp)
    return _FUZZ2["v"]


@pytest.mark.parametrize("kernel", KERNELS)
def test_lzma2_fuzz_vs_oracle_each_kernel(L, kernel):
    items, src, dst_bytes, exp = _fuzz2_set()
    descs = L.make_descs(items)
    plan = L.Plan()
    r, res, dst = L.decode_batch_host(descs, src, dst_bytes, _opts(L, kernel), plan)
    assert r == 0, L.last_error()
    bad = []
    for k in range(len(items)):
        got = (res[k].res, res[k].status, res[k].dest_len, res[k].src_len)
        out = dst[items[k]["dst_off"]:items[k]["dst_off"] + res[k].dest_len]
        want = exp[k][:4]
        if got != want or out != exp[k][4]:
            bad.append((k, got, exp[k][:4]))
    assert not bad, (kernel, len(bad), bad[:8])


# ---------------------------------------------------------------- full-size configs

def _device_decode(L, torch, descs, comp, dst_bytes, opts=None):
    """LzmaGpu_PlanBatch{Ex,Opt} + LzmaGpu_DecodeBatchEx over device buffers
    (the bench's path).  Returns (plan, results, d_dst)."""
    plan, order = L.plan_ex(descs, opts)
    dev = torch.device("cuda", 0)
    n = len(descs)
    d_src = torch.from_numpy(np.concatenate([np.asarray(comp, np.uint8),
                                             np.zeros(16, np.uint8)])).to(dev)
    d_dst = torch.zeros(dst_bytes + 16, dtype=torch.uint8, device=dev)
    d_ws = torch.empty(max(int(plan.workspace_bytes), 16), dtype=torch.uint8, device=dev)
    d_desc = torch.frombuffer(bytearray(bytes(descs)), dtype=torch.uint8).to(dev)
    d_order = torch.frombuffer(bytearray(bytes(order)), dtype=torch.uint8).to(dev)
    d_res = torch.empty(n * 24, dtype=torch.uint8, device=dev)
    sh = torch.cuda.current_stream(dev).cuda_stream
    r = L.decode_batch_device_ex(plan, d_desc.data_ptr(), d_order.data_ptr(), d_src.data_ptr(),
                                 d_dst.data_ptr(), d_ws.data_ptr(), d_res.data_ptr(), sh)
    assert r == 0, L.last_error()
    torch.cuda.synchronize()
    res = np.frombuffer(d_res.cpu().numpy().tobytes(), dtype=RES_DT)
    return plan, res, d_dst


def _uniform_descs(L, lens, n, props, finish=1):
    count = len(lens)
    offs = np.zeros(count, dtype=np.uint64)
    offs[1:] = np.cumsum(lens)[:-1]
    return L.make_descs([dict(src_off=int(offs[i]), src_len=int(lens[i]), dst_off=i * n,
                              dst_cap=n, props=props, finish=finish) for i in range(count)])


def test_cfg3_full_64k_streams_throughput_kernel(L, torch):
    """BASELINE config 3 at full size: 65,536 x 4 KiB, lc0/lp0/pb0, 4 KiB dict --
    the headline batch, on the kernel that produces the headline number."""
    count, n = 65536, 4096
    plain, comp, lens, props = W.uniform_batch(count, n, 0, 0, 0, 4096)
    descs = _uniform_descs(L, lens, n, props)
    plan, res, d_dst = _device_decode(L, torch, descs, comp, count * n)
    assert plan.n_classes == 1 and plan.n_lds == count
    c = plan.classes[0]
    assert (c.lds_mask, c.lanes_per_group, c.groups_per_cu, c.waves_per_simd) == \
        (M_THR | ILV, 32, 8, 2)
    assert (res["res"] == 0).all() and (res["status"] == 1).all()
    assert (res["dest_len"] == n).all() and (res["src_len"] == lens).all()
    assert np.array_equal(d_dst[:count * n].cpu().numpy(), plain)


def test_cfg3_full_finish_any_and_short_caps(L, torch):
    """The same 64K batch with FINISH_ANY and every 7th stream's capacity cut
    short (NOT_FINISHED mid-stream, the DecodeReal2 limit path) on the 0x105
    kernel; a 1,024-stream sample is checked against the oracle."""
    count, n = 65536, 4096
    plain, comp, lens, props = W.uniform_batch(count, n, 0, 0, 0, 4096, first=1 << 20)
    offs = np.zeros(count, dtype=np.uint64)
    offs[1:] = np.cumsum(lens)[:-1]
    caps = [n - (i % 97) * 13 if i % 7 == 0 else n for i in range(count)]
    descs = L.make_descs([dict(src_off=int(offs[i]), src_len=int(lens[i]), dst_off=i * n,
                               dst_cap=caps[i], props=props, finish=0) for i in range(count)])
    plan, res, d_dst = _device_decode(L, torch, descs, comp, count * n)
    assert plan.classes[0].lds_mask == M_THR | ILV and plan.classes[0].lanes_per_group == 32
    out = d_dst[:count * n].cpu().numpy().reshape(count, n)
    rows = plain.reshape(count, n)
    caps = np.array(caps)
    assert (res["res"] == 0).all() and (res["dest_len"] == caps).all()
    full = caps == n
    # FINISH_ANY stops at the capacity, in front of the end mark: NOT_FINISHED
    assert (res["status"] == 2).all() and (res["src_len"] < lens).all()
    for i in np.nonzero(~full)[0][:64]:
        assert np.array_equal(out[i, :caps[i]], rows[i, :caps[i]])
    assert np.array_equal(out[full], rows[full])
    orc = native.oracle()
    comp_b = comp.tobytes()
    for i in range(0, count, 64):
        s = comp_b[int(offs[i]):int(offs[i]) + int(lens[i])]
        e = native.decode(orc, "orc", s, props, int(caps[i]), 0)
        assert (int(res["res"][i]), int(res["status"][i]), int(res["dest_len"][i]),
                int(res["src_len"][i])) == e[:4], i


def test_cfg2_full_4096_streams_latency_kernel(L, torch):
    """BASELINE config 2 at full size: 4,096 x 64 KiB, lc3/lp0/pb2, 64 KiB dict,
    on the latency kernel (one stream per wave, placement 0x1BF)."""
    count, n = 4096, 65536
    plain, comp, lens, props = W.uniform_batch(count, n, 3, 0, 2, 65536)
    descs = _uniform_descs(L, lens, n, props)
    plan, res, d_dst = _device_decode(L, torch, descs, comp, count * n)
    assert plan.n_classes == 1 and plan.n_lds == count
    c = plan.classes[0]
    assert (c.lds_mask, c.lanes_per_group, c.groups_per_cu) == (M_LAT, 1, 16)
    assert (res["res"] == 0).all() and (res["status"] == 1).all()
    assert (res["dest_len"] == n).all() and (res["src_len"] == lens).all()
    assert np.array_equal(d_dst[:count * n].cpu().numpy(), plain)


def test_cfg5_full_count_mixed_props(L, torch):
    """BASELINE config 5's stream count and props mix: 32,768 streams, lc 0-4,
    lp 0-2, pb 0-4, dict 4K-1M, half FINISH_END / half FINISH_ANY -- lengths
    log-uniform 1-16 KiB instead of 1-256 KiB so the encode fits a test; the
    planner sees the same width classes and streams per CU."""
    count = 32768
    with ThreadPoolExecutor(W.workers()) as ex:
        parts = list(ex.map(lambda i: W.cfg5_stream(i, max_log2=4), range(count)))
    nout = np.array([len(p[0]) for p in parts], dtype=np.uint64)
    lens = np.array([len(p[1]) for p in parts], dtype=np.uint64)
    fin = np.array([p[3] for p in parts])
    so = np.zeros(count, np.uint64)
    so[1:] = np.cumsum(lens)[:-1]
    do = np.zeros(count, np.uint64)
    do[1:] = np.cumsum(nout)[:-1]
    descs = L.make_descs([dict(src_off=int(so[i]), src_len=int(lens[i]), dst_off=int(do[i]),
                               dst_cap=int(nout[i]), props=parts[i][2], finish=int(fin[i]))
                          for i in range(count)])
    comp = np.frombuffer(b"".join(p[1] for p in parts), dtype=np.uint8)
    plain = b"".join(p[0] for p in parts)
    # the planner's default: the four width buckets all land in the one-lane
    # latency regime and are merged into one class (one launch; its widest
    # slice, 10,636 bytes = 9 of the CU's 128 LDS blocks of 1,280 bytes, would
    # allow 14 workgroups per CU, so the slot trees go global: 8 blocks, 16
    # per CU); LZMA_GPU_PLAN_NO_MERGE_LAT: four classes
    # launched concurrently on forked streams
    for opts, n_classes in ((None, 1), (L.plan_options("auto", flags=8), 4)):
        plan, res, d_dst = _device_decode(L, torch, descs, comp, int(nout.sum()), opts)
        masks = sorted(plan.classes[k].lds_mask for k in range(plan.n_classes))
        assert plan.n_classes == n_classes and plan.n_lds == count and \
            set(masks) <= {M_LAT, M_LAT_SG}, masks
        if n_classes == 1:
            assert plan.classes[0].groups_per_cu == 16 and plan.classes[0].lanes_per_group == 1
            assert plan.classes[0].lds_mask == M_LAT_SG
        # FINISH_END reads the end mark (FINISHED_WITH_MARK); FINISH_ANY stops
        # at destLen in front of it (NOT_FINISHED)
        want_status = np.where(fin == 1, 1, 2)
        assert (res["res"] == 0).all() and (res["status"] == want_status).all()
        assert (res["dest_len"] == nout).all()
        assert (res["src_len"][fin == 1] == lens[fin == 1]).all()
        assert (res["src_len"][fin == 0] < lens[fin == 0]).all()
        out = d_dst[:int(nout.sum())].cpu().numpy().tobytes()
        assert out == plain


def test_cfg5_full_length_1_to_256k(L, torch):
    """BASELINE config 5 at its stated size: 32,768 streams, lc 0-4,
    lp 0-2 (lc + lp <= 4), pb 0-4, dict 4K-1M, lengths log-uniform 1 KiB-256 KiB
    (1.46 GB decompressed), end mark on half -- one planned batch, round trip to
    the plaintext and exact per-stream results; a 512-stream sample (every 64th
    stream) against the oracle's LzmaDecode, output and results.  Encoded by
    liblzma preset 1 so the 1.5 GB encode fits a test (the encoder does not
    affect decode parity; bench.py's cfg5 leg encodes preset 6)."""
    count = 32768
    with ThreadPoolExecutor(W.workers()) as ex:
        parts = list(ex.map(lambda i: W.cfg5_stream(i, max_log2=8, preset=1), range(count)))
    nout = np.array([len(p[0]) for p in parts], dtype=np.uint64)
    lens = np.array([len(p[1]) for p in parts], dtype=np.uint64)
    fin = np.array([p[3] for p in parts])
    assert nout.min() >= 1024 and nout.max() <= 262144 and nout.max() > 200000
    so = np.zeros(count, np.uint64)
    so[1:] = np.cumsum(lens)[:-1]
    do = np.zeros(count, np.uint64)
    do[1:] = np.cumsum(nout)[:-1]
    descs = L.make_descs([dict(src_off=int(so[i]), src_len=int(lens[i]), dst_off=int(do[i]),
                               dst_cap=int(nout[i]), props=parts[i][2], finish=int(fin[i]))
                          for i in range(count)])
    comp = np.frombuffer(b"".join(p[1] for p in parts), dtype=np.uint8)
    plan, res, d_dst = _device_decode(L, torch, descs, comp, int(nout.sum()))
    assert plan.n_lds == count
    want_status = np.where(fin == 1, 1, 2)
    assert (res["res"] == 0).all() and (res["status"] == want_status).all()
    assert (res["dest_len"] == nout).all()
    assert (res["src_len"][fin == 1] == lens[fin == 1]).all()
    out = d_dst[:int(nout.sum())].cpu().numpy()
    for i in range(count):
        assert out[int(do[i]):int(do[i] + nout[i])].tobytes() == parts[i][0], i
    orc = native.oracle()
    comp_b = comp.tobytes()
    for i in range(0, count, 64):
        s = comp_b[int(so[i]):int(so[i] + lens[i])]
        e = native.decode(orc, "orc", s, parts[i][2], int(nout[i]), int(fin[i]))
        assert (int(res["res"][i]), int(res["status"][i]), int(res["dest_len"][i]),
                int(res["src_len"][i])) == e[:4], i
        assert out[int(do[i]):int(do[i]) + e[2]].tobytes() == e[4], i


def test_cfg4_1024_lzma2_blocks_coop_kernel(L, torch):
    """BASELINE config 4's per-GPU shard: 1,024 LZMA2 dict-reset blocks of 1 MiB
    (lc3/lp0/pb2, dict 1 MiB) in one file, split on the host by chunk headers,
    one block per item -- 4 blocks per CU, so the wave-cooperative kernel.  16
    distinct blocks repeat through the file (encode time)."""
    uniq, nb = 16, 1024
    with ThreadPoolExecutor(W.workers()) as ex:
        ub = list(ex.map(lambda i: W.lzma2_block(50000 + i, 1 << 20), range(uniq)))
    blob = b"".join(ub[b % uniq][1] for b in range(nb)) + b"\0"
    blocks = L.split_lzma2_blocks(blob)
    assert len(blocks) == nb and all(u == 1 << 20 for _, _, u in blocks)
    items = [dict(src_off=int(o), src_len=int(ln), dst_off=k << 20, dst_cap=int(u),
                  props=bytes([16]), finish=0, kind=L.KIND_LZMA2)
             for k, (o, ln, u) in enumerate(blocks)]
    descs = L.make_descs(items)
    plan, res, d_dst = _device_decode(L, torch, descs, np.frombuffer(blob, np.uint8), nb << 20)
    assert plan.n_classes == 1 and plan.classes[0].lds_mask == M_ALL | COOP
    assert (res["res"] == 0).all() and (res["status"] == 2).all()
    assert (res["dest_len"] == 1 << 20).all()
    assert (res["src_len"] == np.array([ln for _, ln, _ in blocks])).all()
    out = d_dst[:nb << 20].cpu().numpy().reshape(nb, 1 << 20)
    for k in range(nb):
        assert out[k].tobytes() == ub[k % uniq][0], k


@pytest.mark.parametrize("kernel", ("throughput", "throughput_slices", "latency"))
def test_cfg4_blocks_on_lane_kernels(L, torch, kernel):
    """The same LZMA2 dict-reset blocks (256 KiB here) on the per-lane kernels,
    forced: LZMA2 chunk walking on 0x105 (32 lanes per wave) and 0x1BF."""
    uniq, nb = 8, 512
    with ThreadPoolExecutor(W.workers()) as ex:
        ub = list(ex.map(lambda i: W.lzma2_block(52000 + i, 1 << 18, dsz=1 << 18), range(uniq)))
    blob = b"".join(ub[b % uniq][1] for b in range(nb)) + b"\0"
    blocks = L.split_lzma2_blocks(blob)
    assert len(blocks) == nb
    items = [dict(src_off=int(o), src_len=int(ln), dst_off=k << 18, dst_cap=int(u),
                  props=bytes([14]), finish=1 if k % 2 else 0, kind=L.KIND_LZMA2)
             for k, (o, ln, u) in enumerate(blocks)]
    descs = L.make_descs(items)
    plan, res, d_dst = _device_decode(L, torch, descs, np.frombuffer(blob, np.uint8), nb << 18,
                                      _opts(L, kernel))
    _check_plan(plan, kernel)
    # FINISH_END over a block without its EOS byte: NEEDS_MORE_INPUT, all bytes out
    want_status = np.array([3 if k % 2 else 2 for k in range(nb)])
    assert (res["res"] == 0).all() and (res["status"] == want_status).all()
    assert (res["dest_len"] == 1 << 18).all()
    out = d_dst[:nb << 18].cpu().numpy().reshape(nb, 1 << 18)
    for k in range(nb):
        assert out[k].tobytes() == ub[k % uniq][0], k

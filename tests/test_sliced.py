"""Time-sliced batches (second half; include/lzma_gpu.h
LzmaGpu_PlanSliced / LzmaGpu_DecodeBatchSliced): a batch decoded in rounds of
at most `slice` output bytes per stream, the CLzmaDec state (LzmaDec.h:50-69)
spilled to device memory between rounds.

The reference has no batch, but it has the contract the rounds rest on:
LzmaDec_DecodeToDic resumes at any output boundary (LzmaDec.c:719-838) and a
sequence of calls with growing dicLimit under LZMA_FINISH_ANY, the last with
the caller's finish mode, ends in the state one LzmaDecode call
(LzmaDec.c:972-1002) reaches.  So every sliced result must equal the
reference's LzmaDecode result -- the golden vectors (reference-decoded) and
the oracle's -- bit for bit, at every slice size and on every kernel.

CPU: the planner (host only, no device).  GPU: goldens and the 1,500-case
fuzz set through the lane / cooperative / global round kernels at slices from
97 bytes to one round; round-by-round control (a stream whose capacity fits r
slices is finished after round r, the active count only falls); long LZMA1
streams (up to 800 KB, 1 MiB dictionaries, distances the 20 KB fuzz never
reaches) against the oracle, sliced and one-shot on every batch kernel.
"""
import lzma
import random

import numpy as np
import pytest

import golden_cases as G
import native
import workloads as W

RES_DT = np.dtype([("res", "<i4"), ("status", "<i4"), ("dest_len", "<u8"), ("src_len", "<u8")])

@pytest.fixture(scope="module")
def L():
    import lzmagpu
    return lzmagpu


def _items(n, cap, src_len=100, props=None, kind=0):
    props = props or W.props_bytes(3, 0, 2, 1 << 16)
    return [dict(src_off=i * src_len, src_len=src_len, dst_off=i * cap, dst_cap=cap, props=props,
                 kind=kind) for i in range(n)]


# ---------------------------------------------------------------- planner (CPU)

def test_plan_rounds_tables_and_order(L):
    items = _items(5, 10_000)
    items[3]["dst_cap"] = 100_000          # the longest: ceil(100000 / 4096) rounds
    items[1]["src_len"] = 4                # too short for the rc init: no table
    items[2]["props"] = bytes([225, 0, 0, 1, 0])  # bad props: no table
    descs = L.make_descs(items)
    plan, order = L.plan_sliced(descs, 4096)
    assert plan.n == 5 and plan.slice_bytes == 4096
    assert plan.rounds == (100_000 + 4095) // 4096
    cells = 56 * 4 + 950 + (768 << 3)      # lc3/lp0/pb2 (table_cells)
    assert plan.table_cells == (cells + 7) // 8 * 8
    assert descs[1].probs_off == 2 ** 64 - 1 and descs[2].probs_off == 2 ** 64 - 1
    offs = [descs[i].probs_off for i in (0, 3, 4)]
    assert all(o % 8 == 0 for o in offs) and len(set(offs)) == 3
    assert all(1024 <= o * 2 < plan.list_off for o in offs)  # behind the 5 sessions
    assert plan.sess_off == 0 and plan.list_off < plan.ctr_off < plan.workspace_bytes
    assert plan.workspace_bytes >= plan.ctr_off + (2 * plan.rounds + 2) * 4
    assert order[0] == 3                   # longest work first
    assert sorted(order[:5]) == [0, 1, 2, 3, 4]


def test_plan_kernel_choice_and_errors(L):
    # few streams per CU: cooperative; many: one lane per wave; wide tables: global
    p, _ = L.plan_sliced(L.make_descs(_items(64, 4096)), 1024)
    assert p.kernel == L.SLICED_KERNELS["coop"]
    p, _ = L.plan_sliced(L.make_descs(_items(8192, 4096)), 1024)
    # lc3: the latency kernel's sections staged (5.2 KB), 16 streams per CU
    assert p.kernel == L.SLICED_KERNELS["lane"] and p.groups_per_cu == 16
    assert p.lds_mask == 0x200001BF and p.table_cells == 2048 + 48 * 3 + 2 * 66 + 256 + 16
    p, _ = L.plan_sliced(L.make_descs(_items(8192, 4096, props=W.props_bytes(0, 0, 0, 4096))), 64)
    assert p.lds_mask == 0x7FF and p.groups_per_cu == 16   # lc0: the whole table fits 16 per CU
    wide = W.props_bytes(8, 4, 2, 1 << 16)  # 768 << 12 cells: too wide for LDS
    p, _ = L.plan_sliced(L.make_descs(_items(4, 4096, props=wide)), 1024)
    assert p.kernel == L.SLICED_KERNELS["global"]
    assert p.n_inplace == 4
    # forced LDS kernel: wide tables run in place on the global kernel, same rounds
    p, _ = L.plan_sliced(L.make_descs(_items(4, 4096, props=wide)), 1024, "lane")
    assert p.kernel == L.SLICED_KERNELS["lane"] and p.table_cells == 0 and p.n_inplace == 4
    mixed = _items(4, 4096)
    mixed[1]["props"] = wide
    p, _ = L.plan_sliced(L.make_descs(mixed), 1024)
    assert p.kernel == L.SLICED_KERNELS["coop"] and p.n_inplace == 1
    assert p.table_cells == (56 * 4 + 950 + 768 * 8 + 7) // 8 * 8
    with pytest.raises(RuntimeError):
        L.plan_sliced(L.make_descs(_items(4, 4096)), 0)          # slice 0
    with pytest.raises(RuntimeError):
        L.plan_sliced(L.make_descs(_items(4, 4096, kind=1)), 4096)  # LZMA2 item
    with pytest.raises(RuntimeError):
        L.plan_sliced(L.make_descs(_items(1, 1 << 40)), 4096)    # > 2^24 rounds
    p, _ = L.plan_sliced(L.make_descs(_items(3, 0)), 4096)      # empty outputs: one round
    assert p.rounds == 1
    p, _ = L.plan_sliced(L.make_descs([]), 4096)
    assert p.n == 0


# ---------------------------------------------------------------- GPU parity

def _gpu(L):
    if L.device_count() <= 0:
        pytest.fail("no HIP device visible: " + L.last_error())


def _golden_lzma():
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
    return items, b"".join(srcs), doff, exp


@pytest.mark.gpu
@pytest.mark.parametrize("kernel,slice_", [("lane", 97), ("lane", 4096), ("coop", 97),
                                           ("coop", 65536), ("global", 4096),
                                           ("auto", 1 << 30)])
def test_goldens_sliced(L, kernel, slice_):
    _gpu(L)
    items, src, dst_bytes, exp = _golden_lzma()
    plan = L.SlicedPlan()
    r, res, dst = L.decode_batch_sliced_host(L.make_descs(items), src, dst_bytes, slice_,
                                             kernel, plan)
    assert r == 0, L.last_error()
    if kernel != "auto":
        assert plan.kernel == L.SLICED_KERNELS[kernel]
    assert plan.rounds == max(1, -(-max(it["dst_cap"] for it in items) // slice_))
    bad = []
    for k, (want, sha, note) in enumerate(exp):
        got = (res[k].res, res[k].status, res[k].dest_len, res[k].src_len)
        out = dst[items[k]["dst_off"]:items[k]["dst_off"] + res[k].dest_len]
        if got != want or G.sha(out) != sha:
            bad.append((k, note, got, want))
    assert not bad, (kernel, slice_, len(bad), bad[:8])


_FZ = {}


def _fuzz():
    if "v" not in _FZ:
        from test_gpu_kernels import _fuzz_set
        _FZ["v"] = _fuzz_set()
    return _FZ["v"]


@pytest.mark.gpu
@pytest.mark.parametrize("kernel,slice_", [("lane", 257), ("coop", 1000), ("global", 4096),
                                           ("auto", 3000)])
def test_fuzz_sliced_vs_oracle(L, kernel, slice_):
    _gpu(L)
    items, src, dst_bytes, exp = _fuzz()
    r, res, dst = L.decode_batch_sliced_host(L.make_descs(items), src, dst_bytes, slice_, kernel)
    assert r == 0, L.last_error()
    bad = []
    for k in range(len(items)):
        got = (res[k].res, res[k].status, res[k].dest_len, res[k].src_len)
        out = dst[items[k]["dst_off"]:items[k]["dst_off"] + res[k].dest_len]
        if got != exp[k][:4] or out != exp[k][4]:
            bad.append((k, got, exp[k][:4]))
    assert not bad, (kernel, slice_, len(bad), bad[:8])


@pytest.mark.gpu
def test_round_by_round_control(L):
    """Rounds enqueued one at a time: after round r every stream whose capacity
    is at most (r + 1) slices has its final result, the others are still
    unfinished (a round never decodes more than one slice per stream), and the
    active count never rises."""
    _gpu(L)
    import torch
    rng = random.Random(5)
    items, srcs, plains, off, doff = [], [], [], 0, 0
    for i in range(300):
        n = rng.choice([0, 500, 3000, 9000, 20000, 41000])
        data = native.gen("text", 61_000 + i, n)
        comp = lzma.compress(data, format=lzma.FORMAT_RAW, filters=[
            {"id": lzma.FILTER_LZMA1, "dict_size": 1 << 16, "lc": 3, "lp": 0, "pb": 2}])
        items.append(dict(src_off=off, src_len=len(comp), dst_off=doff, dst_cap=n,
                          props=W.props_bytes(3, 0, 2, 1 << 16), finish=0))
        srcs.append(comp)
        plains.append(data)
        off += len(comp)
        doff += n
    slice_ = 4096
    descs = L.make_descs(items)
    plan, order = L.plan_sliced(descs, slice_)
    dev = torch.device("cuda:0")
    t_src = torch.frombuffer(bytearray(b"".join(srcs)), dtype=torch.uint8).to(dev)
    t_dst = torch.full((max(doff, 1),), 0xA5, dtype=torch.uint8, device=dev)
    t_ws = torch.empty(plan.workspace_bytes, dtype=torch.uint8, device=dev)
    t_desc = torch.frombuffer(bytearray(bytes(descs)), dtype=torch.uint8).to(dev)
    t_ord = torch.frombuffer(bytearray(bytes(order)), dtype=torch.uint8).to(dev)
    n = len(items)
    t_res = torch.full((n * 24,), 0xFF, dtype=torch.uint8, device=dev)
    active = [n]
    for r in range(plan.rounds):
        rc = L.decode_batch_sliced_device(plan, t_desc.data_ptr(), t_ord.data_ptr(),
                                          t_src.data_ptr(), t_dst.data_ptr(), t_ws.data_ptr(),
                                          t_res.data_ptr(), r, 1)
        assert rc == 0, L.last_error()
        active.append(L.sliced_active(plan, t_ws.data_ptr(), r + 1))
        res = np.frombuffer(t_res.cpu().numpy().tobytes(), dtype=RES_DT)
        for k, it in enumerate(items):
            fits = it["dst_cap"] <= (r + 1) * slice_
            written = res[k]["res"] != -1
            assert written == fits, (r, k, it["dst_cap"], res[k])
    assert active == sorted(active, reverse=True) and active[-1] == 0, active
    res = np.frombuffer(t_res.cpu().numpy().tobytes(), dtype=RES_DT)
    out = t_dst.cpu().numpy().tobytes()
    for k, it in enumerate(items):
        assert res[k]["res"] == 0 and res[k]["dest_len"] == it["dst_cap"], (k, res[k])
        assert out[it["dst_off"]:it["dst_off"] + it["dst_cap"]] == plains[k]


def _long_set():
    """LZMA1 streams up to 600 KB with 1 MiB dictionaries (long distances),
    random presets, some truncated or bit-flipped; oracle expectations."""
    if "long" in _FZ:
        return _FZ["long"]
    rng = random.Random(1709)
    orc = native.oracle()
    items, srcs, exp, off, doff = [], [], [], 0, 0
    for it in range(48):
        lc, lp, pb = rng.randrange(5), rng.randrange(3), rng.randrange(5)
        if lc + lp > 4:
            lp = 0
        n = rng.choice([70_000, 200_000, 600_000])
        data = native.gen(rng.choice(["text", "text", "runs"]), 71_000 + it, n)
        data = data[: n // 2] + data[: n // 3] + data[n // 2:]   # repeats 100+ KB back
        comp = bytearray(lzma.compress(data, format=lzma.FORMAT_RAW, filters=[
            {"id": lzma.FILTER_LZMA1, "dict_size": 1 << 20, "lc": lc, "lp": lp, "pb": pb,
             "preset": rng.choice([6, 9])}]))
        mode = rng.randrange(6)
        if mode == 1:
            comp[rng.randrange(5, len(comp))] ^= 1 << rng.randrange(8)
        elif mode == 2:
            comp = comp[:rng.randrange(len(comp) // 2, len(comp))]
        cap = len(data) + rng.choice([0, 0, -1000])
        props = W.props_bytes(lc, lp, pb, 1 << 20)
        fin = rng.randrange(2)
        comp = bytes(comp)
        items.append(dict(src_off=off, src_len=len(comp), dst_off=doff, dst_cap=cap, props=props,
                          finish=fin))
        srcs.append(comp)
        exp.append(native.decode(orc, "orc", comp, props, cap, fin))
        off += len(comp)
        doff += cap
    _FZ["long"] = (items, b"".join(srcs), doff, exp)
    return _FZ["long"]


def _check(items, res, dst, exp, what):
    bad = []
    for k in range(len(items)):
        got = (res[k].res, res[k].status, res[k].dest_len, res[k].src_len)
        out = dst[items[k]["dst_off"]:items[k]["dst_off"] + res[k].dest_len]
        if got != exp[k][:4] or out != exp[k][4]:
            bad.append((k, got, exp[k][:4]))
    assert not bad, (what, len(bad), bad[:6])


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["latency", "coop", "global", "throughput"])
def test_long_lzma1_one_shot_each_kernel(L, kernel):
    _gpu(L)
    items, src, dst_bytes, exp = _long_set()
    r, res, dst = L.decode_batch_host(L.make_descs(items), src, dst_bytes,
                                      L.plan_options(kernel, cus=8))
    assert r == 0, L.last_error()
    _check(items, res, dst, exp, kernel)


@pytest.mark.gpu
@pytest.mark.parametrize("kernel,slice_", [("lane", 65536), ("coop", 100_000)])
def test_long_lzma1_sliced(L, kernel, slice_):
    _gpu(L)
    items, src, dst_bytes, exp = _long_set()
    r, res, dst = L.decode_batch_sliced_host(L.make_descs(items), src, dst_bytes, slice_, kernel)
    assert r == 0, L.last_error()
    _check(items, res, dst, exp, kernel)

"""CRC-32 of decoded output (reference 7zCrc.c CrcCalc /
CrcUpdate, poly 0xEDB88320).

CPU (no GPU): the oracle restatement and the kernels' per-lane code (host
build, tests/emu) against the golden values the reference produced
(tests/golden/crc_cases.json, tests/golden/make_golden_crc.py) and against
zlib.crc32 (the same CRC-32); the chunk planner.
GPU (-m gpu): CrcCalc / CrcUpdate drop-ins, CrcGpu_Batch over ragged
misaligned ranges, and LzmaGpu_Crc32Batch straight on a decode batch.
"""
import ctypes
import json
import os
import random
import subprocess
import zlib

import pytest

import native

GOLDEN = os.path.join(native.ROOT, "tests", "golden", "crc_cases.json")
EMU_SO = os.path.join(native.ROOT, "tests", "emu", "liblane_emu.so")


def golden():
    with open(GOLDEN) as f:
        d = json.load(f)
    out = []
    for c in d["cases"]:
        if "hex" in c:
            data = bytes.fromhex(c["hex"])
        else:
            data = native.gen(c["gen"], c["seed"], c["n"] + c["skip"])[c["skip"]:]
        out.append((data, c["crc_calc"], c["crc_update"]))
    return d["update_seed"], out


def test_golden_self_consistent_with_zlib():
    _, cases = golden()
    for data, calc, _ in cases:
        assert zlib.crc32(data) == calc


def test_oracle_matches_golden():
    orc = native.oracle()
    upd, calc = native.crc_funcs(orc, "orc_crc_update", "orc_crc_calc")
    seed, cases = golden()
    for data, c, u in cases:
        assert calc(data, len(data)) == c
        assert upd(seed, data, len(data)) == u


@pytest.fixture(scope="module")
def emu():
    subprocess.run(["make", "-s", "-f", "tests/emu/Makefile"], cwd=native.ROOT, check=True)
    lib = ctypes.CDLL(EMU_SO)
    f = lib.emu_crc_ranges
    f.restype = None
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                  ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
    return lib


def emu_crc(emu, datas, init=0xFFFFFFFF, xorout=0xFFFFFFFF, phase=0):
    """All ranges packed (16-byte margins, each starting at a varying
    alignment) in one buffer, through the kernels' per-lane code."""
    buf, offs = bytearray(b"\xAA" * (48 + phase)), []
    for k, d in enumerate(datas):
        offs.append(len(buf))
        buf += d + b"\x55" * ((k * 7) % 16)
    buf += b"\xAA" * 48
    n = len(datas)
    cbuf = ctypes.create_string_buffer(bytes(buf), len(buf))
    off = (ctypes.c_uint64 * max(n, 1))(*offs)
    ln = (ctypes.c_uint64 * max(n, 1))(*[len(d) for d in datas])
    out = (ctypes.c_uint32 * max(n, 1))()
    emu.emu_crc_ranges(cbuf, off, ln, n, init, xorout, out)
    return list(out)[:n]


def test_emu_matches_golden(emu):
    seed, cases = golden()
    datas = [c[0] for c in cases]
    for phase in range(4):
        assert emu_crc(emu, datas, phase=phase * 5) == [c[1] for c in cases]
    assert emu_crc(emu, datas, seed, 0) == [c[2] for c in cases]


def test_emu_fuzz_vs_zlib(emu):
    rng = random.Random(11)
    datas = []
    for i in range(120):
        n = rng.choice([0, 1, 2, 15, 16, 17, 2047, 2048, 2049, 4096, 4111, 8192 + 5,
                        rng.randrange(1, 40000)])
        datas.append(native.gen(rng.choice(["text", "random", "runs"]), 4000 + i, n))
    assert emu_crc(emu, datas, phase=3) == [zlib.crc32(d) for d in datas]


def test_chunk_plan():
    import lzmagpu as L
    caps = [0, 1, 2048, 2049, 4096, 10000]
    base, rng, total = L.crc_plan(caps)
    want = [0, 1, 1, 2, 2, 5]
    assert total == sum(want)
    acc = 0
    for i, w in enumerate(want):
        assert base[i] == acc
        for k in range(w):
            assert rng[acc + k] == i
        acc += w


# ---------------------------------------------------------------- GPU

@pytest.mark.gpu
def test_gpu_crc_dropins_golden():
    import lzmagpu as L
    L.lib.CrcGenerateTable()
    seed, cases = golden()
    for data, c, u in cases:
        assert L.CrcCalc(data) == c
        assert L.CrcUpdate(seed, data) == u


@pytest.mark.gpu
def test_gpu_crc_batch_ragged():
    import torch
    import lzmagpu as L
    rng = random.Random(5)
    datas = [native.gen(rng.choice(["text", "random", "runs"]), 9000 + i,
                        rng.choice([0, 1, 5, 16, 2047, 2048, 2049, 6000, rng.randrange(70000)]))
             for i in range(700)]
    buf, offs = bytearray(), []
    for d in datas:
        buf += b"\x00" * rng.randrange(0, 19)
        offs.append(len(buf))
        buf += d
    n = len(datas)
    caps = [len(d) + rng.choice([0, 0, 3000]) for d in datas]
    base, crange, total = L.crc_plan(caps)
    dev = torch.device("cuda")
    d_data = torch.frombuffer(bytearray(buf) + b"\0", dtype=torch.uint8).to(dev)
    d_off = torch.tensor(offs, dtype=torch.int64, device=dev)
    d_len = torch.tensor([len(d) for d in datas], dtype=torch.int64, device=dev)
    d_base = torch.tensor(list(base)[:n], dtype=torch.int32, device=dev)
    d_range = torch.tensor(list(crange)[:max(total, 1)], dtype=torch.int32, device=dev)
    d_chunks = torch.empty(max(total, 1), dtype=torch.int32, device=dev)
    d_crc = torch.empty(n, dtype=torch.int32, device=dev)
    for init, xorout, ref in ((0xFFFFFFFF, 0xFFFFFFFF, lambda d: zlib.crc32(d)),
                              (0x12345678, 0, None)):
        assert L.crc_batch_device(d_data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), n,
                                  d_base.data_ptr(), d_range.data_ptr(), total, init, xorout,
                                  d_chunks.data_ptr(), d_crc.data_ptr()) == 0
        torch.cuda.synchronize()
        got = [v & 0xFFFFFFFF for v in d_crc.cpu().tolist()]
        if ref is not None:
            assert got == [ref(d) for d in datas]
        else:
            orc = native.oracle()
            upd, _ = native.crc_funcs(orc, "orc_crc_update", "orc_crc_calc")
            assert got == [upd(init, d, len(d)) for d in datas]


@pytest.mark.gpu
def test_gpu_crc_of_decode_batch():
    """LzmaGpu_Crc32Batch on the decode's own device buffers (no host hop)."""
    import lzma
    import torch
    import lzmagpu as L
    rng = random.Random(8)
    items, srcs, plain, off, doff = [], [], [], 0, 0
    for i in range(300):
        n = rng.choice([0, 100, 4096, 9000, 30000])
        data = native.gen(rng.choice(["text", "runs", "random"]), 12000 + i, n)
        f = [{"id": lzma.FILTER_LZMA1, "dict_size": 1 << 16, "lc": 3, "lp": 0, "pb": 2,
              "preset": 6}]
        c = lzma.compress(data, format=lzma.FORMAT_RAW, filters=f)
        cap = n + rng.choice([0, 0, 77])
        items.append(dict(src_off=off, src_len=len(c), dst_off=doff, dst_cap=cap,
                          props=b"\x5d\x00\x00\x01\x00", finish=0))
        srcs.append(c)
        plain.append(data)
        off += len(c)
        doff += cap + rng.randrange(0, 9)
    descs = L.make_descs(items)
    plan, order = L.plan_ex(descs)
    n = len(items)
    dev = torch.device("cuda")
    src = b"".join(srcs)
    d_src = torch.frombuffer(bytearray(src) + b"\0" * 16, dtype=torch.uint8).to(dev)
    d_dst = torch.zeros(doff + 16, dtype=torch.uint8, device=dev)
    d_ws = torch.zeros(max(plan.workspace_bytes, 16), dtype=torch.uint8, device=dev)
    d_desc = torch.frombuffer(bytearray(bytes(descs)), dtype=torch.uint8).to(dev)
    d_order = torch.tensor(list(order), dtype=torch.int32, device=dev)
    d_res = torch.zeros(n * 24, dtype=torch.uint8, device=dev)
    assert L.decode_batch_device_ex(plan, d_desc.data_ptr(), d_order.data_ptr(), d_src.data_ptr(),
                                    d_dst.data_ptr(), d_ws.data_ptr(), d_res.data_ptr()) == 0
    base, crange, total = L.crc32_plan_decoded(descs)
    d_base = torch.tensor(list(base)[:n], dtype=torch.int32, device=dev)
    d_range = torch.tensor(list(crange)[:max(total, 1)], dtype=torch.int32, device=dev)
    d_chunks = torch.empty(max(total, 1), dtype=torch.int32, device=dev)
    d_crc = torch.empty(n, dtype=torch.int32, device=dev)
    assert L.crc32_batch_decoded(d_desc.data_ptr(), d_res.data_ptr(), n, d_dst.data_ptr(),
                                 d_base.data_ptr(), d_range.data_ptr(), total,
                                 d_chunks.data_ptr(), d_crc.data_ptr()) == 0
    torch.cuda.synchronize()
    res = (L.Result * n).from_buffer_copy(bytes(d_res.cpu().numpy()))
    got = [v & 0xFFFFFFFF for v in d_crc.cpu().tolist()]
    for i in range(n):
        assert res[i].res in (0, 6) and res[i].dest_len == len(plain[i])
        assert got[i] == zlib.crc32(plain[i])

"""xz files as GPU block batches, x86 BCJ and CRC-64.

Reference: XzUnpacker_Code (XzDec.c:604-870), x86_Convert (Bra86.c:11-85),
Crc64Calc (XzCrc64.c:30), compiled in place and recorded in
tests/golden/xz_cases.json + xz_blob.bin (tests/golden/make_golden_xz.py;
every valid file there also decodes identically through liblzma).

CPU (no GPU): the index (LzmaGpu_XzIndex is host code) against the
reference's decoded sizes and error codes; the BCJ and CRC-64 kernels'
per-lane code (host build, tests/emu) against the reference's outputs.
GPU (-m gpu): LzmaGpu_XzDecode on every fixture file, the x86_Convert and
Crc64Calc drop-ins, and a many-block file decoded as one batch.
"""
import ctypes
import hashlib
import json
import os
import struct
import subprocess
import sys

import pytest

import native

GOLDEN = os.path.join(native.ROOT, "tests", "golden")
EMU_SO = os.path.join(native.ROOT, "tests", "emu", "liblane_emu.so")
sys.path.insert(0, GOLDEN)
sys.path.insert(0, os.path.join(native.ROOT, "lzma-sdk-zliblike_amd"))


def fixtures():
    with open(os.path.join(GOLDEN, "xz_cases.json")) as f:
        d = json.load(f)
    with open(os.path.join(GOLDEN, "xz_blob.bin"), "rb") as f:
        blob = f.read()
    assert hashlib.sha256(blob).hexdigest() == d["blob_sha256"]
    d["blob"] = blob
    return d


def data_of(d, c):
    return d["blob"][c["off"]:c["off"] + c["len"]]


@pytest.fixture(scope="module")
def L():
    import lzmagpu
    return lzmagpu


@pytest.fixture(scope="module")
def emu():
    subprocess.run(["make", "-s", "-f", "tests/emu/Makefile"], cwd=native.ROOT, check=True)
    lib = ctypes.CDLL(EMU_SO)
    lib.emu_bcj_x86_tiled.restype = ctypes.c_uint64
    lib.emu_bcj_x86_tiled.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint32,
                                      ctypes.POINTER(ctypes.c_uint32), ctypes.c_int]
    lib.emu_bcj_x86.restype = ctypes.c_uint64
    lib.emu_bcj_x86.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint32,
                                ctypes.POINTER(ctypes.c_uint32), ctypes.c_int]
    lib.emu_crc64_ranges.restype = None
    lib.emu_crc64_ranges.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64,
                                     ctypes.c_void_p]
    return lib


def test_index_matches_reference(L):
    d = fixtures()
    for c in d["xz"]:
        r, blocks, total = L.xz_index(data_of(d, c))
        if c["valid"]:
            assert r == 0, c["note"]
            assert total == c["dest_len"], c["note"]
            assert sum(b.unpack_size for b in blocks) == total
            # blocks tile the output in file order
            off = 0
            for b in blocks:
                assert b.dst_off == off and b.check_size in (0, 4, 8, 32)
                assert b.data_off > b.header_off and b.check_off >= b.data_off + b.pack_size
                off += b.unpack_size
        elif c["res"] == 17:  # bad stream magic: the same class of error
            assert r == 17, c["note"]
    notes = {c["note"]: c for c in d["xz"]}
    r, blocks, _ = L.xz_index(data_of(d, notes["24 small blocks, check 4"]))
    assert len(blocks) == 24 and all(b.check_type == 4 for b in blocks)
    r, blocks, _ = L.xz_index(data_of(d, notes["3 concatenated streams + stream padding"]))
    assert [b.stream for b in blocks] == [0, 1, 2]
    assert [b.check_type for b in blocks] == [1, 4, 10]
    x = [c for c in d["xz"] if c["note"].startswith("multi-block, x86")][0]
    r, blocks, _ = L.xz_index(data_of(d, x))
    assert [b.x86 for b in blocks] == [1, 1, 1, 1]
    assert [b.x86_ip for b in blocks] == [0, 0, 0x2000, 0]


def test_index_rejects_malformed(L):
    d = fixtures()
    good = data_of(d, [c for c in d["xz"] if c["note"].startswith("multi-block stream")][0])
    assert L.xz_index(b"")[0] == 17
    assert L.xz_index(good[:-1])[0] == 17                # not a multiple of 4
    bad = bytearray(good)
    bad[-1] ^= 1                                         # footer magic
    assert L.xz_index(bytes(bad))[0] == 17
    bad = bytearray(good)
    bad[-4] ^= 1                                         # footer flags: unsupported
    assert L.xz_index(bytes(bad))[0] in (4, 16)
    bad = bytearray(good)
    bad[-12] ^= 1                                        # footer CRC
    assert L.xz_index(bytes(bad))[0] == 16
    bad = bytearray(good)
    bad[13] ^= 0x10                                      # first block header (CRC)
    assert L.xz_index(bytes(bad))[0] == 16


def test_bcj_emu_matches_reference(emu):
    d = fixtures()
    for c in d["bcj"]:
        n = c["len"]
        buf = ctypes.create_string_buffer(d["blob"][c["off"]:c["off"] + n] + b"\0" * 32, n + 32)
        st = ctypes.c_uint32(c["state_in"])
        done = emu.emu_bcj_x86(buf, n, c["ip"], ctypes.byref(st), c["encoding"])
        assert (done, st.value) == (c["done"], c["state_out"]), c
        assert hashlib.sha256(buf.raw[:n]).hexdigest() == c["sha256"], c


def test_bcj_tiled_emu_matches_reference(emu):
    """The tiled x86 BCJ kernel's phases (hit records per 4 KiB tile, then the
    reference's decisions over them) on every reference fixture, and against
    the lane-serial statement on branch-dense buffers spanning many tiles
    (conversions across tile edges, E8/E9 runs, every start state)."""
    d = fixtures()
    for c in d["bcj"]:
        n = c["len"]
        buf = ctypes.create_string_buffer(d["blob"][c["off"]:c["off"] + n] + b"\0" * 32, n + 32)
        st = ctypes.c_uint32(c["state_in"])
        done = emu.emu_bcj_x86_tiled(buf, n, c["ip"], ctypes.byref(st), c["encoding"])
        assert (done, st.value) == (c["done"], c["state_out"]), c
        assert hashlib.sha256(buf.raw[:n]).hexdigest() == c["sha256"], c
    import random
    rng = random.Random(17)
    for it in range(40):
        n = rng.choice([5, 4099, 4100, 4101, 8192 + 3, 20000, 50001])
        b = bytearray(rng.getrandbits(8) for _ in range(n))
        dens = rng.choice([0.02, 0.1, 0.3, 0.6])
        for i in range(n):
            if rng.random() < dens:
                b[i] = rng.choice([0xE8, 0xE9])
                if i + 4 < n and rng.random() < 0.7:
                    b[i + 4] = rng.choice([0x00, 0xFF])
        # force hits right at the tile edges
        for e in range(4096, n, 4096):
            for k in (-4, -3, -2, -1, 0, 1):
                if 0 <= e + k < n and rng.random() < 0.5:
                    b[e + k] = 0xE8
        ip, s0, enc = rng.getrandbits(32), rng.randrange(8), rng.randrange(2)
        b1 = ctypes.create_string_buffer(bytes(b) + b"\0" * 32, n + 32)
        b2 = ctypes.create_string_buffer(bytes(b) + b"\0" * 32, n + 32)
        s1, s2 = ctypes.c_uint32(s0), ctypes.c_uint32(s0)
        d1 = emu.emu_bcj_x86(b1, n, ip, ctypes.byref(s1), enc)
        d2 = emu.emu_bcj_x86_tiled(b2, n, ip, ctypes.byref(s2), enc)
        assert (d1, s1.value) == (d2, s2.value) and b1.raw == b2.raw, (it, n, dens)


def test_crc64_emu_matches_reference(emu):
    d = fixtures()
    for c in d["crc64"]:
        n = c["len"]
        pad = 16
        buf = b"\0" * pad + d["blob"][c["off"]:c["off"] + n] + b"\0" * 32
        off = (ctypes.c_uint64 * 1)(pad)
        ln = (ctypes.c_uint64 * 1)(n)
        out = (ctypes.c_uint64 * 1)()
        emu.emu_crc64_ranges(buf, off, ln, 1, 2**64 - 1, 2**64 - 1, out)
        assert out[0] == c["crc64"], c


@pytest.mark.gpu
def test_gpu_xz_decode_fixtures(L):
    d = fixtures()
    for c in d["xz"]:
        data = data_of(d, c)
        cap = (c["dest_len"] if c["valid"] else 400000) + 64
        r, out, bad = L.XzDecode(data, cap)
        if c["valid"]:
            assert r == 0, (c["note"], r, bad, L.last_error())
            assert hashlib.sha256(out).hexdigest() == c["sha256"], c["note"]
        else:  # bad magic, corrupt LZMA2 data, check mismatch: the reference's exact code
            assert r == c["res"], (c["note"], r)
            assert out == b""
    # capacity short
    v = [c for c in d["xz"] if c["valid"] and c["dest_len"] > 0][0]
    r, out, _ = L.XzDecode(data_of(d, v), v["dest_len"] - 1)
    assert r == 7 and out == b""


@pytest.mark.gpu
def test_gpu_x86_convert_matches_reference(L):
    d = fixtures()
    for c in d["bcj"]:
        data = d["blob"][c["off"]:c["off"] + c["len"]]
        done, st, out = L.x86_Convert(data, c["ip"], c["state_in"], c["encoding"])
        assert (done, st) == (c["done"], c["state_out"]), c
        assert hashlib.sha256(out).hexdigest() == c["sha256"], c


@pytest.mark.gpu
def test_gpu_crc64_matches_reference(L):
    d = fixtures()
    for c in d["crc64"]:
        assert L.Crc64Calc(d["blob"][c["off"]:c["off"] + c["len"]]) == c["crc64"], c


@pytest.mark.gpu
def test_gpu_xz_many_blocks_round_trip(L):
    """A 512-block file (every check type across 4 concatenated streams, x86
    BCJ on one of them) decodes as one batch; output compared to the input."""
    import lzma
    import xzwrite as M
    parts, files = [], b""
    for s, chk in enumerate((1, 4, 10, 0)):
        blocks = [(native.gen("text", 7000 + 200 * s + i, 3000 + 131 * i),
                   {"x86": 0} if s == 1 else {}) for i in range(128)]
        files += M.make_stream(blocks, chk) + b"\0" * 4
        parts += [b for b, _ in blocks]
    plain = b"".join(parts)
    r, blocks, total = L.xz_index(files)
    assert r == 0 and len(blocks) == 512 and total == len(plain)
    r, out, bad = L.XzDecode(files, total)
    assert r == 0 and out == plain, (r, bad)
    # one flipped check byte in block 300 is reported there
    b = blocks[300]
    bad_file = bytearray(files)
    bad_file[b.check_off] ^= 1
    r, out, badb = L.XzDecode(bytes(bad_file), total)
    assert (r, badb) == (3, 300)


@pytest.mark.gpu
def test_gpu_bcj_x86_tiled_large_batch(L, emu):
    """BcjGpu_X86Batch (the tiled kernel: 4 KiB tiles, hit records, one lane's
    decisions) over 256 ranges x 40 KiB of branch-dense bytes at odd offsets,
    every start state, both directions -- against the lane-serial statement
    (itself pinned to the reference fixtures)."""
    import numpy as np
    import torch
    rng = np.random.default_rng(23)
    n, size = 256, 40000
    raw = rng.integers(0, 256, n * (size + 3) + 64, dtype=np.uint8)
    offs = np.array([i * (size + 3) + (i % 7) for i in range(n)], np.uint64)
    for i in range(n):
        o = int(offs[i])
        seg = raw[o:o + size]
        pick = rng.random(size) < (0.02 if i % 3 else 0.25)
        seg[pick] = rng.choice([0xE8, 0xE9], int(pick.sum()))
        ms = np.nonzero(pick)[0] + 4
        ms = ms[ms < size]
        seg[ms[rng.random(len(ms)) < 0.7]] = 0
    ips = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    st0 = (np.arange(n) % 8).astype(np.uint32)
    for enc in (0, 1):
        want = raw.copy()
        wst, wdone = [], []
        for i in range(n):
            o = int(offs[i])
            b = ctypes.create_string_buffer(want[o:o + size].tobytes() + b"\0" * 32, size + 32)
            s = ctypes.c_uint32(int(st0[i]))
            wdone.append(emu.emu_bcj_x86(b, size, int(ips[i]), ctypes.byref(s), enc))
            wst.append(s.value)
            want[o:o + size] = np.frombuffer(b.raw[:size], np.uint8)
        data = torch.from_numpy(raw.copy()).cuda()
        d_off = torch.from_numpy(offs.view(np.int64).copy()).cuda()
        d_len = torch.full((n,), size, dtype=torch.int64, device="cuda")
        d_ip = torch.from_numpy(ips.view(np.int32).copy()).cuda()
        d_st = torch.from_numpy(st0.view(np.int32).copy()).cuda()
        d_done = torch.zeros(n, dtype=torch.int64, device="cuda")
        assert L.bcj_x86_batch_device(data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(),
                                      d_ip.data_ptr(), d_st.data_ptr(), d_done.data_ptr(), n,
                                      enc) == 0
        torch.cuda.synchronize()
        assert d_done.cpu().tolist() == wdone
        assert (d_st.cpu().numpy().astype(np.uint32) == np.array(wst, np.uint32)).all()
        assert np.array_equal(data.cpu().numpy(), want)

"""RISC branch converters and the delta filter (beyond x86).

Reference: Bra.c (ARM_Convert :6, ARMT_Convert :33, PPC_Convert :68,
SPARC_Convert :99), BraIA64.c (IA64_Convert :14), Delta.c (Delta_Encode :20,
Delta_Decode :42), compiled in place and recorded in tests/golden/bra_cases.json
+ bra_blob.bin (tests/golden/make_golden_bra.py): ragged sizes, wrapping ips,
both directions, chained calls, delta 1..256 with carried state.

CPU (no GPU): the kernels' per-lane code (host build, tests/emu) against every
fixture.  GPU (-m gpu): the drop-ins (ARM_Convert ... Delta_Decode) against
every fixture, every fixture of a kind as one BraGpu_Batch / DeltaGpu_Batch
over unaligned device ranges, and a 512 x 64 KiB batch per kind against the
host build of the same code (itself pinned to the reference above).
"""
import ctypes
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

import native

GOLDEN = os.path.join(native.ROOT, "tests", "golden")
EMU_SO = os.path.join(native.ROOT, "tests", "emu", "liblane_emu.so")
KINDS = {"PPC": 5, "IA64": 6, "ARM": 7, "ARMT": 8, "SPARC": 9}


def fixtures():
    with open(os.path.join(GOLDEN, "bra_cases.json")) as f:
        d = json.load(f)
    with open(os.path.join(GOLDEN, "bra_blob.bin"), "rb") as f:
        blob = f.read()
    assert hashlib.sha256(blob).hexdigest() == d["blob_sha256"]
    d["blob"] = blob
    return d


def _get(d, off, n):
    return d["blob"][off:off + n]


@pytest.fixture(scope="module")
def emu():
    subprocess.run(["make", "-s", "-f", "tests/emu/Makefile"], cwd=native.ROOT, check=True)
    lib = ctypes.CDLL(EMU_SO)
    lib.emu_bra.restype = ctypes.c_uint64
    lib.emu_bra.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint32,
                            ctypes.c_int]
    lib.emu_delta.restype = None
    lib.emu_delta.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64,
                              ctypes.c_int]
    return lib


def test_fixture_coverage():
    d = fixtures()
    changed = {k: 0 for k in KINDS}
    for c in d["bra"]:
        if _get(d, c["in"], c["len"]) != _get(d, c["out"], c["len"]):
            changed[c["kind"]] += 1
    assert all(v >= 10 for v in changed.values()), changed
    assert len(d["delta"]) >= 100
    assert {c["delta"] for c in d["delta"]} >= {1, 2, 256}


def test_emu_bra_matches_reference(emu):
    d = fixtures()
    for c in d["bra"]:
        buf = ctypes.create_string_buffer(_get(d, c["in"], c["len"]), max(c["len"], 1))
        if "chain" in c:
            pos = 0
            for piece in c["chain"]:
                sub = ctypes.create_string_buffer(buf.raw[pos:pos + piece["len"]], max(piece["len"], 1))
                done = emu.emu_bra(c["id"], sub, piece["len"], c["ip"] + pos, 0)
                assert done == piece["done"], c["kind"]
                ctypes.memmove(ctypes.addressof(buf) + pos, sub, piece["len"])
                pos += done
            done = pos
        else:
            done = emu.emu_bra(c["id"], buf, c["len"], c["ip"], c["encoding"])
        assert done == c["done"], c
        assert buf.raw[:c["len"]] == _get(d, c["out"], c["len"]), c


def test_emu_armt_serial_statement_matches_reference(emu):
    """The lane-serial ARMT scan (bra_armt, Bra.c:33-66 as written) and the
    per-position kernel agree with the reference on every ARMT fixture."""
    d = fixtures()
    for c in d["bra"]:
        if c["kind"] != "ARMT" or "chain" in c:
            continue
        buf = ctypes.create_string_buffer(_get(d, c["in"], c["len"]), max(c["len"], 1))
        assert emu.emu_bra(0x108, buf, c["len"], c["ip"], c["encoding"]) == c["done"], c
        assert buf.raw[:c["len"]] == _get(d, c["out"], c["len"]), c


def test_emu_delta_matches_reference(emu):
    d = fixtures()
    for c in d["delta"]:
        st = ctypes.create_string_buffer(_get(d, c["state_in"], 256), 256)
        buf = ctypes.create_string_buffer(_get(d, c["in"], c["len"]), max(c["len"], 1))
        emu.emu_delta(st, c["delta"], buf, c["len"], c["encoding"])
        assert buf.raw[:c["len"]] == _get(d, c["out"], c["len"]), c
        assert st.raw == _get(d, c["state_out"], 256), c
        # the tile scan's head: the same case at every start alignment mod 16
        for shift in (1, 5, 15):
            st = ctypes.create_string_buffer(_get(d, c["state_in"], 256), 256)
            big = ctypes.create_string_buffer(b"\0" * shift + _get(d, c["in"], c["len"]),
                                              shift + max(c["len"], 1))
            emu.emu_delta(st, c["delta"], ctypes.byref(big, shift), c["len"], c["encoding"])
            assert big.raw[shift:shift + c["len"]] == _get(d, c["out"], c["len"]), (c, shift)
            assert st.raw == _get(d, c["state_out"], 256), (c, shift)


def test_batch_entry_points_exported():
    import lzmagpu
    for name in ("ARM_Convert", "ARMT_Convert", "PPC_Convert", "SPARC_Convert", "IA64_Convert",
                 "Delta_Init", "Delta_Encode", "Delta_Decode", "BraGpu_Batch", "DeltaGpu_Batch"):
        assert name in lzmagpu.EXPORTED


# ---------------------------------------------------------------- GPU

@pytest.fixture(scope="module")
def L():
    # torch's HIP context first: the batch tests hand torch allocations to the library
    import torch
    torch.zeros(1, device="cuda")
    import lzmagpu
    return lzmagpu


@pytest.mark.gpu
def test_gpu_dropins_match_reference(L):
    d = fixtures()
    for c in d["bra"]:
        data = _get(d, c["in"], c["len"])
        if "chain" in c:
            buf, pos = bytearray(data), 0
            for piece in c["chain"]:
                done, out = L.bra_convert(c["kind"], bytes(buf[pos:pos + piece["len"]]), c["ip"] + pos, 0)
                assert done == piece["done"], c["kind"]
                buf[pos:pos + piece["len"]] = out
                pos += done
            done, out = pos, bytes(buf)
        else:
            done, out = L.bra_convert(c["kind"], data, c["ip"], c["encoding"])
        assert done == c["done"], c
        assert out == _get(d, c["out"], c["len"]), c
    for c in d["delta"]:
        st, out = L.delta_convert(_get(d, c["in"], c["len"]), c["delta"],
                                  _get(d, c["state_in"], 256), c["encoding"])
        assert out == _get(d, c["out"], c["len"]), c
        assert st == _get(d, c["state_out"], 256), c


def _dev(torch, arr):
    return torch.from_numpy(np.array(arr, copy=True)).cuda()


@pytest.mark.gpu
def test_gpu_bra_batch_fixtures(L):
    import torch
    d = fixtures()
    for kind, kid in KINDS.items():
        for enc in (0, 1):
            cases = [c for c in d["bra"] if c["kind"] == kind and c["encoding"] == enc
                     and "chain" not in c]
            # ranges at odd offsets: the kernels make no alignment assumption
            offs, blob = [], bytearray()
            for c in cases:
                blob += b"\x5a" * (1 + len(offs) % 3)
                offs.append(len(blob))
                blob += _get(d, c["in"], c["len"])
            data = _dev(torch, np.frombuffer(bytes(blob) + b"\0", np.uint8))
            off = _dev(torch, np.array(offs, np.uint64).view(np.int64))
            ln = _dev(torch, np.array([c["len"] for c in cases], np.uint64).view(np.int64))
            ip = _dev(torch, np.array([c["ip"] for c in cases], np.uint32).view(np.int32))
            done = torch.zeros(len(cases), dtype=torch.int64, device="cuda")
            assert L.bra_batch_device(kid, data.data_ptr(), off.data_ptr(), ln.data_ptr(),
                                      ip.data_ptr(), done.data_ptr(), len(cases), enc) == 0
            torch.cuda.synchronize()
            out = data.cpu().numpy().tobytes()
            got = done.cpu().tolist()
            for c, o, dn in zip(cases, offs, got):
                assert dn == c["done"], c
                assert out[o:o + c["len"]] == _get(d, c["out"], c["len"]), c
    rc = L.bra_batch_device(4, 0, 0, 0, 0, 0, 1, 0)  # x86 is BcjGpu_X86Batch, not this entry
    assert rc == 4


@pytest.mark.gpu
def test_gpu_delta_batch_fixtures(L):
    import torch
    d = fixtures()
    cases = d["delta"]
    offs, blob = [], bytearray()
    for c in cases:
        blob += b"\x11"
        offs.append(len(blob))
        blob += _get(d, c["in"], c["len"])
    for enc in (0, 1):
        sel = [i for i, c in enumerate(cases) if c["encoding"] == enc]
        data = _dev(torch, np.frombuffer(bytes(blob) + b"\0", np.uint8))
        off = _dev(torch, np.array([offs[i] for i in sel], np.uint64).view(np.int64))
        ln = _dev(torch, np.array([cases[i]["len"] for i in sel], np.uint64).view(np.int64))
        dl = _dev(torch, np.array([cases[i]["delta"] for i in sel], np.uint32).view(np.int32))
        st = _dev(torch, np.frombuffer(b"".join(_get(d, cases[i]["state_in"], 256) for i in sel), np.uint8))
        assert L.delta_batch_device(data.data_ptr(), off.data_ptr(), ln.data_ptr(), dl.data_ptr(),
                                    st.data_ptr(), len(sel), enc) == 0
        torch.cuda.synchronize()
        out, sto = data.cpu().numpy().tobytes(), st.cpu().numpy().tobytes()
        for j, i in enumerate(sel):
            c = cases[i]
            assert out[offs[i]:offs[i] + c["len"]] == _get(d, c["out"], c["len"]), c
            assert sto[256 * j:256 * j + 256] == _get(d, c["state_out"], 256), c


@pytest.mark.gpu
def test_gpu_bra_large_batch_matches_host_build(L, emu):
    """512 x 64 KiB ranges per kind (32 MiB), branch patterns stamped densely."""
    import torch
    n, size = 512, 65536
    rng = np.random.default_rng(7)
    for kind, kid in KINDS.items():
        raw = rng.integers(0, 256, n * size, dtype=np.uint8)
        w = raw.reshape(-1, 4)
        pick = rng.random(len(w)) < 0.4
        if kind == "ARM":
            w[pick, 3] = 0xEB
        elif kind == "ARMT":
            w[pick, 1] = 0xF0 | (w[pick, 1] & 7)
            w[pick, 3] = 0xF8 | (w[pick, 3] & 7)
        elif kind == "PPC":
            w[pick, 0] = 0x48 | (w[pick, 0] & 3)
            w[pick, 3] = (w[pick, 3] & 0xFC) | 1
        elif kind == "SPARC":
            w[pick, 0] = 0x40
            w[pick, 1] &= 0x3F
        else:
            b = raw.reshape(-1, 16)
            b[:, 0] = (b[:, 0] & 0xE0) | 16
        ips = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
        want = raw.copy()
        dones = []
        for i in range(n):
            seg = ctypes.create_string_buffer(want[i * size:(i + 1) * size].tobytes(), size)
            dones.append(emu.emu_bra(kid, seg, size, int(ips[i]), 0))
            want[i * size:(i + 1) * size] = np.frombuffer(seg.raw, np.uint8)
        data = _dev(torch, raw)
        off = _dev(torch, (np.arange(n, dtype=np.uint64) * size).view(np.int64))
        ln = _dev(torch, np.full(n, size, np.uint64).view(np.int64))
        ip = _dev(torch, ips.view(np.int32))
        done = torch.zeros(n, dtype=torch.int64, device="cuda")
        assert L.bra_batch_device(kid, data.data_ptr(), off.data_ptr(), ln.data_ptr(),
                                  ip.data_ptr(), done.data_ptr(), n, 0) == 0
        torch.cuda.synchronize()
        assert done.cpu().tolist() == dones, kind
        got = data.cpu().numpy()
        assert (got != raw).any(), kind
        assert np.array_equal(got, want), kind


def _delta_decode_np(data, d, state):
    """Delta.c Delta_Decode (Delta.c:42-62) restated with numpy: residue r of the
    output is its state byte plus the running sum of its input bytes (mod 256);
    the new state holds the last d output bytes, oldest first."""
    out = np.empty_like(data)
    n = len(data)
    st = np.frombuffer(state, np.uint8)
    hist = np.concatenate([st[:d], np.zeros(0, np.uint8)])
    for r in range(d):
        seq = data[r::d].astype(np.uint64)
        out[r::d] = ((np.cumsum(seq) + int(hist[r])) & 0xFF).astype(np.uint8)
    new = np.concatenate([st[:d], out])[-d:] if n else st[:d]
    full = np.frombuffer(state, np.uint8).copy()
    full[:d] = new
    return out, full.tobytes()


@pytest.mark.gpu
def test_gpu_delta_large_batch_vs_numpy(L):
    """512 x 64 KiB ranges (the tile scan over 16 tiles, the segmented scan), d in
    {1, 2, 4, 8, 16, 3, 255, 32}, range starts at every residue mod 16, random
    states -- against numpy's per-residue running sums, not the kernel's own host
    build.  Ranges with d = 0 and d = 300 are left untouched (and the call returns)."""
    import torch
    n, size = 512, 65536
    rng = np.random.default_rng(11)
    ds = [1, 2, 4, 8, 16, 3, 255, 32]
    offs, pos = [], 0
    for i in range(n):
        pos += 1 + (i % 16)
        offs.append(pos)
        pos += size
    raw = rng.integers(0, 256, pos + 64, dtype=np.uint8)
    dl = np.array([ds[i % len(ds)] for i in range(n)], np.uint32)
    dl[100], dl[200] = 0, 300
    states = rng.integers(0, 256, 256 * n, dtype=np.uint8)
    data = _dev(torch, raw)
    off = _dev(torch, np.array(offs, np.uint64).view(np.int64))
    ln = _dev(torch, np.full(n, size, np.uint64).view(np.int64))
    dd = _dev(torch, dl.view(np.int32))
    st = _dev(torch, states)
    assert L.delta_batch_device(data.data_ptr(), off.data_ptr(), ln.data_ptr(), dd.data_ptr(),
                                st.data_ptr(), n, 0) == 0
    torch.cuda.synchronize()
    got, sto = data.cpu().numpy(), st.cpu().numpy()
    for i in range(n):
        o = offs[i]
        s_in = states[256 * i:256 * i + 256].tobytes()
        if dl[i] in (0, 300):
            assert np.array_equal(got[o:o + size], raw[o:o + size]), i
            assert sto[256 * i:256 * i + 256].tobytes() == s_in, i
            continue
        want, want_st = _delta_decode_np(raw[o:o + size], int(dl[i]), s_in)
        assert np.array_equal(got[o:o + size], want), (i, dl[i], o % 16)
        assert sto[256 * i:256 * i + 256].tobytes() == want_st, (i, dl[i])


def test_numpy_delta_restatement_matches_reference():
    """The numpy Delta_Decode the large GPU test checks against is pinned to every
    reference-decoded delta fixture (d = 1 .. 256, including 8 and 32)."""
    d = fixtures()
    seen = set()
    for c in d["delta"]:
        if c["encoding"]:
            continue
        out, st = _delta_decode_np(np.frombuffer(_get(d, c["in"], c["len"]), np.uint8),
                                   c["delta"], _get(d, c["state_in"], 256))
        assert out.tobytes() == _get(d, c["out"], c["len"]), c
        assert st == _get(d, c["state_out"], 256), c
        seen.add(c["delta"])
    assert {8, 32} <= seen

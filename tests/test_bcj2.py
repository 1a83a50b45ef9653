"""BCJ2, the four-stream x86 branch decoder of 7z (Bcj2.c:28-128; SURVEY.md
8(f) row 4).

Reference: Bcj2_Decode compiled in place (oracle/_ref/libref.so) over streams
from tests/bcj2enc.py, recorded in tests/golden/bcj2_cases.json +
bcj2_blob.bin (tests/golden/make_golden_bcj2.py): the return value and the
SHA-256 of the whole output buffer (prefilled with 0xA5) for exact, clipped
and overlong outputs, truncated / corrupted rc, CALL and JMP streams, and the
7zDec layout with the main stream in the output's tail.

CPU: the kernel's lane code (bcj2_device.h, host build) on every case; the
encoder round-trips.  GPU (-m gpu): the Bcj2_Decode drop-in on every case, and
all cases as one Bcj2Gpu_Batch launch.
"""
import ctypes
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

import bcj2enc
import native

GOLDEN = os.path.join(native.ROOT, "tests", "golden")
EMU_SO = os.path.join(native.ROOT, "tests", "emu", "liblane_emu.so")


def fixtures():
    with open(os.path.join(GOLDEN, "bcj2_cases.json")) as f:
        d = json.load(f)
    with open(os.path.join(GOLDEN, "bcj2_blob.bin"), "rb") as f:
        blob = f.read()
    assert hashlib.sha256(blob).hexdigest() == d["blob_sha256"]
    d["blob"] = blob
    return d


def streams(d, c):
    return [d["blob"][o:o + n] for o, n in c["streams"]]


def sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.fixture(scope="module")
def emu():
    subprocess.run(["make", "-s", "-f", "tests/emu/Makefile"], cwd=native.ROOT, check=True)
    lib = ctypes.CDLL(EMU_SO)
    lib.emu_bcj2.restype = ctypes.c_int
    lib.emu_bcj2.argtypes = [ctypes.c_void_p, ctypes.c_uint64] * 4 + [ctypes.c_void_p,
                                                                      ctypes.c_uint64]
    return lib


def _emu_run(emu, d, c):
    m, cl, jp, rc = streams(d, c)
    n = c["out_size"]
    out = ctypes.create_string_buffer(bytes([d["fill"]]) * max(n, 1), max(n, 1))
    keep = [ctypes.create_string_buffer(x, max(len(x), 1)) for x in (cl, jp, rc)]
    if c["overlap"]:
        at = n - len(m)
        ctypes.memmove(ctypes.addressof(out) + at, m, len(m))
        mp = ctypes.addressof(out) + at
    else:
        mb = ctypes.create_string_buffer(m, max(len(m), 1))
        keep.append(mb)
        mp = ctypes.addressof(mb)
    r = emu.emu_bcj2(mp, len(m), ctypes.addressof(keep[0]), len(cl), ctypes.addressof(keep[1]),
                     len(jp), ctypes.addressof(keep[2]), len(rc), ctypes.addressof(out), n)
    return r, out.raw[:n]


def test_fixture_coverage():
    d = fixtures()
    res = [c["res"] for c in d["cases"]]
    assert len(res) >= 150 and res.count(0) >= 40 and res.count(1) >= 40
    assert any(c["overlap"] for c in d["cases"])


def test_encoder_round_trip_through_reference_cases():
    """The fixture streams that the reference decoded OK at the full size are
    this encoder's output; re-encoding the synthetic input reproduces them."""
    data = bcj2enc.x86_like(5, 4096, density=0.04 + 0.02 * (5 % 3))
    m, c, j, r = bcj2enc.encode(data)
    d = fixtures()
    case = next(x for x in d["cases"] if x["note"] == "n=4096 by target")
    assert streams(d, case) == [m, c, j, r] and case["res"] == 0


def test_emu_matches_reference(emu):
    d = fixtures()
    for c in d["cases"]:
        r, out = _emu_run(emu, d, c)
        assert r == c["res"], (c["note"], r)
        assert sha(out) == c["out_sha256"], c["note"]


@pytest.fixture(scope="module")
def L():
    import torch
    torch.zeros(1, device="cuda")
    import lzmagpu
    return lzmagpu


@pytest.mark.gpu
def test_gpu_bcj2_dropin_matches_reference(L):
    d = fixtures()
    for c in d["cases"]:
        m, cl, jp, rc = streams(d, c)
        r, out = L.Bcj2_Decode(m, cl, jp, rc, c["out_size"], overlap=c["overlap"], fill=d["fill"])
        assert r == c["res"], (c["note"], r, L.last_error())
        assert sha(out) == c["out_sha256"], c["note"]


@pytest.mark.gpu
def test_gpu_bcj2_batch_matches_reference(L):
    """Every case as one lane of ONE Bcj2Gpu_Batch launch, streams packed at
    odd offsets in one device buffer, main streams of the overlap cases in
    their output's tail."""
    import torch
    d = fixtures()
    cs = d["cases"]
    layout, pos = [], 0
    host = bytearray()

    def place(b):
        nonlocal pos
        host.extend(b"\x33" * (1 + len(host) % 5))
        at = len(host)
        host.extend(b)
        return at

    outs = []
    for c in cs:
        m, cl, jp, rc = streams(d, c)
        n = c["out_size"]
        o = place(bytes([d["fill"]]) * n)
        outs.append(o)
        if c["overlap"]:
            host[o + n - len(m):o + n] = m
            m_at = o + n - len(m)
        else:
            m_at = place(m)
        layout.append((m_at, place(cl), place(jp), place(rc)))
    buf = torch.from_numpy(np.frombuffer(bytes(host) + b"\0" * 16, np.uint8).copy()).cuda()
    base = buf.data_ptr()
    jobs = (L.Bcj2Job * len(cs))()
    for k, c in enumerate(cs):
        sizes = [n for _, n in c["streams"]]
        jobs[k].buf0, jobs[k].buf1, jobs[k].buf2, jobs[k].buf3 = [base + a for a in layout[k]]
        jobs[k].size0, jobs[k].size1, jobs[k].size2, jobs[k].size3 = sizes
        jobs[k].out, jobs[k].out_size = base + outs[k], c["out_size"]
    d_jobs = torch.frombuffer(bytearray(bytes(jobs)), dtype=torch.uint8).cuda()
    d_res = torch.full((len(cs),), -7, dtype=torch.int32, device="cuda")
    assert L.bcj2_batch_device(d_jobs.data_ptr(), len(cs), d_res.data_ptr()) == 0
    torch.cuda.synchronize()
    res = d_res.cpu().tolist()
    got = buf.cpu().numpy().tobytes()
    for k, c in enumerate(cs):
        assert res[k] == c["res"], (c["note"], res[k])
        assert sha(got[outs[k]:outs[k] + c["out_size"]]) == c["out_sha256"], c["note"]

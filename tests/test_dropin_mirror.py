"""The drop-in dictionary interface on its device mirror (dropin_capi.hip):
LzmaDec_DecodeToDic / LzmaDec_DecodeToBuf over host CLzmaDec objects keep the
dictionary, the table and the state on the GPU between calls.

* parity: the 7zDec.c:127-171 loop (16 KiB look windows over a dictionary that
  is the whole 2 MiB output) and the fork's DecodeToBuf loop equal the
  oracle's, call by call; dropping the mirror mid-stream
  (LzmaGpu_DecoderRelease: the next call rebuilds it from the host copy, history
  included) and interleaving two decoders on one thread change nothing;
* traffic: the dictionary loop uploads its input windows plus a fixed few
  hundred bytes per call -- not the dictionary (round 2 uploaded dicBufSize
  per call: 2 MiB x 130 calls here) -- measured with
  LzmaGpu_DropinTransferStats.
"""
import lzma
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "lzma-sdk-zliblike_amd"))
sys.path.insert(0, HERE)

import native  # noqa: E402
import workloads as W  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    import lzmagpu
    if lzmagpu.device_count() <= 0:
        pytest.fail("no HIP device visible: " + lzmagpu.last_error())
    return lzmagpu


def _stream(seed, n, dsz=1 << 16, lc=3, lp=0, pb=2):
    data = native.gen("text", seed, n)
    comp = lzma.compress(data, format=lzma.FORMAT_RAW, filters=[
        {"id": lzma.FILTER_LZMA1, "dict_size": dsz, "lc": lc, "lp": lp, "pb": pb}])
    return data, comp, W.props_bytes(lc, lp, pb, dsz)


def test_dic_loop_uploads_windows_not_the_dictionary(L):
    n, win = 2 << 20, 1 << 14
    data, comp, props = _stream(880001, n)
    want = native.dic_decode(native.oracle(), "orc", comp, props, n, win)
    L.transfer_stats(reset=True)
    calls, trace, out, used = L.dic_decode(comp, props, n, win)
    h2d, d2h, ncalls = L.transfer_stats(reset=True)
    assert [tuple(t) for t in trace] == [tuple(t) for t in want[1]]
    assert out == data == want[2] and used == want[3]
    assert ncalls == calls
    table = 2 * (56 * 4 + 950 + (768 << 3))  # the lc3/pb2 compact table, uploaded once
    assert h2d <= len(comp) + 20 * calls + 256 * calls + table, (h2d, len(comp), calls)
    assert h2d < len(comp) + n // 8  # the dictionary itself is never uploaded
    assert d2h <= n + calls * (256 + table), (d2h, n, calls)


def test_dic_loop_survives_mirror_release_mid_stream(L):
    """Every 7th call drops the decoder's mirror: the next call starts from the
    host copy (history uploaded once) and the trace is unchanged."""
    n, win = 1 << 20, 1 << 14
    data, comp, props = _stream(880002, n)
    want = native.dic_decode(native.oracle(), "orc", comp, props, n, win)
    import ctypes

    def drop(k, dec):
        if k % 7 == 6:
            L.lib.LzmaGpu_DecoderRelease(ctypes.byref(dec))

    calls, trace, out, used = L.dic_decode(comp, props, n, win, between=drop)
    assert [tuple(t) for t in trace] == [tuple(t) for t in want[1]]
    assert out == data


def test_two_decoders_interleaved_on_one_thread(L):
    """Two CLzmaDec objects advanced alternately (two mirrors side by side)."""
    import ctypes
    streams = [_stream(880003 + k, 600_000, lc=k, lp=0, pb=2 - k) for k in range(2)]
    decs, bufs, pos, done = [], [], [0, 0], [False, False]
    for data, comp, props in streams:
        d = L.CLzmaDec()
        d.dic = None
        d.probs = None
        assert L.lib.LzmaDec_AllocateProbs(ctypes.byref(d), props, 5, ctypes.byref(L.g_alloc)) == 0
        b = ctypes.create_string_buffer(len(data))
        d.dic = ctypes.addressof(b)
        d.dicBufSize = len(data)
        L.lib.LzmaDec_Init(ctypes.byref(d))
        decs.append(d)
        bufs.append(b)
    srcs = [ctypes.create_string_buffer(c, len(c)) for _, c, _ in streams]
    try:
        while not all(done):
            for k in range(2):
                if done[k]:
                    continue
                comp = streams[k][1]
                sl = ctypes.c_size_t(min(len(comp) - pos[k], 10000))
                st = ctypes.c_int(-1)
                r = L.lib.LzmaDec_DecodeToDic(ctypes.byref(decs[k]), len(streams[k][0]),
                                              ctypes.addressof(srcs[k]) + pos[k], ctypes.byref(sl),
                                              1, ctypes.byref(st))
                assert r == 0, (k, r, L.last_error())
                pos[k] += sl.value
                if decs[k].dicPos == len(streams[k][0]):
                    done[k] = True
        for k in range(2):
            assert bufs[k].raw == streams[k][0]
    finally:
        for d in decs:
            L.lib.LzmaDec_FreeProbs(ctypes.byref(d), ctypes.byref(L.g_alloc))


def test_decode_to_buf_one_launch_per_call(L):
    """The fork's loop (512 KiB in, 1 MiB out per call) over a 64 KiB ring: each
    call is one launch (the ring loop runs on the device), output and per-call
    results equal the oracle's, and the call uploads only its input window."""
    n = 3 << 20
    data, comp, props = _stream(880005, n)
    want = native.stream_decode(native.oracle(), "orc", comp, props, n, 1 << 19, 1 << 20, 0)
    L.transfer_stats(reset=True)
    calls, trace, out, used = L.stream_decode(comp, props, n, 1 << 19, 1 << 20, 0)
    h2d, d2h, ncalls = L.transfer_stats(reset=True)
    assert trace == want[1] and out == data
    assert ncalls == calls
    assert h2d <= sum(min(1 << 19, len(comp) - sum(x[2] for x in trace[:i]))
                      for i in range(len(trace))) + calls * 256 + 16384


# ---------------------------------------------------------------- rings, host edits
# Driven through the GPU library and through the reference's own LzmaDec.c
# (oracle/_ref/libref_lzma.so, compiled in place) with the same host-side
# actions; both must agree call by call.
needs_ref = pytest.mark.skipif(not native.have_ref(), reason="oracle/_ref/libref_lzma.so not built")


@needs_ref
def test_ring_smaller_than_window_reads_the_ring_slot(L):
    """A caller-owned ring (LzmaDec_AllocateProbs + a 4 KiB dic) smaller than
    the dictionary size (64 KiB) and the session kernel's LDS window (up to
    128 KiB): matches at distance 5,096 read the ring slot the reference reads
    (dicPos - rep0 + dicBufSize: the byte 1,000 back), not the true history byte
    the window would still hold -- the window serves distances up to
    min(window, dicBufSize) only.  Hand-made streams (tests/lzmaenc_min.py)
    keep every such read inside the ring."""
    import lzmaenc_min as E
    ref = native.ref()
    for seed in (1, 2, 3):
        comp, props, out = E.ring_reach_stream(seed)
        for in_chunk, out_chunk in ((1 << 30, 3000), (700, 1000), (1 << 30, 1 << 30)):
            want = E.ring_decode(ref, comp, props, 4096, len(out), in_chunk, out_chunk)
            assert want[1] == out
            got = E.ring_decode(L.lib, comp, props, 4096, len(out), in_chunk, out_chunk)
            assert got == want, (seed, in_chunk, out_chunk, got[0][-3:], want[0][-3:])


@needs_ref
def test_host_edits_between_calls_match_the_reference(L):
    """Host-side changes between DecodeToDic calls reach the device mirror:
    every probability cell reset to 1024 by the host (the table hash check),
    dicPos moved back (not a pure advance: the history is dropped and the whole
    dictionary re-uploaded), and both at once; output and per-call results equal
    the reference's LzmaDec.c given the same edits."""
    import ctypes
    import lzmaenc_min as E
    ref = native.ref()
    n = 300_000
    data, comp, props = _stream(880011, n)

    def reset_probs(k, d):
        if k == 3:
            cells = (ctypes.c_uint16 * d.numProbs).from_address(d.probs)
            for i in range(d.numProbs):
                cells[i] = 1024

    def move_back(k, d):
        if k == 4:
            d.dicPos = d.dicPos - 1000

    def both(k, d):
        reset_probs(k, d)
        move_back(k, d)

    for edit in (None, reset_probs, move_back, both):
        want = E.dic_calls(ref, comp, props, n, 9000, edit)
        got = E.dic_calls(L.lib, comp, props, n, 9000, edit)
        assert got[0] == want[0], (edit, got[0][-3:], want[0][-3:])
        # the dictionary up to the final dicPos (after SZ_ERROR_DATA the
        # reference also leaves the failed pass's bytes beyond dicPos in dic,
        # LzmaDec.c:366-379 returning before the write-back; the drop-in
        # returns dic[0, dicPos) -- the documented difference in
        # include/lzma_gpu.h's header comment, INTEGRATION.md and DESIGN.md §2)
        end = want[0][-1][3]
        assert got[1][:end] == want[1][:end], edit
        if edit is None:
            assert want[1] == data and end == n


def test_decoder_alternating_devices(L):
    """A decoder used on one device, then another, then the first again decodes
    on current state (its mirrors on the other devices are dropped)."""
    import ctypes
    if L.device_count() < 2:
        pytest.skip("one visible device: the alternating-device case needs two")
    n, win = 1 << 19, 1 << 14
    data, comp, props = _stream(880012, n)
    want = native.dic_decode(native.oracle(), "orc", comp, props, n, win)

    hip = ctypes.CDLL("libamdhip64.so")

    def hop(k, dec):  # the next call runs on the other device
        assert hip.hipSetDevice((k + 1) % 2) == 0

    try:
        calls, trace, out, used = L.dic_decode(comp, props, n, win, between=hop)
    finally:
        hip.hipSetDevice(0)
    assert [tuple(t) for t in trace] == [tuple(t) for t in want[1]]
    assert out == data

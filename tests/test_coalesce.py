"""Concurrent one-call decodes share launches (VERDICT r03 item 6b,
dropin_capi.hip's coalescer): LzmaDecode / LzmaUncompress / Lzma2Decode calls
made by several host threads at once run as batch launches -- calls arriving
while a batch runs form the next one -- and every caller still gets exactly
its own LzmaDecode results (LzmaDec.c:972-1002, LzmaLib.c:41-46).

GPU: 400 calls from 48 Python threads (ctypes drops the GIL) over mixed
lc/lp/pb streams, corrupt and truncated ones, both finish modes and LZMA2
items, each checked against the oracle; the coalescer's counters show batches
of more than one call.  The same for the dictionary interface: threads each
running the fork's DecodeToBuf loop on their own decoder share session
launches.  The unchanged multi-threaded C caller
(tests/c_host/lzma_c_threads.c) linked to the library agrees with the same
source linked to the reference's LzmaDec.c, stream by stream (CRCs)."""
import lzma
import os
import random
import zlib
from concurrent.futures import ThreadPoolExecutor

import pytest

import native
import test_c_host as TC
import workloads as W


def _cases(n=400, seed=4242):
    rng = random.Random(seed)
    out = []
    for i in range(n):
        if i % 10 == 9:  # an LZMA2 item through Lzma2Decode
            data = native.gen("text", 91_000 + i, rng.choice([1000, 9000, 40000]))
            comp = lzma.compress(data, format=lzma.FORMAT_RAW,
                                 filters=[{"id": lzma.FILTER_LZMA2, "dict_size": 1 << 16}])
            out.append(("lzma2", comp, 16, len(data) + rng.choice([0, 0, 5]), 1))
            continue
        lc = rng.randrange(5)
        lp = rng.randrange(5 - lc)
        pb = rng.randrange(5)
        dsz = rng.choice([4096, 1 << 16])
        data = native.gen(rng.choice(["text", "random"]), 90_000 + i,
                          rng.choice([0, 100, 4096, 20000]))
        comp = bytearray(lzma.compress(data, format=lzma.FORMAT_RAW, filters=[
            {"id": lzma.FILTER_LZMA1, "dict_size": dsz, "lc": lc, "lp": lp, "pb": pb}]))
        if i % 7 == 3 and len(comp) > 8:
            comp[rng.randrange(5, len(comp))] ^= 0x21
        if i % 11 == 5:
            comp = comp[:rng.randrange(len(comp) + 1)]
        out.append(("lzma", bytes(comp), W.props_bytes(lc, lp, pb, dsz),
                    len(data) + rng.choice([0, 0, 3]), rng.randrange(2)))
    return out


def test_coalesce_case_mix_is_varied():
    kinds = {c[0] for c in _cases()}
    assert kinds == {"lzma", "lzma2"}


@pytest.mark.gpu
def test_gpu_concurrent_calls_coalesce_and_match_oracle():
    import lzmagpu as L
    orc = native.oracle()
    cases = _cases()
    want = []
    for kind, comp, props, cap, fin in cases:
        if kind == "lzma":
            want.append(native.decode(orc, "orc", comp, props, cap, fin))
        else:
            want.append(native.lzma2_decode(orc, "orc", comp, props, cap, fin))

    def call(k):
        kind, comp, props, cap, fin = cases[k]
        if kind == "lzma":
            return L.LzmaDecode(comp, props, cap, fin)
        return L.Lzma2Decode(comp, props, cap, fin)

    L.coalesce_stats(reset=True)
    with ThreadPoolExecutor(48) as ex:
        got = list(ex.map(call, range(len(cases))))
    batches, calls, biggest = L.coalesce_stats()
    bad = []
    for k, (g, w) in enumerate(zip(got, want)):
        res, st, dl, sl, out = g
        wres, wst, wdl, wsl, wout = w
        if (res, dl, sl) != (wres, wdl, wsl) or out != wout or (res == 0 and st != wst):
            bad.append((k, cases[k][0], (res, st, dl, sl), (wres, wst, wdl, wsl)))
    assert not bad, bad[:5]
    # every call reaches the device except LzmaDecode's own early exit on fewer
    # than 5 input bytes (SZ_ERROR_INPUT_EOF before any decode, LzmaDec.c:980)
    reach = sum(1 for c in cases if c[0] == "lzma2" or len(c[1]) >= 5)
    assert calls == reach and batches < calls and biggest > 1, (batches, calls, biggest, reach)


@pytest.mark.gpu
def test_gpu_c_threads_caller_matches_reference_build(tmp_path):
    if not os.path.exists(TC.THREADS_BIN):
        TC.build_c_threads()
    plain, comp, lens, props = W.uniform_batch(600, 4096, 0, 0, 0, 4096)
    offs = [0]
    for ln in lens:
        offs.append(offs[-1] + int(ln))
    comps = [comp[offs[i]:offs[i + 1]].tobytes() for i in range(600)]
    f = TC.write_stream_set(str(tmp_path), comps, [props] * 600, [4096] * 600)
    want = 0
    for i in range(600):
        want ^= zlib.crc32(plain[i * 4096:(i + 1) * 4096].tobytes(), i)
    for mode in ("one", "buf"):
        for threads in (1, 16, 64):
            d = TC.run_c_threads(TC.THREADS_BIN, threads, f, mode=mode)
            assert d["fails"] == 0 and d["crc_xor"] == "%08x" % want, d
            if threads > 1:
                assert d["max_batch"] > 1, d
        if os.path.exists(TC.THREADS_REF):
            d = TC.run_c_threads(TC.THREADS_REF, 16, f, mode=mode)
            assert d["fails"] == 0 and d["crc_xor"] == "%08x" % want, d


@pytest.mark.gpu
@pytest.mark.parametrize("inflight,coalesce", [("1", "1"), ("8", "1"), ("4", "0")])
def test_gpu_c_threads_every_in_flight_setting(tmp_path, inflight, coalesce):
    """The group-commit variants (dropin_capi.hip group_commit): one batch set,
    the most sets, and coalescing off (one launch per call), for both one-call
    and DecodeToBuf callers: every stream's CRC equals the plain data's, and
    with coalescing on concurrent callers share launches."""
    if not os.path.exists(TC.THREADS_BIN):
        TC.build_c_threads()
    plain, comp, lens, props = W.uniform_batch(300, 4096, 0, 0, 0, 4096, first=5000)
    offs = [0]
    for ln in lens:
        offs.append(offs[-1] + int(ln))
    comps = [comp[offs[i]:offs[i + 1]].tobytes() for i in range(300)]
    f = TC.write_stream_set(str(tmp_path), comps, [props] * 300, [4096] * 300)
    want = 0
    for i in range(300):
        want ^= zlib.crc32(plain[i * 4096:(i + 1) * 4096].tobytes(), i)
    env = dict(os.environ, LZGPU_COALESCE_INFLIGHT=inflight, LZGPU_COALESCE=coalesce)
    for mode in ("one", "buf"):
        for threads in (5, 48):
            d = TC.run_c_threads(TC.THREADS_BIN, threads, f, env=env, mode=mode)
            assert d["fails"] == 0 and d["crc_xor"] == "%08x" % want, (mode, threads, d)
            if coalesce == "1" and threads == 48:
                assert d["max_batch"] > 1, d
            if coalesce == "0":
                assert d["max_batch"] == 1, d


@pytest.mark.gpu
@pytest.mark.parametrize("inflight,faults", [("1", "1"), ("4", "2"), ("2", "5")])
def test_gpu_stream_creation_failures_never_hang(tmp_path, inflight, faults):
    """ADVICE r05 (dropin_capi.hip group_commit): a batch set whose stream
    cannot be created is left out and the call tries another set; when no set
    is left and no batch runs, the call and every pending one fail at once
    (SZ_ERROR_FAIL), and later calls create the streams again.  Fault
    injection: LZGPU_FAULT_STREAM_CREATE=N fails the process's first N stream
    creations.  48 threads, one-call and DecodeToBuf callers: the program
    ends (no caller sleeps forever), every stream that decoded has the plain
    data's CRC, and with a set left over nothing fails at all."""
    if not os.path.exists(TC.THREADS_BIN):
        TC.build_c_threads()
    n = 240
    plain, comp, lens, props = W.uniform_batch(n, 4096, 0, 0, 0, 4096, first=9000)
    offs = [0]
    for ln in lens:
        offs.append(offs[-1] + int(ln))
    comps = [comp[offs[i]:offs[i + 1]].tobytes() for i in range(n)]
    f = TC.write_stream_set(str(tmp_path), comps, [props] * n, [4096] * n)
    want = 0
    for i in range(n):
        want ^= zlib.crc32(plain[i * 4096:(i + 1) * 4096].tobytes(), i)
    env = dict(os.environ, LZGPU_COALESCE_INFLIGHT=inflight, LZGPU_FAULT_STREAM_CREATE=faults)
    for mode in ("one", "buf"):
        d = TC.run_c_threads(TC.THREADS_BIN, 48, f, env=env, mode=mode, timeout=120)
        if int(faults) < int(inflight):
            assert d["fails"] == 0 and d["crc_xor"] == "%08x" % want, (mode, d)
        else:
            # every set failed once: the calls of that moment fail, the rest decode
            assert 0 < d["fails"] < n, (mode, d)


@pytest.mark.gpu
def test_gpu_oversized_call_runs_beside_small_ones():
    """a call whose input + capacity exceed the coalescer's item
    limit (dropin_capi.hip kCoalesceItemMax, 256 MiB) runs in a batch of its
    own, so its footprint neither sets nor fails the small calls' batch; every
    call still returns exactly what the oracle does."""
    import lzmagpu as L
    orc = native.oracle()
    rng = random.Random(515)
    cases = []
    for i in range(40):
        data = native.gen("text", 97_000 + i, rng.choice([100, 4096, 20000]))
        comp = lzma.compress(data, format=lzma.FORMAT_RAW, filters=[
            {"id": lzma.FILTER_LZMA1, "dict_size": 1 << 16, "lc": 3, "lp": 0, "pb": 2}])
        cap = len(data) if i != 17 else (256 << 20) + 4096  # one oversized capacity
        cases.append((comp, W.props_bytes(3, 0, 2, 1 << 16), cap, 0 if i == 17 else 1))
    want = [native.decode(orc, "orc", c, p, cap, fin) for c, p, cap, fin in cases]
    L.coalesce_stats(reset=True)
    with ThreadPoolExecutor(16) as ex:
        got = list(ex.map(lambda k: L.LzmaDecode(*cases[k]), range(len(cases))))
    for k, (g, w) in enumerate(zip(got, want)):
        assert g[0] == w[0] and g[2:] == w[2:] and (g[0] != 0 or g[1] == w[1]), (k, g[:4], w[:4])
    batches, calls, _ = L.coalesce_stats()
    assert calls == len(cases) and batches >= 2, (batches, calls)


@pytest.mark.gpu
def test_gpu_concurrent_decode_to_buf_loops_fuzz():
    """Seeded zlib-like DecodeToBuf loops (LZGPU_DROPIN_FUZZ, default 120) run
    from 24 threads at once through the drop-in (dropin_capi.hip: mirrors with
    pooled device buffers, pinned staging, coalesced session launches): every
    call's {res, status, srcLen, destLen}, the output and the input used equal
    the oracle's loop (the restatement pinned to the reference's streaming
    traces)."""
    import lzmagpu as L
    from test_sessions import _fuzz_sessions
    cases = _fuzz_sessions(int(os.environ.get("LZGPU_DROPIN_FUZZ", "120")),
                           int(os.environ.get("LZGPU_DROPIN_SEED", "919")))

    def run(c):
        return L.stream_decode(c["src"], c["props"], c["out_total"], c["in_chunk"],
                               c["out_chunk"], c["finish"])

    with ThreadPoolExecutor(24) as ex:
        got = list(ex.map(run, cases))
    bad = []
    for k, (c, g) in enumerate(zip(cases, got)):
        calls, trace, out, used = g
        if list(map(tuple, trace)) != list(map(tuple, c["trace"])) or out != c["out"] or \
                used != c["used"]:
            bad.append((k, calls, trace[:2], c["trace"][:2]))
    assert not bad, (len(bad), bad[:4])

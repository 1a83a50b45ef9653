"""The drop-in from C: tests/c_host/lzma_c_host.c is written against the LZMA
SDK's own decode API (LzmaUncompress, LzmaDecode, LzmaDec_Allocate + Init +
DecodeToBuf, CrcCalc) the way a user of the reference calls it, compiled with
include/lzma_gpu.h in place of LzmaDec.h / LzmaLib.h / 7zCrc.h and linked to
liblzmagpu.so (no Python, no torch in the process).

CPU: it builds warning-free and, with no device, every call fails loudly with
SZ_ERROR_FAIL (no CPU fallback).  GPU: its results -- res, status, destLen,
srcLen, the CRC-32 of the output, the streaming loop's call count -- equal the
oracle's LzmaDecode / DecodeToBuf loop on the same inputs (the restatement
pinned to the reference's vectors)."""
import os
import subprocess
import zlib

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "c_host", "lzma_c_host.c")
BIN = os.path.join(ROOT, "tests", "c_host", "build", "lzma_c_host")


def build_c_host():
    """gcc -Wall -Wextra -Werror against include/, rpath to the in-tree library."""
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    subprocess.run(["gcc", "-O2", "-std=c99", "-Wall", "-Wextra", "-Werror", "-D_POSIX_C_SOURCE=200809L",
                    "-I", os.path.join(ROOT, "include"), "-o", BIN, SRC,
                    "-L", os.path.join(ROOT, "lzma-sdk-zliblike_amd", "lib"), "-llzmagpu",
                    "-Wl,-rpath,$ORIGIN/../../../lzma-sdk-zliblike_amd/lib"], check=True)
    return BIN


BATCH_SRC = os.path.join(ROOT, "tests", "c_host", "lzma_c_batch.c")
BATCH_BIN = os.path.join(ROOT, "tests", "c_host", "build", "lzma_c_batch")


def build_c_batch():
    """The batch program also calls the HIP runtime's C API (hipMalloc, ...):
    gcc with ROCm's headers (__HIP_PLATFORM_AMD__ is what hipcc would define
    for them) and libamdhip64."""
    os.makedirs(os.path.dirname(BATCH_BIN), exist_ok=True)
    subprocess.run(["gcc", "-O2", "-std=c99", "-Wall", "-Wextra", "-Werror",
                    "-D__HIP_PLATFORM_AMD__", "-I", os.path.join(ROOT, "include"),
                    "-I", "/opt/rocm/include", "-o", BATCH_BIN, BATCH_SRC,
                    "-L", os.path.join(ROOT, "lzma-sdk-zliblike_amd", "lib"), "-llzmagpu",
                    "-L", "/opt/rocm/lib", "-lamdhip64",
                    "-Wl,-rpath,$ORIGIN/../../../lzma-sdk-zliblike_amd/lib",
                    "-Wl,-rpath,/opt/rocm/lib"], check=True)
    return BATCH_BIN


THREADS_SRC = os.path.join(ROOT, "tests", "c_host", "lzma_c_threads.c")
THREADS_BIN = os.path.join(ROOT, "tests", "c_host", "build", "lzma_c_threads")
THREADS_REF = os.path.join(ROOT, "oracle", "_ref", "lzma_c_threads_ref")


def build_c_threads():
    """The multi-threaded LzmaDecode caller against include/lzma_gpu.h, linked
    to the in-tree library (its reference-linked twin: oracle/Makefile.ref)."""
    os.makedirs(os.path.dirname(THREADS_BIN), exist_ok=True)
    subprocess.run(["gcc", "-O2", "-std=c99", "-Wall", "-Wextra", "-Werror",
                    "-D_POSIX_C_SOURCE=200809L", "-I", os.path.join(ROOT, "include"),
                    "-o", THREADS_BIN, THREADS_SRC,
                    "-L", os.path.join(ROOT, "lzma-sdk-zliblike_amd", "lib"), "-llzmagpu",
                    "-lpthread", "-Wl,-rpath,$ORIGIN/../../../lzma-sdk-zliblike_amd/lib"],
                   check=True)
    return THREADS_BIN


def write_stream_set(tmp, comps, props, outs):
    """Files for lzma_c_threads: streams, uint64 lengths, props, output sizes."""
    import struct
    f = {k: os.path.join(tmp, k + ".bin") for k in ("src", "lens", "props", "outs")}
    open(f["src"], "wb").write(b"".join(comps))
    open(f["lens"], "wb").write(b"".join(struct.pack("<Q", len(c)) for c in comps))
    open(f["props"], "wb").write(b"".join(props))
    open(f["outs"], "wb").write(b"".join(struct.pack("<Q", n) for n in outs))
    return f


def run_c_threads(binary, threads, f, repeat=1, env=None, timeout=300, mode="one"):
    import json
    # the result line goes to stderr: the reference build prints a debug line
    # per call to stdout (LzmaDec.c:945), discarded here
    r = subprocess.run([binary, str(threads), f["src"], f["lens"], f["props"], f["outs"],
                        str(repeat), mode], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True,
                       timeout=timeout, env=env)
    assert r.returncode == 0, r.stderr
    return json.loads([ln for ln in r.stderr.splitlines() if ln.startswith("{")][-1])


def _run(tmp, props, src, out_size, in_chunk, out_chunk):
    p, s = os.path.join(tmp, "props.bin"), os.path.join(tmp, "stream.bin")
    open(p, "wb").write(props)
    open(s, "wb").write(src)
    r = subprocess.run([BIN, p, s, str(out_size), str(in_chunk), str(out_chunk)],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return {ln.split()[0]: ln.split()[1:] for ln in r.stdout.splitlines()}


def test_c_host_builds_and_fails_loudly_without_gpu(tmp_path):
    import lzma
    build_c_host()
    build_c_batch()
    build_c_threads()
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is visible: the GPU test covers this host")
    data = b"drop-in from C " * 500
    comp = lzma.compress(data, format=lzma.FORMAT_RAW, filters=[
        {"id": lzma.FILTER_LZMA1, "dict_size": 1 << 16, "lc": 3, "lp": 0, "pb": 2}])
    out = _run(str(tmp_path), bytes([0x5D]) + (1 << 16).to_bytes(4, "little"), comp,
               len(data), 1000, 4096)
    for name in ("LzmaUncompress", "LzmaDecode", "LzmaDec_DecodeToBuf", "LzmaDec_DecodeToDic"):
        assert out[name][0] == "11", (name, out[name])  # SZ_ERROR_FAIL, nothing decoded
        assert out[name][2] == "0"


@pytest.mark.gpu
def test_gpu_c_host_matches_oracle(tmp_path):
    import lzma
    import native
    import workloads as W
    if not os.path.exists(BIN):
        build_c_host()
    orc = native.oracle()
    cases = []
    for k, (lc, lp, pb, dsz, n, mark, cut, in_chunk, out_chunk) in enumerate([
            (3, 0, 2, 1 << 16, 200_000, False, 0, 1000, 4096),
            (3, 0, 2, 1 << 16, 200_000, True, 0, 7, 65536),
            (0, 2, 0, 4096, 50_000, True, 0, 1 << 20, 1),
            (4, 0, 4, 1 << 20, 300_000, False, 100, 4096, 100_000),
            (1, 1, 1, 1 << 14, 30_000, True, 7, 333, 777)]):
        data = native.gen("text", 555_000 + k, n)
        filt = {"id": lzma.FILTER_LZMA1, "dict_size": dsz, "lc": lc, "lp": lp, "pb": pb}
        if mark:
            comp = lzma.compress(data, format=lzma.FORMAT_ALONE, filters=[filt])[13:]
        else:
            comp = lzma.compress(data, format=lzma.FORMAT_RAW, filters=[filt])
        if cut:
            comp = comp[:-cut]
        cases.append((W.props_bytes(lc, lp, pb, dsz), comp, n, in_chunk, out_chunk))
    for props, comp, n, in_chunk, out_chunk in cases:
        out = _run(str(tmp_path), props, comp, n, in_chunk, out_chunk)
        res, st, dl, sl, dec = native.decode(orc, "orc", comp, props, n, 0)
        assert out["LzmaUncompress"] == [str(res), "-", str(dl), str(sl),
                                         "%08x" % zlib.crc32(dec)]
        res, st, dl, sl, dec = native.decode(orc, "orc", comp, props, n, 1)
        got = out["LzmaDecode"]
        assert [got[0], got[2], got[3], got[4]] == [str(res), str(dl), str(sl),
                                                    "%08x" % zlib.crc32(dec)]
        if res == 0:
            assert got[1] == str(st)
        calls, trace, dec, used = native.stream_decode(orc, "orc", comp, props, n, in_chunk,
                                                       out_chunk, 0)
        assert out["LzmaDec_DecodeToBuf"] == [str(trace[-1][0]), str(trace[-1][1]), str(len(dec)),
                                              str(used), "%08x" % zlib.crc32(dec), str(calls)]
        calls, trace, dec, used, _ = native.dic_decode(orc, "orc", comp, props, n, in_chunk)
        assert out["LzmaDec_DecodeToDic"] == [str(trace[-1][0]), str(trace[-1][1]), str(len(dec)),
                                              str(used), "%08x" % zlib.crc32(dec), str(calls)]


@pytest.mark.gpu
def test_gpu_c_batch_host_and_device_match_oracle(tmp_path):
    """300 streams (mixed lc/lp/pb and dictionaries, corrupt and truncated ones)
    through LzmaGpu_DecodeBatchHost, through PlanBatchEx + DecodeBatchEx on the
    C program's own hipMalloc'd buffers, and time-sliced (PlanSliced, rounds of
    4 KiB enqueued one at a time): per-stream results and output CRCs equal the
    oracle's LzmaDecode."""
    import lzma
    import random
    import struct
    import native
    import workloads as W
    if not os.path.exists(BATCH_BIN):
        build_c_batch()
    rng = random.Random(99)
    orc = native.oracle()
    cap = 20000
    srcs, lens, props_all, want = [], [], [], []
    for i in range(300):
        lc = rng.randrange(5)
        lp = rng.randrange(5 - lc)
        pb = rng.randrange(5)
        dsz = rng.choice([4096, 1 << 16])
        n = rng.choice([0, 10, 4096, 15000, 20000])
        data = native.gen(rng.choice(["text", "random"]), 777_000 + i, n)
        comp = bytearray(lzma.compress(data, format=lzma.FORMAT_RAW, filters=[
            {"id": lzma.FILTER_LZMA1, "dict_size": dsz, "lc": lc, "lp": lp, "pb": pb}]))
        if i % 7 == 3 and len(comp) > 8:
            comp[rng.randrange(5, len(comp))] ^= 0x10
        if i % 11 == 5:
            comp = comp[:rng.randrange(len(comp) + 1)]
        props = W.props_bytes(lc, lp, pb, dsz)
        res, st, dl, sl, dec = native.decode(orc, "orc", bytes(comp), props, cap, 0)
        srcs.append(bytes(comp))
        lens.append(len(comp))
        props_all.append(props)
        want.append("%d %d %d %d %08x" % (res, st, dl, sl, zlib.crc32(dec)))
    files = {k: os.path.join(str(tmp_path), k) for k in ("src", "lens", "props")}
    open(files["src"], "wb").write(b"".join(srcs))
    open(files["lens"], "wb").write(b"".join(struct.pack("<Q", x) for x in lens))
    open(files["props"], "wb").write(b"".join(props_all))
    for mode in ("host", "device", "sliced"):
        r = subprocess.run([BATCH_BIN, mode, files["src"], files["lens"], files["props"],
                            str(cap), "0"], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           text=True, timeout=120)
        assert r.returncode == 0, (mode, r.stderr)
        got = r.stdout.splitlines()
        bad = [(k, got[k], want[k]) for k in range(len(want)) if got[k] != want[k]]
        assert len(got) == len(want) and not bad, (mode, bad[:5])


# ---------------------------------------------------------------- reference LZMA2 walker
# oracle/_ref/lzma2_walker: the reference's own Lzma2Dec.c (compiled in place by
# oracle/Makefile.ref) driving this library's LzmaDec_* through the drop-in ABI.
# It writes stored chunks into CLzmaDec.dic itself and advances dicPos /
# processedPos (Lzma2Dec.c:159-166), so LZMA chunks that match into stored bytes
# read what the HOST wrote: the device mirror must upload them (VERDICT r03
# item 5, dropin_capi.hip's coherence check).
WALKER = os.path.join(ROOT, "oracle", "_ref", "lzma2_walker")


def _lzma2_prop(dsz):
    for p in range(41):
        if ((2 | (p & 1)) << (p // 2 + 11)) >= dsz:
            return p
    return 40


def _lzma2_chunks(comp):
    """(control byte, unpacked size) per chunk of an LZMA2 stream."""
    out, i = [], 0
    while i < len(comp) and comp[i] != 0:
        c = comp[i]
        if c & 0x80:
            un = ((c & 0x1F) << 16) + (comp[i + 1] << 8) + comp[i + 2] + 1
            pk = (comp[i + 3] << 8) + comp[i + 4] + 1
            i += 5 + (1 if (c >> 5) & 3 >= 2 else 0) + pk
        else:
            un = (comp[i + 1] << 8) + comp[i + 2] + 1
            i += 3 + un
        out.append((c, un))
    return out


def _stored_then_referenced(seed, dsz=1 << 20):
    """LZMA2 streams (liblzma) whose stored chunks (incompressible random blocks)
    are followed by LZMA chunks copying parts of them: a match into a stored
    chunk reads bytes only the host walker wrote."""
    import lzma
    import random
    import native
    rng = random.Random(seed)
    parts, blocks = [], []
    for k in range(4):
        blk = rng.randbytes(rng.choice([150_000, 200_000, 250_000]))  # incompressible
        blocks.append(blk)
        parts.append(blk)
        text = native.gen("text", seed * 10 + k, rng.randrange(5_000, 30_000))
        parts.append(text)
        for _ in range(40):  # repeats of earlier random (stored) bytes between text
            b = rng.choice(blocks)
            o = rng.randrange(len(b) - 300)
            parts.append(b[o:o + rng.randrange(20, 300)])
            parts.append(text[:rng.randrange(1, 200)])
    data = b"".join(parts)
    comp = lzma.compress(data, format=lzma.FORMAT_RAW,
                         filters=[{"id": lzma.FILTER_LZMA2, "dict_size": dsz}])
    return data, comp, _lzma2_prop(dsz)


def test_lzma2_walker_streams_have_stored_chunks_referenced_later():
    """The vectors exercise what the test is about: stored chunks, and LZMA
    chunks after them in the same dictionary (no dict reset)."""
    for seed in (1, 2):
        data, comp, prop = _stored_then_referenced(seed)
        ch = _lzma2_chunks(comp)
        kinds = [("stored" if c & 0x80 == 0 else "lzma") for c, _ in ch]
        assert "stored" in kinds and "lzma" in kinds[kinds.index("stored"):]
        assert all(c not in (1,) and (c & 0x80 == 0 or (c >> 5) & 3 != 3) for c, _ in ch[1:])
        assert sum(u for _, u in ch) == len(data)


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(WALKER), reason="oracle/_ref/lzma2_walker not built "
                    "(built where /root/reference exists, travels with the tree)")
def test_gpu_reference_lzma2_walker_over_dropin(tmp_path):
    """The reference's Lzma2Dec.c, unchanged, over the GPU LzmaDec_DecodeToDic:
    output and {res, status, dicPos, inPos} equal the oracle's Lzma2 decode and
    the plaintext, for whole-buffer, windowed-input and windowed-dicLimit
    drives (stored chunks are written by the host between GPU calls)."""
    import native
    orc = native.oracle()
    for seed in (1, 2):
        data, comp, prop = _stored_then_referenced(seed)
        res, st, dl, sl, dec = native.lzma2_decode(orc, "orc", comp, prop, len(data), 1)
        assert (res, st, dl, sl) == (0, 1, len(data), len(comp)) and dec == data
        want = "0 1 %d %d %08x" % (len(data), len(comp), zlib.crc32(data))
        s = os.path.join(str(tmp_path), "s%d.bin" % seed)
        open(s, "wb").write(comp)
        for in_chunk, dic_chunk in ((1 << 30, 0), (4096, 0), (777, 5000), (100_000, 65536)):
            r = subprocess.run([WALKER, str(prop), s, str(len(data)), str(in_chunk),
                                str(dic_chunk)], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                               text=True, timeout=300)
            assert r.returncode == 0, r.stderr
            got = r.stdout.split()
            assert " ".join(got[:5]) == want, (seed, in_chunk, dic_chunk, got, want)


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(WALKER), reason="oracle/_ref/lzma2_walker not built "
                    "(built where /root/reference exists, travels with the tree)")
def test_gpu_reference_lzma2_walker_ring_over_dropin(tmp_path):
    """The reference's Lzma2Dec_DecodeToBuf (XzDec's shape) over the GPU
    LzmaDec_*: the decoder's own 256 KiB ring under ~1 MB of output, so stored
    chunks reach the ring in pieces on either side of its end and the device
    mirror sees host-written spans across the wrap (dropin_capi.hip's two-piece
    upload).  Output and {res, status, outPos, inPos} equal the
    plaintext and the oracle's flat decode, for several input / output chunk
    sizes."""
    import native
    orc = native.oracle()
    for seed in (3, 4):
        data, comp, prop = _stored_then_referenced(seed, dsz=1 << 18)
        assert len(data) > 3 * (1 << 18)  # the ring wraps several times
        res, st, dl, sl, dec = native.lzma2_decode(orc, "orc", comp, prop, len(data), 1)
        assert (res, st, dl, sl) == (0, 1, len(data), len(comp)) and dec == data
        want = "0 1 %d %d %08x" % (len(data), len(comp), zlib.crc32(data))
        s = os.path.join(str(tmp_path), "r%d.bin" % seed)
        open(s, "wb").write(comp)
        for in_chunk, out_chunk in ((1 << 30, 1 << 30), (4096, 1 << 16), (100_000, 77_777)):
            r = subprocess.run([WALKER, str(prop), s, str(len(data)), str(in_chunk), "0",
                                str(out_chunk)], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                               text=True, timeout=300)
            assert r.returncode == 0, r.stderr
            got = r.stdout.split()
            assert " ".join(got[:5]) == want, (seed, in_chunk, out_chunk, got, want)

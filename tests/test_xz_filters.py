"""xz blocks with Delta / PPC / IA64 / ARM / ARMT / SPARC filters and chains
(SURVEY.md 8(f) rows 3-4): the reference's BraState_Code (XzDec.c:119-196)
runs the converters of Bra.c / BraIA64.c / Delta.c after LZMA2, last filter
first (MixCoder, XzDec.c:574-585).  Fixtures: tests/golden/xzf_cases.json +
xzf_blob.bin (tests/golden/make_golden_xzf.py, reference compiled in place,
every valid file also decoded by liblzma).

CPU: LzmaGpu_XzIndex (host) reports each block's chain and rejects the
props the reference rejects.  GPU: LzmaGpu_XzDecode on every fixture, and a
file of 192 concatenated streams with mixed chains against liblzma.
"""
import hashlib
import json
import lzma
import os
import sys

import pytest

import native

GOLDEN = os.path.join(native.ROOT, "tests", "golden")
sys.path.insert(0, GOLDEN)
sys.path.insert(0, os.path.join(native.ROOT, "lzma-sdk-zliblike_amd"))


def fixtures():
    with open(os.path.join(GOLDEN, "xzf_cases.json")) as f:
        d = json.load(f)
    with open(os.path.join(GOLDEN, "xzf_blob.bin"), "rb") as f:
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


def test_index_reports_filter_chains(L):
    d = fixtures()
    for c in d["xz"]:
        r, blocks, total = L.xz_index(data_of(d, c))
        if not c["valid"]:
            assert r == c["res"] == 4, c["note"]
            continue
        assert r == 0, c["note"]
        assert total == c["dest_len"]
        for b in blocks:
            chain = [(b.filter_id[k], b.filter_prop[k]) for k in range(b.num_filters)]
            assert chain == [tuple(x) for x in c["chain"]], c["note"]
            assert b.x86 == int(any(i == 4 for i, _ in chain))


@pytest.mark.gpu
def test_gpu_xz_filter_fixtures(L):
    d = fixtures()
    for c in d["xz"]:
        cap = (c["dest_len"] if c["valid"] else 400000) + 64
        r, out, bad = L.XzDecode(data_of(d, c), cap)
        assert r == c["res"], (c["note"], r, bad, L.last_error())
        if c["valid"]:
            assert hashlib.sha256(out).hexdigest() == c["sha256"], c["note"]


@pytest.mark.gpu
def test_gpu_xz_mixed_chains_many_streams(L):
    from make_golden_bra import branchy
    LZ2 = {"id": lzma.FILTER_LZMA2, "preset": 1}
    chains = [[{"id": lzma.FILTER_ARM}], [{"id": lzma.FILTER_ARMTHUMB}],
              [{"id": lzma.FILTER_POWERPC, "start_offset": 0x400}], [{"id": lzma.FILTER_SPARC}],
              [{"id": lzma.FILTER_IA64}], [{"id": lzma.FILTER_DELTA, "dist": 5}],
              [{"id": lzma.FILTER_X86}, {"id": lzma.FILTER_DELTA, "dist": 2}],
              [{"id": lzma.FILTER_DELTA, "dist": 1}, {"id": lzma.FILTER_ARM},
               {"id": lzma.FILTER_DELTA, "dist": 256}], []]
    kinds = ["ARM", "ARMT", "PPC", "SPARC", "IA64"]
    parts, plain = [], []
    for i in range(192):
        data = branchy(kinds[i % 5], 5000 + i, 8192 + 37 * i)
        parts.append(lzma.compress(data, format=lzma.FORMAT_XZ, check=(1, 4, 10)[i % 3],
                                   filters=chains[i % len(chains)] + [LZ2]))
        plain.append(data)
    blob, want = b"".join(parts), b"".join(plain)
    assert lzma.decompress(blob, format=lzma.FORMAT_XZ) == want
    r, out, bad = L.XzDecode(blob, len(want))
    assert r == 0, (r, bad, L.last_error())
    assert out == want

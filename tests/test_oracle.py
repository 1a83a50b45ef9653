"""Pin the CPU restatement (oracle/lzma_oracle.c) to the reference.

1. Every golden vector in tests/golden/ (generated from the reference sources):
   output sha256 + {res, status, destLen, srcLen}; streaming traces.
2. When the in-place reference build oracle/_ref/libref.so is present (build
   container only), a seeded fuzz of bit flips / truncations / finish modes /
   capacities against the live reference.
"""
import os
import random

import pytest

import golden_cases as G
import native


@pytest.fixture(scope="module")
def orc():
    return native.oracle()


@pytest.mark.parametrize("idx", [i for i, _ in G.cases("lzma")])
def test_oracle_lzma_golden(orc, idx):
    d = G.load()
    c = d["cases"][idx]
    src = G.case_input(d, c)
    res, st, dl, sl, out = native.decode(orc, "orc", src, bytes.fromhex(c["props"]),
                                         c["dest_cap"], c["finish"])
    e = c["expect"]
    assert (res, st, dl, sl) == (e["res"], e["status"], e["dest_len"], e["src_len"]), c["note"]
    assert G.sha(out) == e["sha256"], c["note"]


@pytest.mark.parametrize("idx", [i for i, _ in G.cases("stream")])
def test_oracle_stream_golden(orc, idx):
    d = G.load()
    c = d["cases"][idx]
    src = G.case_input(d, c)
    calls, trace, out, used = native.stream_decode(orc, "orc", src, bytes.fromhex(c["props"]),
                                                   c["out_total"], c["in_chunk"], c["out_chunk"],
                                                   c["finish"])
    e = c["expect"]
    assert calls == e["calls"]
    assert G.trace_digest(trace) == e["trace_sha256"]
    assert (len(out), used) == (e["out_len"], e["in_used"])
    assert G.sha(out) == e["sha256"]


@pytest.mark.parametrize("idx", [i for i, _ in G.cases("lzma2")])
def test_oracle_lzma2_golden(orc, idx):
    d = G.load()
    c = d["cases"][idx]
    src = G.case_input(d, c)
    res, st, dl, sl, out = native.lzma2_decode(orc, "orc", src, c["prop"], c["dest_cap"],
                                               c["finish"])
    e = c["expect"]
    assert (res, st, dl, sl) == (e["res"], e["status"], e["dest_len"], e["src_len"]), c["note"]
    assert G.sha(out) == e["sha256"], c["note"]


needs_ref = pytest.mark.skipif(not os.path.exists(native.REF_SO),
                               reason="reference build oracle/_ref/libref.so absent")


@needs_ref
def test_oracle_vs_live_reference_fuzz(orc):
    rng = random.Random(4242)
    ref = native.ref()
    for it in range(300):
        lc, lp, pb = rng.randrange(9), rng.randrange(5), rng.randrange(5)
        d = rng.choice([4096, 1 << 14, 1 << 16])
        n = rng.choice([0, 1, 2, 50, 700, 4000, 12000])
        kind = rng.choice(["text", "random", "runs"])
        data = native.gen(kind, 10_000 + it, n)
        pr, c = native.ref_encode(data, level=rng.choice([0, 5, 9]), dict_size=d, lc=lc, lp=lp,
                                  pb=pb, end_mark=rng.random() < 0.5)
        c = bytearray(c)
        mode = rng.randrange(4)
        if mode == 1 and len(c) > 6:
            c[rng.randrange(5, len(c))] ^= 1 << rng.randrange(8)
        elif mode == 2:
            c = c[:rng.randrange(len(c) + 1)]
        cap = max(0, n + rng.choice([0, 0, 1, -1, 37, -37]))
        fin = rng.randrange(2)
        a = native.decode(ref, "ref", bytes(c), pr, cap, fin)
        b = native.decode(orc, "orc", bytes(c), pr, cap, fin)
        assert a == b, (it, lc, lp, pb, d, n, kind, mode, cap, fin)


@pytest.mark.skipif(not native.have_ref(), reason="oracle/_ref/libref_lzma.so not built")
def test_symbol_encoder_pinned_by_reference_ring_decode():
    """tests/lzmaenc_min.py writes the hand-made ring-reach streams of
    tests/test_dropin_mirror.py.  The reference's own
    LzmaDec_DecodeToBuf over a caller-owned 4 KiB ring reproduces the encoder's
    model of the decoder output exactly; a flat LzmaDecode of the same stream
    does not -- its matches at distance 5,096 read true history where the ring
    decoder reads the slot 1,000 bytes back, which is what the GPU test pins."""
    import lzmaenc_min as E
    for seed in (1, 2, 3):
        comp, props, out = E.ring_reach_stream(seed)
        trace, got = E.ring_decode(native.ref(), comp, props, 4096, len(out), 1 << 30, 3000)
        assert got == out and trace[-1][0] == 0
        flat = native.decode(native.ref(), "ref", comp, props, len(out), 0)
        assert flat[4] != out

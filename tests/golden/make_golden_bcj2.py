"""Generate tests/golden/bcj2_cases.json + bcj2_blob.bin from the REFERENCE
BCJ2 decoder (Bcj2.c Bcj2_Decode, compiled in place into oracle/_ref/libref.so
by oracle/Makefile.ref).

Run in the build container only:

    python tests/golden/make_golden_bcj2.py

The four input streams come from tests/bcj2enc.py (this build's own BCJ2
encoder: the reference has none) over synthetic x86-flavoured bytes, then are
varied to reach every exit of the decoder: exact / short / long output sizes
(a converted operand clipped at outSize, the main stream running out), rc
streams truncated (inside the 5 init bytes, before a NORMALIZE), CALL / JMP
streams truncated, corrupted rc bytes, conversion policies (none, all, by
target), empty streams, and the 7zDec layout where the main stream is the tail
of the output buffer.  Every case records the reference's return value and
the SHA-256 of the whole output buffer (prefilled with 0xA5 before the call,
so bytes the decoder never writes are pinned too).
"""
import ctypes
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import bcj2enc as E  # noqa: E402
import native  # noqa: E402

FILL = 0xA5


def ref_decode(lib, m, c, j, r, out_size, overlap=False):
    """Reference Bcj2_Decode; overlap: main stream placed at the output's tail
    (7zDec.c:367-372), which requires len(m) <= out_size."""
    f = lib.Bcj2_Decode
    f.restype = ctypes.c_int
    sz = ctypes.c_size_t
    if overlap:
        buf = ctypes.create_string_buffer(bytes([FILL]) * max(out_size, 1), max(out_size, 1))
        at = out_size - len(m)
        ctypes.memmove(ctypes.addressof(buf) + at, m, len(m))
        res = f(ctypes.byref(buf, at), sz(len(m)), c, sz(len(c)), j, sz(len(j)), r, sz(len(r)),
                buf, sz(out_size))
        return res, buf.raw[:out_size]
    out = ctypes.create_string_buffer(bytes([FILL]) * max(out_size, 1), max(out_size, 1))
    res = f(m, sz(len(m)), c, sz(len(c)), j, sz(len(j)), r, sz(len(r)), out, sz(out_size))
    return res, out.raw[:out_size]


def main():
    lib = native.ref_cont()
    blob = bytearray()
    seen = {}

    def put(b):  # identical streams are stored once
        b = bytes(b)
        if b not in seen:
            seen[b] = len(blob)
            blob.extend(b)
        return seen[b]

    cases = []

    def add(note, m, c, j, r, out_size, overlap=False):
        res, out = ref_decode(lib, m, c, j, r, out_size, overlap)
        cases.append({"note": note, "overlap": overlap, "out_size": out_size,
                      "streams": [[put(x), len(x)] for x in (m, c, j, r)],
                      "res": res, "out_sha256": hashlib.sha256(out).hexdigest()})

    rng = random.Random(2)
    policies = {"by target": None, "none": lambda p, o, rel: False,
                "all": lambda p, o, rel: True, "half": lambda p, o, rel: (p * 7) % 3 != 0}
    for seed, n in ((1, 0), (2, 1), (3, 5), (4, 64), (5, 4096), (6, 60001), (7, 100000)):
        data = E.x86_like(seed, n, density=0.04 + 0.02 * (seed % 3))
        for pname, pol in policies.items():
            m, c, j, r = E.encode(data, pol)
            add(f"n={n} {pname}", m, c, j, r, n)
            if n >= 64 and pname in ("by target", "all"):
                add(f"n={n} {pname}, main at the output tail", m, c, j, r, n, overlap=True)
                for cut in (1, 2, 3, 5, 1000):
                    if cut < n:
                        add(f"n={n} {pname}, outSize -{cut}", m, c, j, r, n - cut)
                add(f"n={n} {pname}, outSize +7", m, c, j, r, n + 7)
                add(f"n={n} {pname}, rc truncated to 4", m, c, j, r[:4], n)
                add(f"n={n} {pname}, rc -1", m, c, j, r[:-1], n)
                add(f"n={n} {pname}, rc half", m, c, j, r[:len(r) // 2], n)
                if len(c) >= 4:
                    add(f"n={n} {pname}, call -4", m, c[:-4], j, r, n)
                if len(j) >= 4:
                    add(f"n={n} {pname}, jump -4", m, c, j[:-4], r, n)
                add(f"n={n} {pname}, main -1", m[:-1], c, j, r, n)
                for k in range(3):
                    bad = bytearray(r)
                    if len(bad) > 6:
                        bad[rng.randrange(5, len(bad))] ^= 1 << rng.randrange(8)
                    add(f"n={n} {pname}, rc bit flip {k}", m, c, j, bytes(bad), n)
    # degenerate: all streams empty with outSize 0 / 1, rc of exactly 5 bytes
    add("empty, outSize 0, no rc bytes", b"", b"", b"", b"", 0)
    add("empty, outSize 0, 5 rc bytes", b"", b"", b"", b"\0" * 5, 0)
    add("one byte, outSize 1", b"\x90", b"", b"", b"\0" * 5, 1)
    add("E8 last byte", b"\x90\xe8", b"", b"", b"\0" * 5, 2)
    add("Jcc pair at the end", b"\x0f\x85", b"", b"", b"\0" * 5, 2)
    with open(os.path.join(HERE, "bcj2_blob.bin"), "wb") as f:
        f.write(blob)
    meta = {"generator": "tests/golden/make_golden_bcj2.py",
            "reference": "LZMA SDK 9.20 Bcj2.c Bcj2_Decode (oracle/_ref/libref.so)",
            "encoder": "tests/bcj2enc.py (test infrastructure)", "fill": FILL,
            "blob": "bcj2_blob.bin", "blob_sha256": hashlib.sha256(blob).hexdigest(),
            "cases": cases}
    with open(os.path.join(HERE, "bcj2_cases.json"), "w") as f:
        json.dump(meta, f, indent=0)
    print(f"{len(cases)} BCJ2 cases, results {sorted({c['res'] for c in cases})}, "
          f"blob {len(blob)} B")


if __name__ == "__main__":
    main()

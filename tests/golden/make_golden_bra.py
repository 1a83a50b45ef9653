"""Generate tests/golden/bra_cases.json + bra_blob.bin from the REFERENCE RISC
branch converters (Bra.c ARM/ARMT/PPC/SPARC_Convert, BraIA64.c IA64_Convert)
and delta filter (Delta.c Delta_Encode / Delta_Decode).

Run in the build container only (needs oracle/_ref/libref.so from
`make -f oracle/Makefile.ref`, which compiles Bra.c, BraIA64.c and Delta.c in
place):

    python tests/golden/make_golden_bra.py

Inputs are synthetic: random words where a large share carry each kind's
branch pattern (ARM BL 0xEB top byte, Thumb BL halfword pairs, PPC "bl",
SPARC "call", IA64 bundles with branch templates and opcode 5 slots), in
ragged sizes around the unit sizes, start ips that wrap, both directions.
Delta cases cover delta 1..256, sizes below and above delta, non-zero
carried state and chained calls.  Each case records the input, the
reference's output bytes, its return value (converters) or new state (delta).
"""
import ctypes
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import native  # noqa: E402

KINDS = {"PPC": 5, "IA64": 6, "ARM": 7, "ARMT": 8, "SPARC": 9}


def branchy(kind, seed, n):
    """Random bytes where many units hold `kind`'s branch encoding."""
    rng = random.Random(seed)
    b = bytearray(rng.getrandbits(8) for _ in range(n))
    if kind == "ARM":
        for i in range(0, n - 3, 4):
            if rng.random() < 0.5:
                b[i + 3] = 0xEB
    elif kind == "ARMT":
        for i in range(0, n - 3, 2):
            if rng.random() < 0.3:
                b[i + 1] = 0xF0 | (b[i + 1] & 7)
                b[i + 3] = 0xF8 | (b[i + 3] & 7)
    elif kind == "PPC":
        for i in range(0, n - 3, 4):
            if rng.random() < 0.5:
                b[i] = 0x48 | (b[i] & 3)
                b[i + 3] = (b[i + 3] & ~3 & 0xFF) | 1
    elif kind == "SPARC":
        for i in range(0, n - 3, 4):
            r = rng.random()
            if r < 0.25:
                b[i], b[i + 1] = 0x40, b[i + 1] & 0x3F
            elif r < 0.5:
                b[i], b[i + 1] = 0x7F, b[i + 1] | 0xC0
    elif kind == "IA64":
        for i in range(0, n - 15, 16):
            if rng.random() < 0.8:
                b[i] = (b[i] & 0xE0) | rng.choice([16, 17, 18, 19, 22, 23, 24, 25, 28, 29])
                # force opcode 5 and zero btype bits in each slot sometimes
                for slot in range(3):
                    if rng.random() < 0.6:
                        bp = 5 + 41 * slot
                        v = int.from_bytes(b[i:i + 16], "little")
                        v &= ~(0xF << (bp + 37))
                        v |= 0x5 << (bp + 37)
                        v &= ~(0x7 << (bp + 9))
                        b[i:i + 16] = v.to_bytes(16, "little")
    return bytes(b)


def main():
    lib = native.ref_cont()
    for k in KINDS:
        f = getattr(lib, k + "_Convert")
        f.restype = ctypes.c_size_t
        f.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int]
    for f in (lib.Delta_Encode, lib.Delta_Decode):
        f.restype = None
        f.argtypes = [ctypes.c_char_p, ctypes.c_uint, ctypes.c_char_p, ctypes.c_size_t]
    blob = bytearray()

    def put(data):
        off = len(blob)
        blob.extend(data)
        return off

    bra = []
    sizes = [0, 1, 3, 4, 5, 6, 7, 8, 15, 16, 17, 31, 32, 33, 100, 1021, 4096, 65537]
    ips = [0, 0x1000, 0x12345678, 0xFFFFFF00]
    for kind in KINDS:
        for si, n in enumerate(sizes):
            for enc in (0, 1):
                ip = ips[(si + enc) % len(ips)]
                data = branchy(kind, 1000 * KINDS[kind] + 10 * si + enc, n)
                buf = ctypes.create_string_buffer(data, max(n, 1))
                done = getattr(lib, kind + "_Convert")(buf, n, ip, enc)
                bra.append({"kind": kind, "id": KINDS[kind], "ip": ip, "encoding": enc,
                            "len": n, "in": put(data), "out": put(buf.raw[:n]), "done": done})
    # chained calls over one buffer (the reference's loop in Bra.h:40-52)
    for kind in KINDS:
        data = branchy(kind, 77 + KINDS[kind], 10000)
        buf = bytearray(data)
        pos, ip, chain = 0, 0x400000, []
        for piece in (13, 1000, 37, 4096, 9999):
            n = min(piece, len(buf) - pos)
            cb = ctypes.create_string_buffer(bytes(buf[pos:pos + n]), max(n, 1))
            done = getattr(lib, kind + "_Convert")(cb, n, ip + pos, 0)
            buf[pos:pos + n] = cb.raw[:n]
            chain.append({"len": n, "done": done})
            pos += done
        bra.append({"kind": kind, "id": KINDS[kind], "chain": chain, "ip": ip, "encoding": 0,
                    "len": len(data), "in": put(data), "out": put(bytes(buf)), "done": pos})

    delta = []
    rng = random.Random(5)
    # 8 and 32 last (keeps the earlier cases' random draws): d = 8 is a tile-scan
    # distance (one x += x << 64 step), 32 the segmented scan just above it
    for d in (1, 2, 3, 4, 7, 16, 100, 255, 256, 8, 32):
        extra = {20000, 20003} if d in (8, 32) else set()
        for n in sorted({0, 1, d - 1, d, d + 1, 3 * d + 2, 5000} | extra):
            if n < 0:
                continue
            for enc in (0, 1):
                state = bytes(rng.getrandbits(8) for _ in range(256)) if (n + d) % 2 else bytes(256)
                data = bytes(rng.getrandbits(8) for _ in range(n))
                st = ctypes.create_string_buffer(state, 256)
                buf = ctypes.create_string_buffer(data, max(n, 1))
                (lib.Delta_Encode if enc else lib.Delta_Decode)(st, d, buf, n)
                delta.append({"delta": d, "encoding": enc, "len": n, "in": put(data),
                              "out": put(buf.raw[:n]), "state_in": put(state),
                              "state_out": put(st.raw[:256])})
    with open(os.path.join(HERE, "bra_blob.bin"), "wb") as f:
        f.write(blob)
    meta = {"generator": "tests/golden/make_golden_bra.py",
            "reference": "LZMA SDK 9.20 Bra.c, BraIA64.c, Delta.c (oracle/_ref/libref.so)",
            "blob": "bra_blob.bin", "blob_sha256": hashlib.sha256(blob).hexdigest(),
            "bra": bra, "delta": delta}
    with open(os.path.join(HERE, "bra_cases.json"), "w") as f:
        json.dump(meta, f, indent=0)
    print(f"{len(bra)} converter cases, {len(delta)} delta cases, blob {len(blob)} B")


if __name__ == "__main__":
    main()

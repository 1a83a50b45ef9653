"""Generate tests/golden/xz_cases.json + xz_blob.bin from the REFERENCE xz
decoder (XzUnpacker_Code, XzDec.c) and x86 BCJ (x86_Convert, Bra86.c).

Run in the build container only (needs oracle/_ref/libref.so (container library) from
`make -f oracle/Makefile.ref`, which compiles XzDec.c, Xz.c, XzCrc64.c,
Sha256.c and the branch converters in place):

    python tests/golden/make_golden_xz.py

Inputs are xz files written by liblzma (Python's lzma: single-block streams
with every check type, the x86 BCJ filter with and without a start offset,
concatenated streams with stream padding, an empty stream) and multi-block
streams assembled here block by block from raw LZMA2 (liblzma FORMAT_RAW)
following the xz file format (stream header, block headers, padding,
checks, index, footer).  Every valid file is decoded by both the reference
and liblzma and must agree; corrupt variants record the reference's result
code.  x86 BCJ cases record the reference's converted bytes, state and
processed count for ragged buffer sizes and carried state.
"""
import ctypes
import hashlib
import json
import lzma
import os
import struct
import sys
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import native  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "lzma-sdk-zliblike_amd"))
from xzwrite import CHECK_SIZE, check_value, crc64, lzma2_prop, make_block, make_stream, varint  # noqa: E402,F401

_sp = ctypes.POINTER(ctypes.c_size_t)
_ip = ctypes.POINTER(ctypes.c_int)


def x86_like(seed, n):
    """Bytes with many E8/E9 rel32 operands (call/jmp) among text."""
    txt = native.gen("text", seed, n)
    b = bytearray(txt)
    r = seed * 2654435761 & 0xFFFFFFFF
    i = 0
    while i + 5 < n:
        r = (r * 1103515245 + 12345) & 0xFFFFFFFF
        step = 3 + (r >> 24) % 29
        i += step
        if i + 5 >= n:
            break
        b[i] = 0xE8 if (r >> 5) & 1 else 0xE9
        rel = (r >> 8) % 40000 - 20000
        b[i + 1:i + 5] = struct.pack("<i", rel)
        i += 5
    return bytes(b)


def main():
    lib = native.ref_cont()
    lib.ref_xz_decode.restype = ctypes.c_int
    lib.ref_xz_decode.argtypes = [ctypes.c_char_p, _sp, ctypes.c_char_p, _sp, _ip, _ip]
    lib.ref_x86_convert.restype = ctypes.c_size_t
    lib.ref_x86_convert.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint,
                                    ctypes.POINTER(ctypes.c_uint), ctypes.c_int]
    lib.ref_crc64.restype = ctypes.c_uint64
    lib.ref_crc64.argtypes = [ctypes.c_char_p, ctypes.c_size_t]

    files = []  # (note, bytes, plain or None)
    text = native.gen("text", 900, 300000)
    rnd = native.gen("random", 901, 70000)
    for chk, name in ((lzma.CHECK_NONE, "none"), (lzma.CHECK_CRC32, "crc32"),
                      (lzma.CHECK_CRC64, "crc64"), (lzma.CHECK_SHA256, "sha256")):
        files.append((f"liblzma 1 block, check {name}",
                      lzma.compress(text[:100000 + 7 * chk], format=lzma.FORMAT_XZ, check=chk),
                      text[:100000 + 7 * chk]))
    xd = x86_like(902, 120000)
    files.append(("liblzma x86 BCJ + LZMA2, crc64",
                  lzma.compress(xd, format=lzma.FORMAT_XZ, check=lzma.CHECK_CRC64,
                                filters=[{"id": lzma.FILTER_X86},
                                         {"id": lzma.FILTER_LZMA2, "preset": 6}]), xd))
    files.append(("liblzma x86 BCJ start_offset 0x1000, crc32",
                  lzma.compress(xd[:50001], format=lzma.FORMAT_XZ, check=lzma.CHECK_CRC32,
                                filters=[{"id": lzma.FILTER_X86, "start_offset": 0x1000},
                                         {"id": lzma.FILTER_LZMA2, "preset": 6}]), xd[:50001]))
    files.append(("liblzma empty input", lzma.compress(b"", format=lzma.FORMAT_XZ), b""))
    parts = [text[:30000], rnd[:20000], text[40000:41000]]
    cat = b""
    for k, p in enumerate(parts):
        cat += lzma.compress(p, format=lzma.FORMAT_XZ, check=(1, 4, 10)[k]) + b"\0" * (4 * k)
    files.append(("3 concatenated streams + stream padding", cat, b"".join(parts)))
    # multi-block streams assembled block by block
    blocks = [(text[i * 65536:(i + 1) * 65536], {}) for i in range(4)]
    blocks.append((text[262144:262144 + 1000], {"sizes": True}))
    blocks.append((b"", {}))
    blocks.append((rnd[:30000], {"sizes": True}))
    for chk in (1, 4):
        files.append((f"multi-block stream (7 blocks, one empty), check {chk}",
                      make_stream(blocks, chk), b"".join(d for d, _ in blocks)))
    # every block of this stream has the same chain: the reference (9.20 XzDec_Init ->
    # MixCoder_Free) aborts with a double free when consecutive blocks of one
    # stream change their filter chain, so such a file cannot be pinned
    mixed = [(xd[:40000], {"x86": 0}), (text[:5000], {"x86": 0}), (xd[40000:90000], {"x86": 0x2000}),
             (xd[90000:], {"x86": 0, "sizes": True})]
    files.append(("multi-block, x86 BCJ on all 4 blocks (start offsets 0 / 0x2000), check 10",
                  make_stream(mixed, 10), b"".join(d for d, _ in mixed)))
    many = [(native.gen("text", 950 + i, 1000 + 997 * i), {}) for i in range(24)]
    files.append(("24 small blocks, check 4", make_stream(many, 4), b"".join(d for d, _ in many)))

    # corrupt variants of two files
    base = [f for f in files if f[0].startswith("multi-block stream (7 blocks")][0][1]
    blk1 = make_stream(blocks[:1], 1)
    hdr = 12
    chk_at = hdr + len(make_block(blocks[0][0], 1)[0]) - 4  # the CRC-32 field of block 0

    def flip(b, at, mask):
        return b[:at] + bytes([b[at] ^ mask]) + b[at + 1:]

    corrupt = [
        ("corrupt: stream magic", flip(base, 0, 1), None),
        ("corrupt: LZMA2 data byte in block 0", flip(base, hdr + 40, 0x55), None),
        ("corrupt: check field of the only block", flip(blk1, chk_at, 0x80), None),
    ]

    blob = bytearray()
    cases = []
    for note, data, plain in files + corrupt:
        cap = (len(plain) if plain is not None else 400000) + 64
        out = ctypes.create_string_buffer(cap)
        dl, sl = ctypes.c_size_t(cap), ctypes.c_size_t(len(data))
        st, done = ctypes.c_int(-1), ctypes.c_int(0)
        res = lib.ref_xz_decode(out, ctypes.byref(dl), data, ctypes.byref(sl), ctypes.byref(st),
                                ctypes.byref(done))
        got = out.raw[:dl.value]
        if plain is not None:
            assert res == 0 and got == plain and done.value == 1, (note, res, dl.value)
            if "padding" not in note:  # Python's lzma stops at stream padding
                assert lzma.decompress(data, format=lzma.FORMAT_XZ) == plain, note  # liblzma
        cases.append({"note": note, "off": len(blob), "len": len(data), "res": res,
                      "status": st.value, "dest_len": dl.value, "src_len": sl.value,
                      "finished": done.value, "sha256": hashlib.sha256(got).hexdigest(),
                      "valid": plain is not None})
        blob += data

    # x86 BCJ: ragged sizes, carried state, both directions
    bcj = []
    sizes = [0, 4, 5, 6, 9, 17, 100, 1023, 4096, 65537, 31, 32, 33, 63, 64, 65, 1000, 5000]
    for k, n in enumerate(sizes):
        d = x86_like(960 + k, n) if n else b""
        if k >= 10:  # dense: an E8/E9 every 3 bytes (overlapping candidates, masks)
            b = bytearray(d)
            for i in range(0, n, 3):
                b[i] = 0xE8 if (i // 3 + k) % 2 else 0xE9
            d = bytes(b)
        for enc in (0, 1):
            for ip, st0 in ((0, 0), (0x401000, 5), (123, 7)):
                buf = ctypes.create_string_buffer(d, max(n, 1))
                st = ctypes.c_uint(st0)
                done = lib.ref_x86_convert(buf, n, ip, ctypes.byref(st), enc)
                bcj.append({"off": len(blob), "len": n, "ip": ip, "state_in": st0,
                            "encoding": enc, "done": done, "state_out": st.value,
                            "sha256": hashlib.sha256(buf.raw[:n]).hexdigest()})
        blob += d
    crc = []
    for n in (0, 1, 7, 8, 15, 16, 17, 2047, 2048, 2049, 6000, 100003):
        d = native.gen("random", 990 + n % 97, n) if n else b""
        crc.append({"off": len(blob), "len": n, "crc64": lib.ref_crc64(d, n)})
        assert lib.ref_crc64(d, n) == crc64(d)
        blob += d

    with open(os.path.join(HERE, "xz_blob.bin"), "wb") as f:
        f.write(blob)
    with open(os.path.join(HERE, "xz_cases.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden_xz.py",
                   "reference": "LZMA SDK 9.20 XzUnpacker_Code (XzDec.c), x86_Convert (Bra86.c), "
                                "Crc64Calc (XzCrc64.c) -- oracle/Makefile.ref",
                   "blob_sha256": hashlib.sha256(blob).hexdigest(), "xz": cases, "bcj": bcj,
                   "crc64": crc}, f, indent=0)
    print(f"{len(cases)} xz files, {len(bcj)} BCJ cases, {len(crc)} CRC-64 cases, "
          f"blob {len(blob)} bytes")


if __name__ == "__main__":
    main()

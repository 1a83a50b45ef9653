"""Generate tests/golden/sz_cases.json + sz_blob.bin from the REFERENCE 7z
reader (SzArEx_Open + SzArEx_Extract, 7zIn.c / 7zDec.c) compiled in place.

Run in the build container only (needs oracle/_ref/libref.so (container library) from
`make -f oracle/Makefile.ref`):

    python tests/golden/make_golden_7z.py

Archives are written here (tests/sevenzwrite.py) around
coder data from liblzma (LZMA1 with end marker, LZMA2) and from the
reference encoder (LzmaEnc.c, no end marker): single and multi-folder
archives, Copy / LZMA / LZMA2 / BCJ x86 + LZMA folders, folder and file
CRCs, empty files and directories, LZMA- and LZMA2-encoded headers, and
corrupt variants (signature, start header CRC, next header CRC, file CRC,
coder data, trailing pack bytes, truncation, an unsupported coder), and BCJ2
folders (streams from tests/bcj2enc.py: LZMA / LZMA2 / Copy coders, every or
no branch converted, encoded header) with their failure modes (short rc or
CALL stream, flipped rc byte, archive cut in the rc stream, PARAM).  For
every archive the reference's open result, per-file extract result and
size, the extracted bytes (files that extract OK, in file order) and the
raw UTF-16LE name buffer are recorded.
"""
import ctypes
import hashlib
import json
import os
import struct
import sys
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import native  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "lzma-sdk-zliblike_amd"))
import sevenzwrite as W  # noqa: E402
from make_golden_xz import x86_like  # noqa: E402

_sp = ctypes.POINTER(ctypes.c_size_t)


def ref_extract(lib, arc, max_files=4096):
    cap = 64 << 20
    out = ctypes.create_string_buffer(cap)
    ol = ctypes.c_size_t(0)
    fres = (ctypes.c_int * max_files)()
    fsz = (ctypes.c_uint64 * max_files)()
    nf = ctypes.c_uint(0)
    names = ctypes.create_string_buffer(1 << 20)
    nl = ctypes.c_size_t(0)
    r = lib.ref_7z_extract(arc, len(arc), out, cap, ctypes.byref(ol), fres, fsz, ctypes.byref(nf),
                           max_files, names, len(names), ctypes.byref(nl))
    n = nf.value
    return r, [fres[i] for i in range(n)], [fsz[i] for i in range(n)], out.raw[:ol.value], \
        names.raw[:nl.value]


def archives():
    text = native.gen("text", 700, 400000)
    rnd = native.gen("random", 701, 50000)
    xd = x86_like(702, 90000)
    A = []

    def files(prefix, *parts):
        return [(f"{prefix}/f{i}.txt", p) for i, p in enumerate(parts)]

    A.append(("LZMA (liblzma, end mark), 3 files", W.archive(
        [W.Folder(files("a", text[:10000], text[10000:30000], text[30000:30500]))])))
    props, packed = native.ref_encode(text[:60000], dict_size=1 << 16)
    A.append(("LZMA (reference encoder, no end mark), 2 files, folder CRC", W.archive(
        [W.Folder(files("b", text[:45000], text[45000:60000]), packed=packed, props=props,
                  crc=True)])))
    A.append(("LZMA2, 2 files", W.archive(
        [W.Folder(files("c", text[:70000], rnd[:20000]), method=W.M_LZMA2)])))
    A.append(("Copy folder, 2 files", W.archive(
        [W.Folder(files("d", rnd[:3000], text[:5000]), method=W.M_COPY)])))
    A.append(("BCJ x86 + LZMA, folder CRC", W.archive(
        [W.Folder(files("e", xd[:50000], xd[50000:]), bcj=True, crc=True)])))
    A.append(("BCJ x86 + LZMA2", W.archive(
        [W.Folder(files("e2", xd), method=W.M_LZMA2, bcj=True)])))
    props4, packed4 = native.ref_encode(text[:4096], dict_size=4096, lc=0, lp=0, pb=0)
    mixed = [
        W.Folder(files("m0", text[:4096]), packed=packed4, props=props4),
        W.Folder(files("m1", text[5000:9000], b"", text[9000:9100]), method=W.M_LZMA2, crc=True),
        W.Folder(files("m2", rnd[:1000]), method=W.M_COPY, crc=True),
        W.Folder(files("m3", xd[:20000]), bcj=True),
        W.Folder(files("m4", *[text[i * 997:(i + 1) * 997] for i in range(12)]), lc=1, lp=1, pb=1),
    ]
    A.append(("5 folders (LZMA lc0 4 KiB dict, LZMA2, Copy, BCJ, 12 files), empty file + dir",
              W.archive(mixed, empty=[("empty.txt", False), ("dir", True)])))
    A.append(("encoded header (LZMA), 5 folders", W.archive(mixed, encode_header=True)))
    A.append(("encoded header (LZMA2), 1 folder", W.archive(
        [W.Folder(files("h", text[:20000]))], encode_header=True, header_method=W.M_LZMA2)))
    A.append(("only empty entries", W.archive([], empty=[("a", False), ("b", True)])))
    A.append(("256 small files in one LZMA folder", W.archive(
        [W.Folder([(f"s/{i}", native.gen("text", 720 + i, 50 + 37 * i)) for i in range(256)])])))

    # unnamed stream files (no kName): the reader takes their count and sizes
    # from the substreams alone (7zIn.c:986-1104), however many there are
    A.append(("3000 unnamed files in one LZMA folder (no kName property)", W.archive(
        [W.Folder([("", native.gen("text", 760 + (i % 7), 1 + (i * 13) % 97)) for i in range(3000)])],
        names=False)))

    from make_golden_bra import branchy
    ad = branchy("ARM", 730, 70001)
    A.append(("ARM + LZMA, folder CRC", W.archive(
        [W.Folder(files("arm", ad[:30000], ad[30000:]), arm=True, crc=True)])))
    A.append(("ARM + LZMA2 and BCJ x86 + LZMA folders", W.archive(
        [W.Folder(files("a2", ad[:50000]), method=W.M_LZMA2, arm=True),
         W.Folder(files("b2", xd[:30000]), bcj=True)])))

    # BCJ2 folders (7zDec.c:412-440): streams from tests/bcj2enc.py
    import bcj2enc
    x2 = bcj2enc.x86_like(740, 120000)
    A.append(("BCJ2 (LZMA x3), 3 files, folder CRC", W.archive(
        [W.Bcj2Folder(files("j", x2[:40000], x2[40000:100000], x2[100000:]), crc=True)])))
    A.append(("BCJ2 (Copy JMP, Copy CALL, LZMA2 main), every branch converted", W.archive(
        [W.Bcj2Folder(files("j2", x2[:70000]), methods=(W.M_COPY, W.M_COPY, W.M_LZMA2),
                      convert=lambda p, o, rel: True)])))
    A.append(("BCJ2 + LZMA + Copy folders, encoded header", W.archive(
        [W.Folder(files("k1", text[:20000])),
         W.Bcj2Folder(files("k2", x2[:50000], x2[50000:60000]), methods=(W.M_LZMA2, W.M_LZMA, W.M_LZMA)),
         W.Folder(files("k3", rnd[:4000]), method=W.M_COPY, crc=True)], encode_header=True)))
    A.append(("BCJ2 with no branch converted, 1 file", W.archive(
        [W.Bcj2Folder(files("j3", x2[:30000]), convert=lambda p, o, rel: False)])))
    A.append(("BCJ2 over text (no branch opcodes)", W.archive(
        [W.Bcj2Folder(files("j4", text[:25000]))])))

    base = A[6][1]  # 5 folders

    def flip(b, at, mask=1):
        return b[:at] + bytes([b[at] ^ mask]) + b[at + 1:]

    def fix_start(b):
        """recompute the start header CRC after editing next-header fields"""
        return b[:8] + struct.pack("<I", zlib.crc32(b[12:32])) + b[12:]

    def fix_next(b):
        """recompute the next header CRC after editing the header"""
        off, size = struct.unpack("<QQ", b[12:28])
        h = b[32 + off:32 + off + size]
        return fix_start(b[:28] + struct.pack("<I", zlib.crc32(h)) + b[32:])

    C = []
    C.append(("corrupt: signature", flip(base, 2)))
    C.append(("corrupt: start header CRC", flip(base, 9)))
    C.append(("corrupt: next header CRC", flip(base, 28)))
    C.append(("corrupt: next header byte (CRC caught)", flip(base, len(base) - 5)))
    C.append(("corrupt: LZMA data in folder 0", flip(base, 32 + 20, 0x40)))
    m4_off = 32 + sum(len(f.packed) for f in mixed[:4])
    C.append(("corrupt: LZMA data in folder 4 (12 files)", flip(base, m4_off + 300, 0x10)))
    # a file CRC in the substreams digests: edit the header and fix its CRC
    one = W.archive([W.Folder(files("k", text[:3000], text[3000:7000]))])
    off, size = struct.unpack("<QQ", one[12:28])
    h = bytearray(one[32 + off:32 + off + size])
    crc1 = struct.pack("<I", zlib.crc32(text[3000:7000]))
    k = bytes(h).find(crc1)
    h[k] ^= 0xFF
    C.append(("corrupt: CRC of file 1 (header re-signed)",
              fix_next(one[:32 + off] + bytes(h) + one[32 + off + size:])))
    C.append(("truncated archive (header cut)", base[:len(base) - 7]))
    C.append(("truncated archive (pack data cut)", base[:200]))
    # a pack size one larger than the coder data (one trailing byte)
    f = W.Folder(files("t", text[:9000]))
    f.packed += b"\x55"
    C.append(("LZMA pack stream with a trailing byte", W.archive([f])))
    f = W.Folder(files("u", rnd[:500]), method=W.M_COPY)
    C.append(("Copy folder, unpack size != pack size", _copy_size_mismatch(f)))
    g = W.Folder(files("v", text[:500]))
    g.method = 0x030401  # PPMd: not built into the reference reader
    C.append(("unsupported coder (PPMd id)", W.archive([g, W.Folder(files("w", text[:800]))])))
    props_bad = b"\xe1" + struct.pack("<I", 1 << 16)  # lc/lp/pb byte >= 225
    C.append(("LZMA props byte >= 225", W.archive(
        [W.Folder(files("x", text[:800])), W.Folder(files("y", text[:900]), packed=packed,
                                                    props=props_bad)])))
    # BCJ2 failures: the rc stream short (Bcj2_Decode's RC_TEST), a Copy CALL
    # stream short (SzDecodeCopy size check), an rc bit flipped, the archive
    # cut inside the rc stream, the main coder larger than the folder (PARAM)
    C.append(("BCJ2: rc stream 3 bytes short", W.archive(
        [W.Bcj2Folder(files("q1", x2[:50000]), cut=(1, 3))])))
    C.append(("BCJ2: Copy CALL stream 4 bytes short", W.archive(
        [W.Bcj2Folder(files("q2", x2[:50000]), methods=(W.M_COPY, W.M_COPY, W.M_LZMA),
                      cut=(2, 4))])))
    bf = W.Bcj2Folder(files("q3", x2[:50000]), crc=True)
    arc = W.archive([W.Folder(files("q0", text[:3000])), bf])
    rc_at = 32 + len(W.Folder(files("q0", text[:3000])).packed) + len(bf.pack_streams()[0])
    C.append(("BCJ2: rc byte flipped (second folder)", flip(arc, rc_at + 40, 0x08)))
    C.append(("BCJ2: archive cut inside the rc stream", arc[:rc_at + 10]))
    bm = W.Bcj2Folder(files("q4", x2[:20000]))
    bm.main_size_delta = len(bm.data)  # main stream coder larger than the folder output
    C.append(("BCJ2: main coder unpack size > folder size", W.archive([bm])))
    return A, C


def _copy_size_mismatch(f):
    """A Copy folder whose unpack size is one more than its pack size."""
    f.data = f.data + b"\0"
    f.files = [(f.files[0][0], f.files[0][1] + b"\0")]
    return W.archive([f])


def main():
    lib = native.ref_cont()
    lib.ref_7z_extract.restype = ctypes.c_int
    lib.ref_7z_extract.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                   ctypes.c_size_t, _sp, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.POINTER(ctypes.c_uint), ctypes.c_uint, ctypes.c_char_p,
                                   ctypes.c_size_t, _sp]
    A, C = archives()
    blob = bytearray()
    cases = []
    for valid, lst in ((True, A), (False, C)):
        for note, arc in lst:
            r, fres, fsz, out, names = ref_extract(lib, arc)
            if valid:
                assert r == 0 and all(x == 0 for x in fres), (note, r, fres)
            cases.append({"note": note, "off": len(blob), "len": len(arc), "open_res": r,
                          "file_res": fres, "file_size": fsz, "out_len": len(out),
                          "sha256": hashlib.sha256(out).hexdigest(),
                          "names_sha256": hashlib.sha256(names).hexdigest(),
                          "names_len": len(names), "valid": valid})
            blob += arc
            print(f"{note}: open {r}, files {len(fres)}, res {sorted(set(fres))}, out {len(out)}")
    with open(os.path.join(HERE, "sz_blob.bin"), "wb") as f:
        f.write(blob)
    with open(os.path.join(HERE, "sz_cases.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden_7z.py",
                   "reference": "LZMA SDK 9.20 fork SzArEx_Open / SzArEx_Extract (7zIn.c, 7zDec.c) "
                                "-- oracle/Makefile.ref",
                   "blob_sha256": hashlib.sha256(blob).hexdigest(), "cases": cases}, f, indent=0)
    print(f"{len(cases)} archives, blob {len(blob)} bytes")


if __name__ == "__main__":
    main()

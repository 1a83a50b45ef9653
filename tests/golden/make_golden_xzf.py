"""Generate tests/golden/xzf_cases.json + xzf_blob.bin: xz files whose blocks
carry the filters beyond x86 (Delta, PPC, IA64, ARM, ARMT, SPARC and chains
of them), decoded by the REFERENCE xz decoder (XzUnpacker_Code, XzDec.c, whose
BraState_Code drives Bra.c / BraIA64.c / Delta.c).

Run in the build container only (needs oracle/_ref/libref.so (container library) from
`make -f oracle/Makefile.ref`):

    python tests/golden/make_golden_xzf.py

Files are written by liblzma (Python's lzma module); every one decodes
identically through the reference and through liblzma.  Branchy inputs come
from make_golden_bra.branchy; unsupported props (a misaligned ARM start
offset, a 2-byte delta prop) record the reference's error code.
"""
import ctypes
import hashlib
import json
import lzma
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
import native  # noqa: E402
from make_golden_bra import branchy  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "lzma-sdk-zliblike_amd"))
from xzwrite import make_stream  # noqa: E402,F401

_sp = ctypes.POINTER(ctypes.c_size_t)
_ip = ctypes.POINTER(ctypes.c_int)
LZ2 = {"id": lzma.FILTER_LZMA2, "preset": 6}
FID = {"PPC": lzma.FILTER_POWERPC, "IA64": lzma.FILTER_IA64, "ARM": lzma.FILTER_ARM,
       "ARMT": lzma.FILTER_ARMTHUMB, "SPARC": lzma.FILTER_SPARC}


def main():
    lib = native.ref_cont()
    lib.ref_xz_decode.restype = ctypes.c_int
    lib.ref_xz_decode.argtypes = [ctypes.c_char_p, _sp, ctypes.c_char_p, _sp, _ip, _ip]
    text = native.gen("text", 1900, 200000)
    files = []  # (note, bytes, plain or None, [(id, prop)...] expected pre-filters)
    for k, (name, fid) in enumerate(FID.items()):
        d = branchy(name, 3000 + k, 90000 + 13 * k)
        files.append((f"{name} + LZMA2, crc64", lzma.compress(
            d, format=lzma.FORMAT_XZ, check=lzma.CHECK_CRC64,
            filters=[{"id": fid}, LZ2]), d, [(fid, 0)]))
        so = 0x1000 if name != "IA64" else 0x10000
        files.append((f"{name} start_offset {so:#x} + LZMA2, crc32", lzma.compress(
            d[:40001], format=lzma.FORMAT_XZ, check=lzma.CHECK_CRC32,
            filters=[{"id": fid, "start_offset": so}, LZ2]), d[:40001], [(fid, so)]))
    for dist in (1, 2, 4, 7, 256, 8, 32):
        d = text[:60000 + dist]
        files.append((f"Delta dist {dist} + LZMA2, sha256", lzma.compress(
            d, format=lzma.FORMAT_XZ, check=lzma.CHECK_SHA256,
            filters=[{"id": lzma.FILTER_DELTA, "dist": dist}, LZ2]), d,
            [(lzma.FILTER_DELTA, dist)]))
    d = branchy("ARM", 3100, 70000)
    files.append(("chain Delta 4, ARM, LZMA2, crc64", lzma.compress(
        d, format=lzma.FORMAT_XZ, check=lzma.CHECK_CRC64,
        filters=[{"id": lzma.FILTER_DELTA, "dist": 4}, {"id": lzma.FILTER_ARM}, LZ2]), d,
        [(lzma.FILTER_DELTA, 4), (lzma.FILTER_ARM, 0)]))
    d = branchy("IA64", 3101, 50000)
    files.append(("chain x86, SPARC, Delta 3, LZMA2, crc32", lzma.compress(
        d, format=lzma.FORMAT_XZ, check=lzma.CHECK_CRC32,
        filters=[{"id": lzma.FILTER_X86}, {"id": lzma.FILTER_SPARC},
                 {"id": lzma.FILTER_DELTA, "dist": 3}, LZ2]), d,
        [(lzma.FILTER_X86, 0), (lzma.FILTER_SPARC, 0), (lzma.FILTER_DELTA, 3)]))
    files.append(("ARMT + LZMA2, empty input", lzma.compress(
        b"", format=lzma.FORMAT_XZ, filters=[{"id": lzma.FILTER_ARMTHUMB}, LZ2]), b"",
        []))
    # unsupported props, patched in the block header (header CRC recomputed)
    base = lzma.compress(text[:5000], format=lzma.FORMAT_XZ, check=lzma.CHECK_CRC32,
                         filters=[{"id": lzma.FILTER_ARM, "start_offset": 0x100}, LZ2])
    bad = bytearray(base)
    hs = (bad[12] + 1) * 4
    # header: size, flags, [filter id 7, props size 4, offset LE32], [0x21, 1, dict], pad, crc
    at = bytes(bad[12:12 + hs]).index(bytes([7, 4, 0, 1, 0, 0])) + 12 + 2
    bad[at] = 2  # start offset 0x102: not a multiple of 4
    import zlib
    bad[12 + hs - 4:12 + hs] = zlib.crc32(bytes(bad[12:12 + hs - 4])).to_bytes(4, "little")
    files.append(("ARM start offset 0x102 (misaligned): unsupported", bytes(bad), None, None))

    blob = bytearray()
    cases = []
    for note, data, plain, chain in files:
        cap = (len(plain) if plain is not None else 400000) + 64
        out = ctypes.create_string_buffer(cap)
        dl, sl = ctypes.c_size_t(cap), ctypes.c_size_t(len(data))
        st, done = ctypes.c_int(-1), ctypes.c_int(0)
        res = lib.ref_xz_decode(out, ctypes.byref(dl), data, ctypes.byref(sl), ctypes.byref(st),
                                ctypes.byref(done))
        got = out.raw[:dl.value]
        if plain is not None:
            assert res == 0 and got == plain and done.value == 1, (note, res, dl.value)
            assert lzma.decompress(data, format=lzma.FORMAT_XZ) == plain, note  # liblzma
        else:
            assert res != 0, note
        cases.append({"note": note, "off": len(blob), "len": len(data), "res": res,
                      "status": st.value, "dest_len": dl.value, "src_len": sl.value,
                      "finished": done.value, "sha256": hashlib.sha256(got).hexdigest(),
                      "valid": plain is not None, "chain": chain})
        blob += data
    with open(os.path.join(HERE, "xzf_blob.bin"), "wb") as f:
        f.write(blob)
    with open(os.path.join(HERE, "xzf_cases.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden_xzf.py",
                   "reference": "LZMA SDK 9.20 XzUnpacker_Code (XzDec.c) with BraState_Code "
                                "(Bra.c, BraIA64.c, Delta.c) -- oracle/Makefile.ref",
                   "blob_sha256": hashlib.sha256(blob).hexdigest(), "xz": cases}, f, indent=0)
    print(f"{len(cases)} xz files, blob {len(blob)} bytes; results "
          f"{sorted(set(c['res'] for c in cases))}")


if __name__ == "__main__":
    main()

"""xzwrite -- writes xz files block by block (the xz file format: stream
header, block headers with [x86 BCJ,] LZMA2 filter chains, block padding,
checks, index, footer) around raw LZMA2 data from liblzma (Python lzma,
FORMAT_RAW).  A workload writer for bench.py --config xz and the xz test
fixtures (tests/golden/make_golden_xz.py); not part of the decode path.
"""
import hashlib
import lzma
import struct
import zlib


def varint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def crc64(data):
    t = []
    for i in range(256):
        r = i
        for _ in range(8):
            r = (r >> 1) ^ (0xC96C5795D7870F42 if r & 1 else 0)
        t.append(r)
    c = 0xFFFFFFFFFFFFFFFF
    for b in data:
        c = t[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFFFFFFFFFF


CHECK_SIZE = {0: 0, 1: 4, 4: 8, 10: 32}


def check_value(kind, data):
    if kind == 0:
        return b""
    if kind == 1:
        return struct.pack("<I", zlib.crc32(data))
    if kind == 4:
        return struct.pack("<Q", crc64(data))
    return hashlib.sha256(data).digest()


def lzma2_prop(dict_size):
    for p in range(41):
        if ((2 | (p & 1)) << (p // 2 + 11)) >= dict_size:
            return p
    return 40


def make_block(data, check, dict_size=1 << 20, x86=None, sizes=False):
    """One xz block: header (filters [x86 BCJ,] LZMA2), LZMA2 data, padding, check."""
    filters = []
    if x86 is not None:
        f = {"id": lzma.FILTER_X86}
        if x86:
            f["start_offset"] = x86
        filters.append(f)
    filters.append({"id": lzma.FILTER_LZMA2, "preset": 6, "dict_size": dict_size})
    raw = lzma.compress(data, format=lzma.FORMAT_RAW, filters=filters)
    flt = b""
    if x86 is not None:
        flt += varint(4) + ((varint(4) + struct.pack("<I", x86)) if x86 else varint(0))
    flt += varint(0x21) + varint(1) + bytes([lzma2_prop(dict_size)])
    flags = len(filters) - 1
    opt = b""
    if sizes:
        flags |= 0x40 | 0x80
    body_len = 1 + 1 + len(flt)
    # sizes depend on the header size only through the pack size field, not the total
    if sizes:
        opt = varint(len(raw)) + varint(len(data))
    hsize = (body_len + len(opt) + 4 + 3) // 4 * 4
    h = bytes([hsize // 4 - 1, flags]) + opt + flt
    h += b"\0" * (hsize - 4 - len(h))
    h += struct.pack("<I", zlib.crc32(h))
    blk = h + raw + b"\0" * ((-len(h) - len(raw)) % 4) + check_value(check, data)
    unpadded = len(h) + len(raw) + CHECK_SIZE[check]
    return blk, unpadded, len(data)


def make_stream(blocks, check):
    """Assemble a stream from (data, kwargs) blocks."""
    flags = bytes([0, check])
    out = b"\xfd7zXZ\0" + flags + struct.pack("<I", zlib.crc32(flags))
    recs = []
    for data, kw in blocks:
        b, unp, n = make_block(data, check, **kw)
        out += b
        recs.append((unp, n))
    idx = b"\0" + varint(len(recs)) + b"".join(varint(u) + varint(n) for u, n in recs)
    idx += b"\0" * ((-len(idx)) % 4)
    idx += struct.pack("<I", zlib.crc32(idx))
    out += idx
    back = struct.pack("<I", len(idx) // 4 - 1) + flags
    out += struct.pack("<I", zlib.crc32(back)) + back + b"YZ"
    return out

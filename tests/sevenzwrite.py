"""sevenzwrite -- writes 7z archives (format 0.4: signature header, packed
streams, header with pack / unpack / substreams info and file names,
optionally an LZMA-encoded header) around coder data from liblzma (Python
lzma, FORMAT_RAW: LZMA1 with end marker, LZMA2) or from any caller-supplied
encoder.  A workload writer for bench.py --config 7z and the 7z fixtures
(tests/golden/make_golden_7z.py); not part of the decode path.

Folder layouts follow what the reference reader accepts
(CheckSupportedFolder, 7zDec.c:269-322): one coder (Copy / LZMA / LZMA2), or
the main coder followed by a BCJ x86 coder bound to its output
(bind pair in 1 <- out 0).
"""
import lzma
import struct
import zlib

# property ids (7z.h:17-45)
END, HEADER, MAIN_STREAMS, FILES, PACK_INFO, UNPACK_INFO, SUBSTREAMS = 0, 1, 4, 5, 6, 7, 8
SIZE, CRC, FOLDER, CODERS_UNPACK_SIZE, NUM_UNPACK_STREAM = 9, 10, 11, 12, 13
EMPTY_STREAM, EMPTY_FILE, NAME, ENCODED_HEADER = 14, 15, 17, 23

M_COPY, M_LZMA, M_LZMA2, M_BCJ, M_ARM = 0, 0x030101, 0x21, 0x03030103, 0x03030501


def number(v):
    """7z variable-length number (SzReadNumber, 7zIn.c:348-369)."""
    for n in range(9):
        if n == 8:
            return bytes([0xFF]) + struct.pack("<Q", v)
        if (v >> (8 * n)) < (1 << (7 - n)):
            first = ((0xFF00 >> n) & 0xFF) | (v >> (8 * n))
            return bytes([first]) + (v & ((1 << (8 * n)) - 1)).to_bytes(n, "little")


def bools(v):
    out = bytearray((len(v) + 7) // 8)
    for i, b in enumerate(v):
        if b:
            out[i // 8] |= 0x80 >> (i % 8)
    return bytes(out)


def method_id(m):
    if m == 0:
        return b"\0"
    n = (m.bit_length() + 7) // 8
    return m.to_bytes(n, "big")


def lzma_props(dict_size=1 << 16, lc=3, lp=0, pb=2):
    return bytes([(pb * 5 + lp) * 9 + lc]) + struct.pack("<I", dict_size)


def lzma2_prop(dict_size):
    for p in range(41):
        if ((2 | (p & 1)) << (p // 2 + 11)) >= dict_size:
            return p
    return 40


def encode(method, data, dict_size=1 << 16, lc=3, lp=0, pb=2):
    """(packed bytes, props) for one main coder via liblzma raw streams."""
    if method == M_COPY:
        return data, b""
    if method == M_LZMA:
        f = {"id": lzma.FILTER_LZMA1, "dict_size": dict_size, "lc": lc, "lp": lp, "pb": pb}
        return (lzma.compress(data, format=lzma.FORMAT_RAW, filters=[f]),
                lzma_props(dict_size, lc, lp, pb))
    if method == M_LZMA2:
        f = {"id": lzma.FILTER_LZMA2, "dict_size": dict_size}
        return (lzma.compress(data, format=lzma.FORMAT_RAW, filters=[f]),
                bytes([lzma2_prop(dict_size)]))
    raise ValueError(method)


def x86_encode(data, fid=lzma.FILTER_X86):
    f = [{"id": fid}, {"id": lzma.FILTER_LZMA2, "dict_size": 1 << 16}]
    raw = lzma.compress(data, format=lzma.FORMAT_RAW, filters=f)
    # liblzma cannot emit the filter alone: decode LZMA2 only to get x86(data)
    return lzma.decompress(raw, format=lzma.FORMAT_RAW,
                           filters=[{"id": lzma.FILTER_LZMA2, "dict_size": 1 << 16}])


def coder(m, props):
    b = len(method_id(m)) | (0x20 if props else 0)
    out = bytes([b]) + method_id(m)
    if props:
        out += number(len(props)) + props
    return out


class Folder:
    """One folder: `files` (list of (name, bytes)), packed with `packed`
    (bytes) by `method` with `props`; `bcj` adds the x86 coder, `arm` the
    ARM one; `crc` writes the folder CRC (unpack CRC) too."""

    def __init__(self, files, method=M_LZMA, packed=None, props=None, bcj=False, crc=False,
                 arm=False, **enc):
        self.files, self.method, self.bcj, self.crc = files, method, bcj or arm, crc
        self.filter = M_ARM if arm else M_BCJ
        self.data = b"".join(d for _, d in files)
        if packed is None:
            src = (x86_encode(self.data, lzma.FILTER_ARM if arm else lzma.FILTER_X86)
                   if self.bcj else self.data)
            packed, props = encode(method, src, **enc)
        self.packed, self.props = packed, props

    def coders(self):
        if not self.bcj:
            return number(1) + coder(self.method, self.props)
        # coder 0 = main, coder 1 = BCJ; bind pair: in 1 <- out 0
        return number(2) + coder(self.method, self.props) + coder(self.filter, b"") + number(1) + number(0)

    def unpack_sizes(self):
        n = len(self.data)
        return number(n) + (number(n) if self.bcj else b"")

    def pack_streams(self):
        return [self.packed]


M_BCJ2 = 0x0303011B


class Bcj2Folder:
    """A BCJ2 folder in the only layout the 9.20 reader accepts
    (CheckSupportedFolder, 7zDec.c:303-319): coders 0, 1, 2 = the JMP, CALL
    and main streams (each Copy / LZMA / LZMA2), coder 3 = BCJ2 (4 in, 1 out);
    pack streams in order: main (coder 2), the raw rc stream, CALL (coder 1),
    JMP (coder 0).  The streams come from tests/bcj2enc.py.  `methods` gives
    the (jump, call, main) coders; `cut` trims pack stream k by n bytes."""

    def __init__(self, files, methods=(M_LZMA, M_LZMA, M_LZMA), crc=False, convert=None,
                 cut=None, main_dict=1 << 16):
        import bcj2enc
        self.files, self.crc, self.bcj = files, crc, False
        self.data = b"".join(d for _, d in files)
        m, c, j, r = bcj2enc.encode(self.data, convert)
        self.raw = (j, c, m)  # coder 0, 1, 2 outputs
        self.rc = r
        self.methods = methods
        self.enc = []
        for k, (meth, raw) in enumerate(zip(methods, self.raw)):
            if meth == M_COPY:
                self.enc.append((raw, b""))
            else:
                self.enc.append(encode(meth, raw, dict_size=main_dict if k == 2 else 1 << 16,
                                       **({"lc": 0, "lp": 2} if k < 2 and meth == M_LZMA else {})))
        streams = [self.enc[2][0], self.rc, self.enc[1][0], self.enc[0][0]]
        if cut:
            k, n = cut
            streams[k] = streams[k][:len(streams[k]) - n]
        self._packs = streams
        self.packed = b"".join(streams)

    def coders(self):
        bid = method_id(M_BCJ2)
        out = number(4)
        for meth, (_, props) in zip(self.methods, self.enc):
            out += coder(meth, props)
        out += bytes([len(bid) | 0x10]) + bid + number(4) + number(1)
        for i, o in ((5, 0), (4, 1), (3, 2)):   # bind pairs: in <- out
            out += number(i) + number(o)
        out += b"".join(number(x) for x in (2, 6, 1, 0))  # pack stream -> in index
        return out

    def unpack_sizes(self):
        sizes = [len(x) for x in self.raw] + [len(self.data)]
        if getattr(self, "main_size_delta", 0):
            sizes[2] += self.main_size_delta
        return b"".join(number(x) for x in sizes)

    def pack_streams(self):
        return self._packs


def streams_info(folders, pack_pos, substreams=True):
    packs = [p for f in folders for p in f.pack_streams()]
    out = bytes([PACK_INFO]) + number(pack_pos) + number(len(packs)) + bytes([SIZE])
    out += b"".join(number(len(p)) for p in packs) + bytes([END])
    out += bytes([UNPACK_INFO, FOLDER]) + number(len(folders)) + b"\0"
    out += b"".join(f.coders() for f in folders)
    out += bytes([CODERS_UNPACK_SIZE]) + b"".join(f.unpack_sizes() for f in folders)
    if any(f.crc for f in folders):
        out += bytes([CRC, 0]) + bools([f.crc for f in folders])
        out += b"".join(struct.pack("<I", zlib.crc32(f.data)) for f in folders if f.crc)
    out += bytes([END])
    if substreams:
        out += bytes([SUBSTREAMS, NUM_UNPACK_STREAM])
        out += b"".join(number(len([1 for _, d in f.files if d is not None])) for f in folders)
        sizes = b""
        for f in folders:
            ds = [d for _, d in f.files if d is not None]
            sizes += b"".join(number(len(d)) for d in ds[:-1])
        out += bytes([SIZE]) + sizes
        dig = []
        for f in folders:
            ds = [d for _, d in f.files if d is not None]
            if len(ds) == 1 and f.crc:
                continue
            dig += [zlib.crc32(d) for d in ds]
        out += bytes([CRC, 1]) + b"".join(struct.pack("<I", c) for c in dig) + bytes([END])
    return out + bytes([END])


def header(folders, empty=(), pack_pos=0, names=True):
    """The plain header; `empty` lists (name, is_dir) entries without data,
    written after the folders' files; names=False leaves out the kName
    property (files known only by their substream sizes)."""
    want_names = names
    names = [n for f in folders for n, _ in f.files] + [n for n, _ in empty]
    nfiles = len(names)
    out = bytes([HEADER, MAIN_STREAMS]) + streams_info(folders, pack_pos)
    out += bytes([FILES]) + number(nfiles)
    if empty:
        flags = [False] * (nfiles - len(empty)) + [True] * len(empty)
        v = bools(flags)
        out += bytes([EMPTY_STREAM]) + number(len(v)) + v
        v = bools([not d for _, d in empty])
        out += bytes([EMPTY_FILE]) + number(len(v)) + v
    if want_names:
        nb = b"".join(n.encode("utf-16-le") + b"\0\0" for n in names)
        out += bytes([NAME]) + number(len(nb) + 1) + b"\0" + nb
    return out + bytes([END, END])


def archive(folders, empty=(), encode_header=False, header_method=M_LZMA, names=True):
    """A whole .7z archive: signature header, the folders' packed streams,
    the (optionally LZMA-encoded) header."""
    body = b"".join(f.packed for f in folders)
    hdr = header(folders, empty, names=names)
    if encode_header:
        hf = Folder([("", hdr)], method=header_method, crc=True)
        pos = len(body)
        body += hf.packed
        hdr = bytes([ENCODED_HEADER]) + streams_info([hf], pos, substreams=False)
    start = struct.pack("<QQI", len(body), len(hdr), zlib.crc32(hdr))
    sig = b"7z\xbc\xaf\x27\x1c\x00\x04" + struct.pack("<I", zlib.crc32(start)) + start
    return sig + body + hdr

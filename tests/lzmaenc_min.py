"""Symbol-level LZMA encoder -- TEST INFRASTRUCTURE (fixture generation only).

Writes an LZMA stream from an explicit list of symbols (literals and plain
matches with chosen distances and lengths), so a test can place a match
exactly where it wants one.  Its probability model is the decoder's
(LzmaDec.c:131-426: IsMatch / IsRep, the literal and matched-literal trees,
the length coder, slot / SpecPos / direct / align distance coding), and it
tracks the bytes a DECODER produces -- including a decoder whose dictionary
is a ring smaller than the distances it is asked to reach (LzmaDec_DecodeToBuf
over a caller-owned `dic` of `ring` bytes), where the reference reads the ring
slot `dicPos - rep0 + dicBufSize` (LzmaDec.c:176, :388-407) rather than the
true history byte.  Parity is pinned on the reference's own LzmaDec.c decoding
these streams (tests/test_dropin_mirror.py), never on this encoder.
"""
import random

K_TOP = 1 << 24


class _Rc:
    def __init__(self):
        self.low, self.range, self.cache, self.cache_size = 0, 0xFFFFFFFF, 0, 1
        self.out = bytearray()
        self.probs = {}

    def _shift_low(self):
        if self.low < 0xFF000000 or self.low >= (1 << 32):
            carry = self.low >> 32
            temp = self.cache
            while True:
                self.out.append((temp + carry) & 0xFF)
                temp = 0xFF
                self.cache_size -= 1
                if self.cache_size == 0:
                    break
            self.cache = (self.low >> 24) & 0xFF
        self.cache_size += 1
        self.low = (self.low & 0x00FFFFFF) << 8

    def bit(self, key, b):
        p = self.probs.get(key, 1024)
        bound = (self.range >> 11) * p
        if b == 0:
            self.range = bound
            self.probs[key] = p + ((2048 - p) >> 5)
        else:
            self.low += bound
            self.range -= bound
            self.probs[key] = p - (p >> 5)
        while self.range < K_TOP:
            self.range = (self.range << 8) & 0xFFFFFFFF
            self._shift_low()

    def direct(self, v, n):
        for i in reversed(range(n)):
            self.range >>= 1
            if (v >> i) & 1:
                self.low += self.range
            while self.range < K_TOP:
                self.range = (self.range << 8) & 0xFFFFFFFF
                self._shift_low()

    def tree(self, pre, v, bits):
        m = 1
        for i in reversed(range(bits)):
            b = (v >> i) & 1
            self.bit((pre, m), b)
            m = (m << 1) | b

    def rtree(self, pre, v, bits):
        m = 1
        for i in range(bits):
            b = (v >> i) & 1
            self.bit((pre, m), b)
            m = (m << 1) | b

    def flush(self):
        for _ in range(5):
            self._shift_low()
        return bytes(self.out)


class Encoder:
    """Encode symbols while modelling the decoder's output in a dictionary of
    `ring` bytes (0: a flat dictionary)."""

    def __init__(self, lc=3, lp=0, pb=2, ring=0):
        self.lc, self.lp, self.pb = lc, lp, pb
        self.ring = ring
        self.rc = _Rc()
        self.state = 0
        self.reps = [1, 1, 1, 1]
        self.total = 0          # processedPos
        self.out = bytearray()  # what the decoder outputs, in order
        self.dic = bytearray(ring) if ring else None

    # the decoder's dictionary byte at distance d before the next position
    def back(self, d):
        if not self.ring:
            return self.out[-d]
        q = self.total % self.ring
        i = q - d + (self.ring if q < d else 0)
        if i < 0:
            raise ValueError("ring read out of range (the reference would read outside dic)")
        return self.dic[i]

    def _put(self, b):
        if self.ring:
            self.dic[self.total % self.ring] = b
        self.out.append(b)
        self.total += 1

    def literal(self, byte):
        ps = self.total & ((1 << self.pb) - 1)
        self.rc.bit(("M", self.state, ps), 0)
        prev = self.back(1) if self.total else 0
        ctx = ((self.total & ((1 << self.lp) - 1)) << self.lc) + (prev >> (8 - self.lc))
        if self.state < 7:
            sym = 1
            for i in reversed(range(8)):  # the plain tree: cells ctx * 0x300 + sym
                b = (byte >> i) & 1
                self.rc.bit(("L", ctx, sym), b)
                sym = (sym << 1) | b
        else:
            mb = self.back(self.reps[0])
            offs, sym = 0x100, 1
            for i in reversed(range(8)):
                b = (byte >> i) & 1
                mb <<= 1
                mbit = mb & offs
                self.rc.bit(("L", ctx, offs + mbit + sym), b)
                sym = (sym << 1) | b
                offs = (offs & mbit) if b else (offs & ~mbit)
        self.state = 0 if self.state < 4 else (self.state - 3 if self.state < 10 else self.state - 6)
        self._put(byte)

    def _length(self, ln, ps):
        v = ln - 2
        if v < 8:
            self.rc.bit(("Lc",), 0)
            self.rc.tree(("Llo", ps), v, 3)
        elif v < 16:
            self.rc.bit(("Lc",), 1)
            self.rc.bit(("Lc2",), 0)
            self.rc.tree(("Lmid", ps), v - 8, 3)
        else:
            self.rc.bit(("Lc",), 1)
            self.rc.bit(("Lc2",), 1)
            self.rc.tree(("Lhi",), v - 16, 8)

    def match(self, dist, ln):
        """A plain match (IsRep = 0): rep0 = dist, ln bytes (2..273)."""
        assert 2 <= ln <= 273 and 1 <= dist <= self.total
        ps = self.total & ((1 << self.pb) - 1)
        self.rc.bit(("M", self.state, ps), 1)
        self.rc.bit(("R", self.state), 0)
        self._length(ln, ps)
        d = dist - 1
        slot = d if d < 4 else (d.bit_length() - 1) * 2 + ((d >> (d.bit_length() - 2)) & 1)
        self.rc.tree(("S", min(ln - 2, 3)), slot, 6)
        if slot >= 4:
            nb = (slot >> 1) - 1
            base = (2 | (slot & 1)) << nb
            rest = d - base
            if slot < 14:
                self.rc.rtree(("SP", base - slot), rest, nb)
            else:
                self.rc.direct(rest >> 4, nb - 4)
                self.rc.rtree(("A",), rest & 15, 4)
        self.reps = [dist] + self.reps[:3]
        self.state = 7 if self.state < 7 else 10
        for _ in range(ln):
            self._put(self.back(dist))

    def finish(self):
        return self.rc.flush()


def props(lc, lp, pb, dict_size):
    return bytes([(pb * 5 + lp) * 9 + lc]) + int(dict_size).to_bytes(4, "little")


def ring_reach_stream(seed, ring=4096, far=5096, total=None, lc=3, lp=0, pb=2):
    """A stream whose matches at distance `far` > `ring` read, in a decoder with
    a `ring`-byte dictionary ring, the ring slot the reference reads (the byte
    at distance far - ring), never outside the ring: a far match starts at a
    ring position >= far - ring and ends inside the ring; a matched literal
    against rep0 = far comes only from such positions; elsewhere short matches
    (distance <= 8) reset rep0.  Returns (stream, props, the decoder's output)."""
    rng = random.Random(seed)
    total = total or 5 * ring
    e = Encoder(lc, lp, pb, ring)
    for _ in range(ring):  # fill the ring
        e.literal(rng.randrange(256))
    low = far - ring
    while e.total < total:
        q = e.total % ring
        left = total - e.total
        r0_ok = e.reps[0] <= ring or q >= e.reps[0] - ring
        if q >= low and ring - q >= 2 and left >= 2 and rng.random() < 0.5:
            e.match(far, min(rng.randrange(2, 40), ring - q, left, 273))
        elif e.state < 7 or r0_ok:
            e.literal(rng.randrange(256))
        elif left >= 2:
            # rep0 = far is out of reach from here: a short match resets it
            e.match(rng.randrange(1, 9), min(rng.randrange(2, 12), left))
        else:
            break
    return e.finish(), props(lc, lp, pb, 1 << 16), bytes(e.out)


def ring_decode(lib, comp, props, ring, out_total, in_chunk, out_chunk):
    """The fork's zlib-like loop (LzmaDec_DecodeToBuf, LzmaDec.c:840-878) over a
    caller-owned dictionary ring of `ring` bytes (LzmaDec_AllocateProbs + its
    own `dic`, as LzmaDec.h allows), through `lib`: liblzmagpu.so or the
    reference's LzmaDec.c compiled in place (oracle/_ref/libref_lzma.so).
    Returns (trace of (res, status, destLen, srcLen) per call, output)."""
    import ctypes
    import lzmagpu as L
    vp = ctypes.c_void_p
    for name, args in (("LzmaDec_AllocateProbs", [vp, ctypes.c_char_p, ctypes.c_uint, vp]),
                       ("LzmaDec_Init", [vp]),
                       ("LzmaDec_DecodeToBuf", [vp, vp, vp, vp, vp, ctypes.c_int, vp]),
                       ("LzmaDec_FreeProbs", [vp, vp])):
        getattr(lib, name).argtypes = args
    lib.LzmaDec_AllocateProbs.restype = ctypes.c_int
    lib.LzmaDec_DecodeToBuf.restype = ctypes.c_int
    d = L.CLzmaDec()
    d.dic = None
    d.probs = None
    r = lib.LzmaDec_AllocateProbs(ctypes.byref(d), bytes(props), len(props), ctypes.byref(L.g_alloc))
    if r != 0:
        return [(r, -1, 0, 0)], b""
    dic = ctypes.create_string_buffer(ring)
    d.dic = ctypes.addressof(dic)
    d.dicBufSize = ring
    lib.LzmaDec_Init(ctypes.byref(d))
    src = ctypes.create_string_buffer(bytes(comp), len(comp))
    out = ctypes.create_string_buffer(max(out_total, 1))
    trace, ip, op = [], 0, 0
    try:
        while True:
            sl = ctypes.c_size_t(min(in_chunk, len(comp) - ip))
            n = min(out_chunk, out_total - op)
            dl = ctypes.c_size_t(n)
            fin = 1 if op + n == out_total else 0
            st = ctypes.c_int(-1)
            r = lib.LzmaDec_DecodeToBuf(ctypes.byref(d), ctypes.addressof(out) + op, ctypes.byref(dl),
                                        ctypes.addressof(src) + ip, ctypes.byref(sl), fin,
                                        ctypes.byref(st))
            trace.append((r, st.value, dl.value, sl.value))
            ip += sl.value
            op += dl.value
            if r != 0 or op == out_total or (dl.value == 0 and sl.value == 0) or len(trace) > 100000:
                break
    finally:
        lib.LzmaDec_FreeProbs(ctypes.byref(d), ctypes.byref(L.g_alloc))
    return trace, out.raw[:op]


def dic_calls(lib, comp, props, out_total, win, edit=None, max_calls=100000):
    """LzmaDec_DecodeToDic calls over a caller-owned flat dictionary of
    `out_total` bytes (LzmaDec_AllocateProbs + own dic), input in windows of at
    most `win` bytes, FINISH_ANY, through `lib`; edit(k, dec) runs on the host
    CLzmaDec between calls k and k + 1 (a host-side change both libraries see
    alike).  Returns (trace of (res, status, srcLen, dicPos), dictionary)."""
    import ctypes
    import lzmagpu as L
    vp = ctypes.c_void_p
    for name, args in (("LzmaDec_AllocateProbs", [vp, ctypes.c_char_p, ctypes.c_uint, vp]),
                       ("LzmaDec_Init", [vp]),
                       ("LzmaDec_DecodeToDic", [vp, ctypes.c_size_t, vp, vp, ctypes.c_int, vp]),
                       ("LzmaDec_FreeProbs", [vp, vp])):
        getattr(lib, name).argtypes = args
    lib.LzmaDec_AllocateProbs.restype = ctypes.c_int
    lib.LzmaDec_DecodeToDic.restype = ctypes.c_int
    d = L.CLzmaDec()
    d.dic = None
    d.probs = None
    r = lib.LzmaDec_AllocateProbs(ctypes.byref(d), bytes(props), len(props), ctypes.byref(L.g_alloc))
    if r != 0:
        return [(r, -1, 0, 0)], b""
    dic = ctypes.create_string_buffer(max(out_total, 1))
    d.dic = ctypes.addressof(dic)
    d.dicBufSize = out_total
    lib.LzmaDec_Init(ctypes.byref(d))
    src = ctypes.create_string_buffer(bytes(comp), len(comp))
    trace, ip = [], 0
    try:
        for k in range(max_calls):
            sl = ctypes.c_size_t(min(win, len(comp) - ip))
            st = ctypes.c_int(-1)
            pos0 = d.dicPos
            r = lib.LzmaDec_DecodeToDic(ctypes.byref(d), out_total, ctypes.addressof(src) + ip,
                                        ctypes.byref(sl), 0, ctypes.byref(st))
            trace.append((r, st.value, sl.value, d.dicPos))
            ip += sl.value
            if r != 0 or d.dicPos == out_total or (sl.value == 0 and d.dicPos == pos0):
                break
            if edit:
                edit(k, d)
    finally:
        lib.LzmaDec_FreeProbs(ctypes.byref(d), ctypes.byref(L.g_alloc))
    return trace, dic.raw[:out_total]

"""BCJ2 encoder -- TEST INFRASTRUCTURE (fixture generation only).

The reference (LZMA SDK 9.20 C) ships only the BCJ2 decoder (Bcj2.c); this is
its inverse, written from the decoder's contract so that test archives and raw
four-stream vectors can be made here.  Parity is pinned on the reference's own
Bcj2_Decode / SzFolder_Decode run over these streams (tests/golden/
make_golden_bcj2.py, make_golden_7z.py), never on this encoder.

  main  every byte except the 4 operand bytes of a converted branch
  call  big-endian absolute targets of converted E8 (CALL rel32)
  jump  big-endian absolute targets of converted E9 / 0F 8x (JMP, Jcc rel32)
  rc    one adaptive bit per branch opcode (the decoder's model: p[prevByte]
        for E8, p[256] for E9, p[257] for Jcc), LZMA-style range encoder with
        the 5-byte flush
A branch opcode is a byte b with (b & 0xFE) == 0xE8, or 0x80..0x8F after 0x0F
(IsJ, Bcj2.c:5-6), the previous byte being the last OUTPUT byte before it.
"""
import struct


class RangeEncoder:
    def __init__(self):
        self.low, self.range, self.cache, self.cache_size = 0, 0xFFFFFFFF, 0, 1
        self.out = bytearray()

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

    def bit(self, probs, i, b):
        p = probs[i]
        bound = (self.range >> 11) * p
        if b == 0:
            self.range = bound
            probs[i] = p + ((2048 - p) >> 5)
        else:
            self.low += bound
            self.range -= bound
            probs[i] = p - (p >> 5)
        while self.range < (1 << 24):
            self.range = (self.range << 8) & 0xFFFFFFFF
            self._shift_low()

    def flush(self):
        for _ in range(5):
            self._shift_low()
        return bytes(self.out)


def is_j(b0, b1):
    return (b1 & 0xFE) == 0xE8 or (b0 == 0x0F and (b1 & 0xF0) == 0x80)


def encode(data, convert=None):
    """Split x86 code into the four BCJ2 streams.  convert(pos, opcode, rel) ->
    bool decides per branch (default: the target lies inside the data, as
    7-Zip's encoder decides for file-relative calls).  Returns
    (main, call, jump, rc)."""
    n = len(data)
    if convert is None:
        def convert(pos, op, rel):
            return 0 <= (pos + 5 + rel) % (1 << 32) < n
    probs = [1024] * 258
    rc = RangeEncoder()
    main, call, jump = bytearray(), bytearray(), bytearray()
    prev, i = 0, 0
    while i < n:
        b = data[i]
        main.append(b)
        i += 1
        if not is_j(prev, b):
            prev = b
            continue
        if i == n:  # the opcode is the last output byte: no bit (Bcj2.c:70-71)
            break
        pi = prev if b == 0xE8 else (256 if b == 0xE9 else 257)
        conv = False
        if i + 4 <= n:
            rel = struct.unpack_from("<I", data, i)[0]
            rel_s = rel - (1 << 32) if rel & 0x80000000 else rel
            conv = bool(convert(i - 1, b, rel_s))
        rc.bit(probs, pi, 1 if conv else 0)
        if not conv:
            prev = b
            continue
        dest = (rel + i + 4) & 0xFFFFFFFF  # absolute: rel + position after the operand
        (call if b == 0xE8 else jump).extend(struct.pack(">I", dest))
        i += 4
        prev = data[i - 1]
    return bytes(main), bytes(call), bytes(jump), rc.flush()


def x86_like(seed, n, density=0.06):
    """Synthetic x86-flavoured bytes: text-ish filler with E8/E9 rel32 branches
    (near targets, some far), 0F 8x Jcc, and stray E8/0F bytes."""
    import random
    rng = random.Random(seed)
    out = bytearray()
    while len(out) < n:
        r = rng.random()
        if r < density:
            op = rng.choice([b"\xe8", b"\xe8", b"\xe9", b"\x0f\x84", b"\x0f\x85", b"\x0f\x8c"])
            far = rng.random() < 0.2
            rel = rng.randrange(-(1 << 31), 1 << 31) if far else rng.randrange(-4000, 4000)
            out += op + struct.pack("<i", rel)
        elif r < density * 1.3:
            out += rng.choice([b"\xe8", b"\x0f", b"\xe9\x00", b"\x0f\x0f\x80"])
        else:
            out += bytes([rng.randrange(256) if rng.random() < 0.3 else rng.randrange(0x20, 0x7F)])
    return bytes(out[:n])

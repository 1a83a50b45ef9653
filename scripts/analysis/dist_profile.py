# Analysis only (not product, not test): how far back the decoder reads its
# own output on config-2 streams (4096 x 64 KiB, lc3/lp0/pb2, 64 KiB dict) --
# the reach an LDS history window of the one-lane latency kernel needs
# (VERDICT r04 item 2).  A plain-Python LZMA decode (LzmaDec.c:131-426) of the
# bench's own streams (C generator + liblzma) records, per symbol, its kind and
# the distance of every dictionary read: the matched literal's byte at rep0
# (LzmaDec.c:176), a short rep's byte (:216) and a match copy (:388-407).
#   python scripts/analysis/dist_profile.py [streams] [n] [lc] [pb] [dict]
import lzma
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(R, "tests"))
sys.path.insert(0, os.path.join(R, "lzma-sdk-zliblike_amd"))
import native  # noqa: E402

COUNT = int(sys.argv[1]) if len(sys.argv) > 1 else 8
N = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
LC = int(sys.argv[3]) if len(sys.argv) > 3 else 3
PB = int(sys.argv[4]) if len(sys.argv) > 4 else 2
DICT = int(sys.argv[5]) if len(sys.argv) > 5 else 65536


def decode(buf, n, lc, pb):
    pos = [5]
    st = [0xFFFFFFFF, int.from_bytes(buf[1:5], "big")]
    probs = {}

    def norm():
        if st[0] < (1 << 24):
            st[0] = (st[0] << 8) & 0xFFFFFFFF
            st[1] = ((st[1] << 8) | buf[pos[0]]) & 0xFFFFFFFF
            pos[0] += 1

    def bit(key):
        p = probs.get(key, 1024)
        norm()
        b = (st[0] >> 11) * p
        if st[1] < b:
            st[0] = b
            probs[key] = p + ((2048 - p) >> 5)
            return 0
        st[0] -= b
        st[1] -= b
        probs[key] = p - (p >> 5)
        return 1

    def tree(pre, bits):
        m = 1
        for _ in range(bits):
            m = (m << 1) | bit((pre, m))
        return m - (1 << bits)

    def rtree(pre, bits):
        m, v = 1, 0
        for i in range(bits):
            b = bit((pre, m))
            m = (m << 1) | b
            v |= b << i
        return v

    def length(pre, ps):
        if not bit((pre, "c")):
            return tree((pre, "lo", ps), 3)
        if not bit((pre, "c2")):
            return 8 + tree((pre, "mid", ps), 3)
        return 16 + tree((pre, "hi"), 8)

    out = bytearray()
    state = 0
    reps = [1, 1, 1, 1]
    ev = []  # (kind, dist, nbytes)
    pbm = (1 << pb) - 1
    while len(out) < n:
        ps = len(out) & pbm
        if not bit(("M", state, ps)):
            prev = out[-1] if out else 0
            ctx = prev >> (8 - lc)
            if state < 7:
                sym = 1
                while sym < 0x100:
                    sym = (sym << 1) | bit(("L", ctx, sym))
                ev.append(("lit", 0, 1))
            else:
                mb = out[-reps[0]]
                offs, sym = 0x100, 1
                while sym < 0x100:
                    mb <<= 1
                    mbit = mb & offs
                    b = bit(("L", ctx, offs + mbit + sym))
                    sym = (sym << 1) | b
                    offs = (offs & mbit) if b else (offs & ~mbit)
                ev.append(("mlit", reps[0], 1))
            out.append(sym & 0xFF)
            state = 0 if state < 4 else (state - 3 if state < 10 else state - 6)
            continue
        if bit(("R", state)):
            if not bit(("G0", state)):
                if not bit(("R0L", state, ps)):
                    out.append(out[-reps[0]])
                    ev.append(("short", reps[0], 1))
                    state = 9 if state < 7 else 11
                    continue
            else:
                if not bit(("G1", state)):
                    d = reps[1]
                else:
                    if not bit(("G2", state)):
                        d = reps[2]
                    else:
                        d = reps[3]
                        reps[3] = reps[2]
                    reps[2] = reps[1]
                reps[1] = reps[0]
                reps[0] = d
            ln = length("RL", ps) + 2
            state = 8 if state < 7 else 11
            kind = "rep"
        else:
            ln = length("L", ps) + 2
            reps[3], reps[2], reps[1] = reps[2], reps[1], reps[0]
            slot = tree(("S", min(ln - 2, 3)), 6)
            if slot < 4:
                d = slot
            else:
                nb = (slot >> 1) - 1
                d = (2 | (slot & 1)) << nb
                if slot < 14:
                    d += rtree(("SP", d - slot), nb)
                else:
                    v = 0
                    for _ in range(nb - 4):
                        norm()
                        st[0] >>= 1
                        b = 1 if st[1] >= st[0] else 0
                        if b:
                            st[1] -= st[0]
                        v = (v << 1) | b
                    d += (v << 4) + rtree("A", 4)
            reps[0] = d + 1
            state = 7 if state < 7 else 10
            kind = "match"
        ln = min(ln, n - len(out))
        for _ in range(ln):
            out.append(out[-reps[0]])
        ev.append((kind, reps[0], ln))
    return bytes(out), ev


def main():
    plain = np.zeros(COUNT * N, dtype=np.uint8)
    native.synth().synth_batch(0, 0, plain.ctypes.data, N, COUNT, 8)
    filt = [{"id": lzma.FILTER_LZMA1, "dict_size": DICT, "lc": LC, "lp": 0, "pb": PB,
             "preset": 6}]
    evs = []
    for i in range(COUNT):
        src = plain[i * N:(i + 1) * N].tobytes()
        c = lzma.compress(src, format=lzma.FORMAT_RAW, filters=filt)
        dec, ev = decode(c, N, LC, PB)  # raw LZMA1: the rc stream starts with its 0 byte
        assert dec == src, "decode mismatch"
        evs += ev
    kinds = {}
    for k, d, nb in evs:
        a = kinds.setdefault(k, [0, 0])
        a[0] += 1
        a[1] += nb
    print(f"{COUNT} streams x {N} B, lc{LC} pb{PB} dict {DICT}")
    for k, (cnt, nb) in sorted(kinds.items()):
        print(f"  {k:6s} symbols {cnt / COUNT:9.1f}/stream  bytes {nb / COUNT:9.1f}/stream")
    reads = [(k, d, nb) for k, d, nb in evs if k != "lit"]
    for lim in (1024, 2048, 4096, 8192, 16384, 32768):
        sym_in = sum(1 for k, d, nb in reads if d <= lim) / max(1, len(reads))
        byt_in = sum(nb for k, d, nb in reads if d <= lim) / max(1, sum(nb for _, _, nb in reads))
        ml = [d for k, d, nb in reads if k == "mlit"]
        ml_in = sum(1 for d in ml if d <= lim) / max(1, len(ml))
        print(f"  reach {lim:6d}: reads {sym_in:.3f} of symbols, {byt_in:.3f} of copied bytes, "
              f"matched literals {ml_in:.3f}")


if __name__ == "__main__":
    main()

"""Golden fixture of BASELINE config 1: ONE 1 MiB
stream, lc3/lp0/pb2, 64 KiB dictionary, through the single-stream drop-in API.

Run in the build container only (needs oracle/_ref/libref_lzma.so, the
reference LzmaDec.c / LzmaEnc.c compiled in place by oracle/Makefile.ref):

    python tests/golden/make_golden_cfg1.py

enwik8 is not available offline: the plaintext is 1 MiB of the synthetic
English-like text (lzma-sdk-zliblike_amd/csrc/synth.c, seed 1), encoded by the
REFERENCE encoder (LzmaEnc.c, level 5, dict 64 KiB, lc3/lp0/pb2, no end mark --
the .lzma layout LzmaUtil writes).  Every expected value is what the reference
decoder returned for that stream, through each entry point of config 1:

  * LzmaDecode (LzmaDec.c:972-1002), FINISH_END and FINISH_ANY, exact and
    roomier capacities; LzmaUncompress (LzmaLib.c:41-46) is LzmaDecode with
    FINISH_ANY;
  * the fork's zlib-like LzmaDec_DecodeToBuf loop (7zDec.c:567-648) with its
    buffers (512 KiB in / 1 MiB out), and with 16 KiB in / 64 KiB out (many
    calls, the 64 KiB ring wrapping) -- the full per-call
    {res, status, srcLen, destLen} trace;
  * the 7zDec.c:127-171 dictionary loop: LzmaDec_DecodeToDic over a dic that is
    the whole output, input in look windows of 16 KiB (LookToRead_BUF_SIZE,
    Types.h:190) and 256 KiB (SzDecodeLzma's lookahead) -- the full per-call
    {res, status, srcLen, dicPos} trace.

Writes cfg1_blob.bin (the compressed stream) and cfg1_cases.json.
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import native  # noqa: E402

N = 1 << 20
DICT = 1 << 16
ANY, END = 0, 1


def sha(b):
    return hashlib.sha256(b).hexdigest()


def main():
    plain = native.gen("text", 1, N)
    props, comp = native.ref_encode(plain, level=5, dict_size=DICT, lc=3, lp=0, pb=2)
    assert props[0] == 0x5D, props.hex()
    ref = native.ref()
    cases = []
    for finish, cap in ((END, N), (ANY, N), (END, N + 4096), (ANY, N + 4096), (END, N - 4096)):
        res, st, dl, sl, out = native.decode(ref, "ref", comp, props, cap, finish)
        cases.append({"kind": "lzma", "dest_cap": cap, "finish": finish,
                      "expect": {"res": res, "status": st, "dest_len": dl, "src_len": sl,
                                 "sha256": sha(out)}})
    for in_chunk, out_chunk, finish in ((1 << 19, 1 << 20, ANY), (1 << 19, 1 << 20, END),
                                        (1 << 14, 1 << 16, ANY)):
        calls, trace, out, used = native.stream_decode(ref, "ref", comp, props, N, in_chunk,
                                                       out_chunk, finish)
        cases.append({"kind": "stream", "in_chunk": in_chunk, "out_chunk": out_chunk,
                      "finish": finish,
                      "expect": {"calls": calls, "trace": [list(t) for t in trace],
                                 "out_len": len(out), "in_used": used, "sha256": sha(out)}})
    for win in (1 << 14, 1 << 18):
        calls, trace, out, used, _ = native.dic_decode(ref, "ref", comp, props, N, win)
        cases.append({"kind": "dic", "win": win,
                      "expect": {"calls": calls, "trace": [list(t) for t in trace],
                                 "out_len": len(out), "in_used": used, "sha256": sha(out)}})
    with open(os.path.join(HERE, "cfg1_blob.bin"), "wb") as f:
        f.write(comp)
    doc = {"generator": "tests/golden/make_golden_cfg1.py",
           "reference": "LZMA SDK 9.20 LzmaDec.c / LzmaEnc.c (oracle/_ref/libref_lzma.so)",
           "plaintext": {"kind": "text", "seed": 1, "bytes": N, "sha256": sha(plain)},
           "props": props.hex(), "comp_len": len(comp), "comp_sha256": sha(comp),
           "cases": cases}
    with open(os.path.join(HERE, "cfg1_cases.json"), "w") as f:
        json.dump(doc, f, indent=1)
    print(f"cfg1: {len(comp)} compressed bytes, {len(cases)} cases")


if __name__ == "__main__":
    main()

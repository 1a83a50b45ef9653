"""Seed corpora for the libFuzzer targets (TEST INFRASTRUCTURE): the committed
golden fixtures, prefixed with the targets' selector bytes.

    python tests/fuzz/seeds.py OUTDIR   -> OUTDIR/containers/*, OUTDIR/lanes/*
"""
import json
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(os.path.dirname(HERE), "golden")


def _load(name, blob):
    with open(os.path.join(GOLDEN, name)) as f:
        d = json.load(f)
    with open(os.path.join(GOLDEN, blob), "rb") as f:
        d["blob"] = f.read()
    return d


def write(out):
    con, lan = os.path.join(out, "containers"), os.path.join(out, "lanes")
    os.makedirs(con, exist_ok=True)
    os.makedirs(lan, exist_ok=True)
    k = 0

    def put(dirname, data):
        nonlocal k
        with open(os.path.join(dirname, f"seed{k:05d}"), "wb") as f:
            f.write(data)
        k += 1

    sz = _load("sz_cases.json", "sz_blob.bin")
    for c in sz["cases"]:
        put(con, b"\x00" + sz["blob"][c["off"]:c["off"] + c["len"]])
    for name, blob in (("xz_cases.json", "xz_blob.bin"), ("xzf_cases.json", "xzf_blob.bin")):
        d = _load(name, blob)
        for c in d.get("xz", d.get("files", [])):
            if "off" in c and c["len"] < 400000:
                put(con, b"\x01" + d["blob"][c["off"]:c["off"] + c["len"]])
                put(con, b"\x02" + d["blob"][c["off"]:c["off"] + min(c["len"], 4096)])
    g = _load("cases.json", "blob.bin")
    for c in g["cases"][:300]:
        if c["kind"] not in ("lzma", "lzma2"):
            continue
        s = g["streams"][c["stream"]]
        src = g["blob"][s["off"]:s["off"] + min(s["len"], 20000)]
        if c["kind"] == "lzma":
            head = bytes([0]) + struct.pack("<I", c["dest_cap"]) + bytes([c["finish"]])
            put(lan, head + bytes.fromhex(c["props"]) + src)
        else:
            head = bytes([1]) + struct.pack("<I", c["dest_cap"]) + bytes([c["finish"]])
            put(lan, head + bytes([c["prop"]]) + b"\0" * 4 + src)
    b2 = _load("bcj2_cases.json", "bcj2_blob.bin")
    for c in b2["cases"][:40]:
        parts = [b2["blob"][o:o + min(n, 3000)] for o, n in c["streams"]]
        put(lan, bytes([2]) + struct.pack("<I", c["out_size"]) + b"\0" + b"".join(parts))


if __name__ == "__main__":
    write(sys.argv[1])

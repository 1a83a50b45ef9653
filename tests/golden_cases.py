"""Load the committed golden fixtures (tests/golden/cases.json + blob.bin)."""
import hashlib
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")

_cache = {}


def load():
    if "d" not in _cache:
        with open(os.path.join(GOLDEN, "cases.json")) as f:
            d = json.load(f)
        with open(os.path.join(GOLDEN, "blob.bin"), "rb") as f:
            blob = f.read()
        assert hashlib.sha256(blob).hexdigest() == d["blob_sha256"], "golden blob corrupted"
        d["blob"] = blob
        _cache["d"] = d
    return _cache["d"]


def case_input(d, c):
    """Materialize the compressed input bytes of case c (truncation + XOR flips)."""
    s = d["streams"][c["stream"]]
    b = bytearray(d["blob"][s["off"]:s["off"] + s["len"]])
    for off, mask in c["flips"]:
        b[off] ^= mask
    if c["trunc"] is not None:
        b = b[:c["trunc"]]
    return bytes(b)


def cases(kind):
    d = load()
    return [(i, c) for i, c in enumerate(d["cases"]) if c["kind"] == kind]


def sha(b):
    return hashlib.sha256(b).hexdigest()


def trace_digest(trace):
    return hashlib.sha256(";".join(",".join(str(v) for v in t) for t in trace).encode()).hexdigest()

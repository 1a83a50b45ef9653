"""Branch-converter / delta kernels on one MI355X.

    python scripts/bra_bench.py [--ranges 1024] [--size 262144] [--steps 10]

Per kind: `ranges` device ranges of `size` bytes (random bytes with each kind's
branch pattern on 40 % of the units), decoded in place by BraGpu_Batch /
DeltaGpu_Batch / BcjGpu_X86Batch, timed with HIP events on the launch stream.
Algorithmic bytes per launch = 2 x ranges x size (each byte read once and
written once).  Prints one JSON line per kind.  Each launch re-converts the
previous output (decode is not an involution, but the work per launch is the
same data-dependent scan).
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lzma-sdk-zliblike_amd"))

KINDS = {"PPC": 5, "IA64": 6, "ARM": 7, "ARMT": 8, "SPARC": 9, "x86": 4, "Delta4": 3,
         "Delta1": 3}


def stamp(kind, raw, rng):
    w = raw.reshape(-1, 4)
    pick = rng.random(len(w)) < 0.4
    if kind == "ARM":
        w[pick, 3] = 0xEB
    elif kind == "ARMT":
        w[pick, 1] = 0xF0 | (w[pick, 1] & 7)
        w[pick, 3] = 0xF8 | (w[pick, 3] & 7)
    elif kind == "PPC":
        w[pick, 0] = 0x48 | (w[pick, 0] & 3)
        w[pick, 3] = (w[pick, 3] & 0xFC) | 1
    elif kind == "SPARC":
        w[pick, 0] = 0x40
        w[pick, 1] &= 0x3F
    elif kind == "IA64":
        b = raw.reshape(-1, 16)
        b[:, 0] = (b[:, 0] & 0xE0) | 16
    elif kind == "x86":
        w[pick, 0] = 0xE8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranges", type=int, default=1024)
    ap.add_argument("--size", type=int, default=1 << 18)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    import torch
    torch.zeros(1, device="cuda")
    import lzmagpu as L
    n, size = a.ranges, a.size
    rng = np.random.default_rng(11)
    dev = torch.device("cuda")
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    for name, kid in KINDS.items():
        raw = rng.integers(0, 256, n * size, dtype=np.uint8)
        stamp(name, raw, rng)
        data = torch.from_numpy(raw).to(dev)
        off = torch.arange(n, dtype=torch.int64, device=dev) * size
        ln = torch.full((n,), size, dtype=torch.int64, device=dev)
        arg = torch.full((n,), 4 if name == "Delta4" else 1, dtype=torch.int32, device=dev)
        if kid in (5, 6, 7, 8, 9):
            arg.zero_()
        state = torch.zeros(n * 256, dtype=torch.uint8, device=dev)
        st32 = torch.zeros(n, dtype=torch.int32, device=dev)
        done = torch.zeros(n, dtype=torch.int64, device=dev)

        def launch():
            if kid == 3:
                return L.delta_batch_device(data.data_ptr(), off.data_ptr(), ln.data_ptr(),
                                            arg.data_ptr(), state.data_ptr(), n, 0, sp)
            if kid == 4:
                return L.bcj_x86_batch_device(data.data_ptr(), off.data_ptr(), ln.data_ptr(),
                                              arg.data_ptr(), st32.data_ptr(), done.data_ptr(), n,
                                              0, sp)
            return L.bra_batch_device(kid, data.data_ptr(), off.data_ptr(), ln.data_ptr(),
                                      arg.data_ptr(), done.data_ptr(), n, 0, sp)
        assert launch() == 0
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(a.steps)]
        for s, e in ev:
            s.record(stream)
            assert launch() == 0
            e.record(stream)
        torch.cuda.synchronize()
        ms = sorted(s.elapsed_time(e) for s, e in ev)
        avg = sum(ms) / len(ms)
        alg = 2 * n * size
        print(json.dumps({"kind": name, "ranges": n, "range_bytes": size, "avg_ms": round(avg, 4),
                          "min_ms": round(ms[0], 4), "GB_per_s_decoded": round(n * size / avg / 1e6, 1),
                          "roofline": {"bound": "hbm", "achieved": round(alg / avg / 1e6, 1),
                                       "peak": 8000.0, "unit": "GB/s",
                                       "frac": round(alg / avg / 1e6 / 8000.0, 4),
                                       "alg_bytes_per_launch": alg}}), flush=True)


if __name__ == "__main__":
    main()

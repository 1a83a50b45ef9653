"""Synthetic batches shaped like BASELINE.json's configs.

Shared by the full-size GPU parity tests and bench.py.  Plaintext comes from
the C generator (lib/liblzsynth.so, splitmix64 English-like text, stream i
seeded by its global index); streams are encoded with liblzma (Python stdlib
``lzma``) on a thread pool -- liblzma drops the GIL, so this needs no fork
(safe in a process that has already touched the GPU).  The encoder choice does
not affect decode parity: every decoded stream is compared with its plaintext.
"""
import lzma
import os
import random
from concurrent.futures import ThreadPoolExecutor

import numpy as np

import native

CFG5_DICTS = (4096, 16384, 65536, 262144, 1 << 20)


def workers():
    """Host threads for encoding: the process's CPU share, at most 16 (the GPU
    box gives one GPU's job a 16-CPU share whatever nproc says)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 8
    return max(1, min(16, n))


def props_bytes(lc, lp, pb, dsz):
    return bytes([(pb * 5 + lp) * 9 + lc]) + dsz.to_bytes(4, "little")


def _pool_map(fn, items, nthreads=None):
    with ThreadPoolExecutor(nthreads or workers()) as ex:
        return list(ex.map(fn, items))


def uniform_batch(count, n, lc, lp, pb, dsz, first=0, preset=6):
    """count streams of n bytes (text, seeds first..first+count-1), one props.
    Returns (plain uint8[count*n], comp uint8[], lens uint64[count], props)."""
    plain = np.zeros(count * n, dtype=np.uint8)
    native.synth().synth_batch(0, first, plain.ctypes.data, n, count, workers())
    filt = [{"id": lzma.FILTER_LZMA1, "dict_size": dsz, "lc": lc, "lp": lp, "pb": pb,
             "preset": preset}]

    def enc(i):
        return lzma.compress(plain[i * n:(i + 1) * n].tobytes(), format=lzma.FORMAT_RAW,
                             filters=filt)

    parts = _pool_map(enc, list(range(count)))
    lens = np.array([len(c) for c in parts], dtype=np.uint64)
    comp = np.frombuffer(b"".join(parts), dtype=np.uint8)
    return plain, comp, lens, props_bytes(lc, lp, pb, dsz)


def cfg5_params(i, max_log2=8):
    """Props, dict, length and finish mode of config-5 stream i (SURVEY 8(d):
    lc 0-4, lp 0-2 with lc+lp <= 4, pb 0-4, dict in {4K..1M}, length
    log-uniform 1 KiB .. 2^max_log2 KiB, end marker on half), seeded by (5, i)."""
    rng = random.Random(5 * 1000003 + i)
    while True:
        lc, lp = rng.randrange(5), rng.randrange(3)
        if lc + lp <= 4:
            break
    pb = rng.randrange(5)
    dsz = rng.choice(CFG5_DICTS)
    n = int(round(1024 * 2 ** (rng.uniform(0, 8) * max_log2 / 8)))
    fin = rng.randrange(2)
    return lc, lp, pb, dsz, n, fin


def cfg5_stream(i, max_log2=8, preset=6):
    lc, lp, pb, dsz, n, fin = cfg5_params(i, max_log2)
    data = native.gen("text", 70000 + i, n)
    f = [{"id": lzma.FILTER_LZMA1, "dict_size": dsz, "lc": lc, "lp": lp, "pb": pb,
          "preset": preset}]
    c = lzma.compress(data, format=lzma.FORMAT_RAW, filters=f)
    return data, c, props_bytes(lc, lp, pb, dsz), fin


def lzma2_block(seed, n, dsz=1 << 20, preset=6):
    """One LZMA2 dict-reset block of n text bytes (lc3/lp0/pb2) without the EOS byte."""
    data = native.gen("text", seed, n)
    f = [{"id": lzma.FILTER_LZMA2, "dict_size": dsz, "lc": 3, "lp": 0, "pb": 2,
          "preset": preset}]
    c = lzma.compress(data, format=lzma.FORMAT_RAW, filters=f)
    assert c[-1] == 0
    return data, c[:-1]

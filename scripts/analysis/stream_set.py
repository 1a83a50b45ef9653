"""Write N config-3 streams (bench.py's workload) as the stream-set files of
tests/c_host/lzma_c_threads.c into DIR (for profiling the drop-in callers).
  python scripts/analysis/stream_set.py DIR [N]"""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "tests"))
sys.path.insert(0, os.path.join(R, "lzma-sdk-zliblike_amd"))
import numpy as np  # noqa: E402

import bench  # noqa: E402
import test_c_host as TC  # noqa: E402

d = sys.argv[1]
count = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
os.makedirs(d, exist_ok=True)
plain, comp, lens, props = bench.build_workload("cfg3", 0, count, 8)
offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
comps = [comp[offs[i]:offs[i + 1]].tobytes() for i in range(count)]
f = TC.write_stream_set(d, comps, [props] * count, [4096] * count)
print(" ".join(os.path.abspath(f[k]) for k in ("src", "lens", "props", "outs")))

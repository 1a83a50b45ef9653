"""Timeline of the pipelined end-to-end path (investigation, run via gpurun):
per batch, when its H2D, decode and D2H start and end (HIP events, ms from
the first event), to see which stages overlap."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "lzma-sdk-zliblike_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "three"
    plain, comp, lens, props = bench.build_workload("cfg3", 0, 65536, 16)
    import torch
    import lzmagpu as L
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    n = 4096
    count = 65536
    descs, order, plan, offs = bench.make_descs(lens, n, props)
    d_ws = torch.empty(int(plan.workspace_bytes), dtype=torch.uint8, device=dev)
    d_desc = torch.frombuffer(bytearray(descs), dtype=torch.uint8).to(dev)
    d_order = torch.frombuffer(bytearray(order), dtype=torch.uint8).to(dev)
    d_res = torch.empty(count * 24, dtype=torch.uint8, device=dev)
    nb = int(comp.size)
    h_src = torch.from_numpy(np.array(comp)).pin_memory()
    h_dst = [torch.empty(count * n, dtype=torch.uint8).pin_memory() for _ in range(2)]
    d_src = [torch.empty(nb + 64, dtype=torch.uint8, device=dev) for _ in range(2)]
    d_dst = [torch.empty(count * n + 64, dtype=torch.uint8, device=dev) for _ in range(2)]
    if mode in ("three", "ahead"):
        s_h2d, s_dec, s_d2h = (torch.cuda.Stream(dev) for _ in range(3))
    else:  # one copy stream for both directions
        s_dec = torch.cuda.Stream(dev)
        s_h2d = s_d2h = torch.cuda.Stream(dev)
    E = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    t0e = E()
    t0e.record(torch.cuda.current_stream(dev))
    marks = []
    dec_done = [E(), E()]
    d2h_done = [E(), E()]
    for e in dec_done + d2h_done:
        e.record(torch.cuda.current_stream(dev))
    torch.cuda.synchronize()
    w0 = time.perf_counter()
    B = 6
    if mode.startswith("ahead"):
        return ahead(mode, L, torch, plan, d_desc, d_order, d_ws, d_res, d_src, d_dst, h_src, h_dst,
                     s_h2d, s_dec, s_d2h, E, t0e, dec_done, d2h_done, nb, count, n, plain, B, w0)
    for b in range(B):
        k = b % 2
        m = [E() for _ in range(6)]
        s_h2d.wait_event(dec_done[k])
        m[0].record(s_h2d)
        with torch.cuda.stream(s_h2d):
            d_src[k][:nb].copy_(h_src, non_blocking=True)
        m[1].record(s_h2d)
        s_dec.wait_event(m[1])
        s_dec.wait_event(d2h_done[k])
        m[2].record(s_dec)
        assert L.decode_batch_device_ex(plan, d_desc.data_ptr(), d_order.data_ptr(),
                                        d_src[k].data_ptr(), d_dst[k].data_ptr(),
                                        d_ws.data_ptr(), d_res.data_ptr(), s_dec.cuda_stream) == 0
        m[3].record(s_dec)
        dec_done[k] = m[3]
        s_d2h.wait_event(m[3])
        m[4].record(s_d2h)
        with torch.cuda.stream(s_d2h):
            h_dst[k].copy_(d_dst[k][:count * n], non_blocking=True)
        m[5].record(s_d2h)
        d2h_done[k] = m[5]
        marks.append(m)
        print(f"enqueued batch {b} at host {1e3 * (time.perf_counter() - w0):.2f} ms", flush=True)
    torch.cuda.synchronize()
    wall = time.perf_counter() - w0
    for b, m in enumerate(marks):
        t = [t0e.elapsed_time(x) for x in m]
        print(f"batch {b}: h2d {t[0]:8.2f}-{t[1]:8.2f}  dec {t[2]:8.2f}-{t[3]:8.2f}  "
              f"d2h {t[4]:8.2f}-{t[5]:8.2f}")
    print(f"mode {mode}: {B} batches in {wall * 1e3:.1f} ms = {wall / B * 1e3:.2f} ms/batch; "
          f"last ok {np.array_equal(h_dst[(B - 1) % 2].numpy(), plain)}")


def ahead(mode, L, torch, plan, d_desc, d_order, d_ws, d_res, d_src, d_dst, h_src, h_dst,
          s_h2d, s_dec, s_d2h, E, t0e, dec_done, d2h_done, nb, count, n, plain, B, w0):
    """Enqueue order H2D(b+1), decode(b), D2H(b): the next batch's upload is
    queued before this batch's download, so a copy queue shared by both
    directions never holds the upload behind a download that waits for a decode."""
    marks = [[E() for _ in range(6)] for _ in range(B)]
    h2d_done = [None, None]

    def h2d(b):
        k = b % 2
        m = marks[b]
        s_h2d.wait_event(dec_done[k])
        m[0].record(s_h2d)
        with torch.cuda.stream(s_h2d):
            d_src[k][:nb].copy_(h_src, non_blocking=True)
        m[1].record(s_h2d)
        h2d_done[k] = m[1]

    h2d(0)
    for b in range(B):
        k = b % 2
        m = marks[b]
        if b + 1 < B:
            h2d(b + 1)
        s_dec.wait_event(h2d_done[k])
        s_dec.wait_event(d2h_done[k])
        m[2].record(s_dec)
        assert L.decode_batch_device_ex(plan, d_desc.data_ptr(), d_order.data_ptr(),
                                        d_src[k].data_ptr(), d_dst[k].data_ptr(),
                                        d_ws.data_ptr(), d_res.data_ptr(), s_dec.cuda_stream) == 0
        m[3].record(s_dec)
        dec_done[k] = m[3]
        s_d2h.wait_event(m[3])
        m[4].record(s_d2h)
        with torch.cuda.stream(s_d2h):
            h_dst[k].copy_(d_dst[k][:count * n], non_blocking=True)
        m[5].record(s_d2h)
        d2h_done[k] = m[5]
    torch.cuda.synchronize()
    wall = time.perf_counter() - w0
    for b, m in enumerate(marks):
        t = [t0e.elapsed_time(x) for x in m]
        print(f"batch {b}: h2d {t[0]:8.2f}-{t[1]:8.2f}  dec {t[2]:8.2f}-{t[3]:8.2f}  "
              f"d2h {t[4]:8.2f}-{t[5]:8.2f}")
    print(f"mode {mode}: {B} batches in {wall * 1e3:.1f} ms = {wall / B * 1e3:.2f} ms/batch; "
          f"last ok {np.array_equal(h_dst[(B - 1) % 2].numpy(), plain)}")


if __name__ == "__main__":
    main()

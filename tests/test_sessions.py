"""Device-resident streaming sessions: many concurrent
zlib-like LzmaDec_DecodeToBuf streams, one batched launch per round of calls
(LzmaGpu_SessionDecodeBatch, mode 1), decoder state kept in device memory.

CPU: the session struct layout and LzmaGpu_SessionInit (host logic).  The
kernel body's DecodeToBuf ring loop is checked on the host by
tests/test_emu.py::test_emu_golden_streaming[device_ring].
GPU: all golden streaming cases as concurrent sessions in lockstep rounds;
each session's full per-call {res, status, srcLen, destLen} trace and output
must equal what the reference's LzmaDec_DecodeToBuf loop produced."""
import ctypes

import pytest

import golden_cases as G


def test_session_layout_and_init():
    import lzmagpu as L
    assert ctypes.sizeof(L.Session) == 192
    assert L.Session.out.offset == 176 and L.Session.temp_buf.offset == 148
    assert ctypes.sizeof(L.Plan) == 248
    assert L.session_probs_bytes(b"\x5d\x00\x00\x01\x00") == 2 * (56 * 4 + 950 + (768 << 3))
    assert L.session_probs_bytes(b"\xe1\x00\x00\x01\x00") == 0  # props byte 225
    r, s = L.session_init(b"\x5d\x00\x00\x01\x00", 0x1000, 0x2000, 65536)
    assert r == 0
    assert (s.lc, s.lp, s.pb, s.dict_size) == (3, 0, 2, 65536)
    assert (s.dic_pos, s.need_flush, s.need_init_state, s.remain_len, s.temp_buf_size) == \
        (0, 1, 1, 0, 0)
    assert (s.processed_pos, s.check_dic_size, s.dic_buf_size) == (0, 0, 65536)
    r, _ = L.session_init(b"\xe1\x00\x00\x01\x00", 0x1000, 0x2000, 65536)
    assert r == L.SZ_ERROR_UNSUPPORTED
    r, _ = L.session_init(b"\x5d\x00\x00\x01\x00", 0, 0x2000, 65536)
    assert r == L.SZ_ERROR_PARAM


@pytest.mark.gpu
def test_gpu_sessions_golden_streams_lockstep():
    import torch
    import lzmagpu as L
    d = G.load()
    dev = torch.device("cuda")
    cases = G.cases("stream")
    keep, sess, st = [], [], []
    for i, c in cases:
        props = bytes.fromhex(c["props"])
        src = G.case_input(d, c)
        dict_size = int.from_bytes(props[1:5], "little")
        dict_size = max(dict_size, 4096)
        t_probs = torch.zeros(max(L.session_probs_bytes(props), 2), dtype=torch.uint8, device=dev)
        t_dic = torch.zeros(dict_size, dtype=torch.uint8, device=dev)
        t_src = torch.frombuffer(bytearray(src) + b"\0" * 16, dtype=torch.uint8).to(dev)
        t_out = torch.zeros(max(c["out_total"], 1), dtype=torch.uint8, device=dev)
        keep += [t_probs, t_dic, t_src, t_out]
        r, s = L.session_init(props, t_probs.data_ptr(), t_dic.data_ptr(), dict_size)
        assert r == 0
        sess.append(s)
        st.append(dict(c=c, src=t_src, out=t_out, n_src=len(src), in_pos=0, out_pos=0,
                       trace=[], done=False))
    n = len(sess)
    arr = (L.Session * n)(*sess)
    d_arr = torch.empty(ctypes.sizeof(arr), dtype=torch.uint8, device=dev)
    rounds = 0
    while not all(x["done"] for x in st):
        for k, x in enumerate(st):
            c = x["c"]
            s = arr[k]
            if x["done"]:
                s.in_len = 0
                s.out_len = 0
                s.mode = 1
                continue
            sl = min(x["n_src"] - x["in_pos"], c["in_chunk"])
            dl = min(c["out_total"] - x["out_pos"], c["out_chunk"])
            s.mode = 1
            s.in_ = x["src"].data_ptr() + x["in_pos"]
            s.in_len = sl
            s.out = x["out"].data_ptr() + x["out_pos"]
            s.out_len = dl
            s.finish_mode = c["finish"]
        d_arr.copy_(torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8))
        assert L.session_decode_batch(d_arr.data_ptr(), n) == 0, L.last_error()
        torch.cuda.synchronize()
        ctypes.memmove(arr, bytes(d_arr.cpu().numpy()), ctypes.sizeof(arr))
        rounds += 1
        for k, x in enumerate(st):
            if x["done"]:
                continue
            s = arr[k]
            res, status, got_in, got_out = s.res, s.status, s.in_used, s.out_len
            x["trace"].append((res, status, got_in, got_out))
            x["in_pos"] += got_in
            x["out_pos"] += got_out
            if (res != 0 or status == 1 or x["out_pos"] == x["c"]["out_total"] or
                    (got_in == 0 and got_out == 0)):
                x["done"] = True
    assert rounds == max(c["expect"]["calls"] for _, c in cases)
    for x in st:
        e = x["c"]["expect"]
        assert len(x["trace"]) == e["calls"]
        assert G.trace_digest(x["trace"]) == e["trace_sha256"], (x["c"]["note"], x["trace"][:3])
        assert (x["out_pos"], x["in_pos"]) == (e["out_len"], e["in_used"])
        out = bytes(x["out"].cpu().numpy()[:x["out_pos"]])
        assert G.sha(out) == e["sha256"]


def _fuzz_sessions(count, seed):
    """Seeded zlib-like streams: presets, dictionaries, text / random / runs,
    corruption, truncation, output totals, finish modes and chunk sizes (in
    and out, 1 byte up), with the oracle's DecodeToBuf loop trace as the
    expectation (the restatement pinned to the reference's streaming traces)."""
    import lzma
    import random
    import native
    import workloads as W
    rng = random.Random(seed)
    orc = native.oracle()
    out = []
    while len(out) < count:
        it = len(out)
        lc = rng.randrange(5)
        lp = rng.randrange(5 - lc)
        pb = rng.randrange(5)
        dsz = rng.choice([4096, 1 << 14, 1 << 16])
        n = rng.choice([0, 100, 3000, 20000, 100000])
        in_chunk = rng.choice([1, 7, 333, 4096, 1 << 20])
        out_chunk = rng.choice([1, 17, 1000, 65536, 1 << 22])
        data = native.gen(rng.choice(["text", "text", "random", "runs"]), 123_000 + it, n)
        comp = bytearray(lzma.compress(data, format=lzma.FORMAT_RAW, filters=[
            {"id": lzma.FILTER_LZMA1, "dict_size": dsz, "lc": lc, "lp": lp, "pb": pb,
             "preset": rng.choice([0, 6])}]))
        mode = rng.randrange(5)
        if mode == 1 and len(comp) > 6:
            comp[rng.randrange(5, len(comp))] ^= 1 << rng.randrange(8)
        elif mode == 2:
            comp = comp[:rng.randrange(len(comp) + 1)]
        total = max(0, n + rng.choice([0, 0, 1, -1, 500, -500]))
        if max(len(comp) / in_chunk, total / out_chunk) > 1500:
            continue  # keep the lockstep rounds bounded
        props = W.props_bytes(lc, lp, pb, dsz)
        fin = rng.randrange(2)
        calls, trace, dec, used = native.stream_decode(orc, "orc", bytes(comp), props, total,
                                                       in_chunk, out_chunk, fin)
        out.append(dict(props=props, src=bytes(comp), out_total=total, in_chunk=in_chunk,
                        out_chunk=out_chunk, finish=fin, trace=trace, out=dec, used=used))
    return out


@pytest.mark.gpu
def test_gpu_sessions_fuzz_lockstep():
    """400 seeded streams (LZGPU_SESSION_FUZZ / LZGPU_SESSION_SEED) as concurrent
    device sessions: every call's {res, status, srcLen, destLen} and the output
    equal the oracle's DecodeToBuf loop."""
    import os
    import torch
    import lzmagpu as L
    cases = _fuzz_sessions(int(os.environ.get("LZGPU_SESSION_FUZZ", "400")),
                           int(os.environ.get("LZGPU_SESSION_SEED", "4242")))
    dev = torch.device("cuda")
    keep, sess, st = [], [], []
    for c in cases:
        props = c["props"]
        dict_size = max(int.from_bytes(props[1:5], "little"), 4096)
        t_probs = torch.zeros(max(L.session_probs_bytes(props), 2), dtype=torch.uint8, device=dev)
        t_dic = torch.zeros(dict_size, dtype=torch.uint8, device=dev)
        t_src = torch.frombuffer(bytearray(c["src"]) + b"\0" * 16, dtype=torch.uint8).to(dev)
        t_out = torch.zeros(max(c["out_total"], 1), dtype=torch.uint8, device=dev)
        keep += [t_probs, t_dic, t_src, t_out]
        r, s = L.session_init(props, t_probs.data_ptr(), t_dic.data_ptr(), dict_size)
        assert r == 0
        sess.append(s)
        st.append(dict(c=c, src=t_src, out=t_out, in_pos=0, out_pos=0, trace=[], done=False))
    n = len(sess)
    arr = (L.Session * n)(*sess)
    d_arr = torch.empty(ctypes.sizeof(arr), dtype=torch.uint8, device=dev)
    while not all(x["done"] for x in st):
        for k, x in enumerate(st):
            c, s = x["c"], arr[k]
            s.mode = 1
            if x["done"]:
                s.in_len = s.out_len = 0
                continue
            s.in_ = x["src"].data_ptr() + x["in_pos"]
            s.in_len = min(len(c["src"]) - x["in_pos"], c["in_chunk"])
            s.out = x["out"].data_ptr() + x["out_pos"]
            s.out_len = min(c["out_total"] - x["out_pos"], c["out_chunk"])
            s.finish_mode = c["finish"]
        d_arr.copy_(torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8))
        assert L.session_decode_batch(d_arr.data_ptr(), n) == 0, L.last_error()
        torch.cuda.synchronize()
        ctypes.memmove(arr, bytes(d_arr.cpu().numpy()), ctypes.sizeof(arr))
        for k, x in enumerate(st):
            if x["done"]:
                continue
            s = arr[k]
            x["trace"].append((s.res, s.status, s.in_used, s.out_len))
            x["in_pos"] += s.in_used
            x["out_pos"] += s.out_len
            if (s.res != 0 or s.status == 1 or x["out_pos"] == x["c"]["out_total"] or
                    (s.in_used == 0 and s.out_len == 0)):
                x["done"] = True
    bad = []
    for k, x in enumerate(st):
        c = x["c"]
        out = bytes(x["out"].cpu().numpy()[:x["out_pos"]])
        if (x["trace"] != [tuple(t) for t in c["trace"]] or out != c["out"] or
                x["in_pos"] != c["used"]):
            bad.append((k, x["trace"][:3], c["trace"][:3]))
    assert not bad, (len(bad), bad[:4])

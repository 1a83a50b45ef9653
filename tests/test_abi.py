"""CPU-side checks of the C-ABI library (no GPU needed).

- liblzmagpu.so loads and exports every function include/lzma_gpu.h declares;
- struct sizes match the reference layouts (CLzmaDec is public ABI);
- without a device, decode entry points fail loudly (SZ_ERROR_FAIL), never
  silently fall back to a CPU path;
- the host-side LZMA2 block splitter and batch planner (pure host logic).
"""
import ctypes
import os
import re
import subprocess

import pytest

import native

ILV = 0x40000000  # placement bit: lane-interleaved global sections (throughput kernel)

ROOT = native.ROOT
HEADER = os.path.join(ROOT, "include", "lzma_gpu.h")
LIB = os.path.join(ROOT, "lzma-sdk-zliblike_amd", "lib", "liblzmagpu.so")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = re.findall(r"^\s*(?:SRes|void|int|size_t|UInt32|const char \*)\s*\*?\s*(\w+)\s*\(", txt,
                       flags=re.M)
    return sorted(set(names))


def test_header_declares_reference_surface():
    names = header_functions()
    for ref_name in ("LzmaProps_Decode", "LzmaDec_AllocateProbs", "LzmaDec_FreeProbs",
                     "LzmaDec_Allocate", "LzmaDec_Free", "LzmaDec_Init", "LzmaDec_DecodeToDic",
                     "LzmaDec_DecodeToBuf", "LzmaDecode", "LzmaUncompress",
                     "Lzma2Dec_AllocateProbs", "Lzma2Dec_Allocate", "Lzma2Dec_Init",
                     "Lzma2Dec_DecodeToDic", "Lzma2Dec_DecodeToBuf", "Lzma2Decode",
                     "CrcGenerateTable", "CrcUpdate", "CrcCalc"):
        assert ref_name in names


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [n for n in header_functions() if n not in exported]
    assert not missing, missing
    lib = ctypes.CDLL(LIB)
    for n in header_functions():
        assert hasattr(lib, n)


def test_struct_layouts():
    import lzmagpu as L
    assert ctypes.sizeof(L.CLzmaDec) == 136
    assert L.CLzmaDec.dicPos.offset == 48 and L.CLzmaDec.tempBuf.offset == 112
    assert ctypes.sizeof(L.StreamDesc) == 48
    assert ctypes.sizeof(L.Result) == 24


def test_props_decode_host():
    import lzmagpu as L
    p = L.CLzmaProps()
    assert L.lib.LzmaProps_Decode(ctypes.byref(p), b"\x5d\x00\x00\x01\x00", 5) == 0
    assert (p.lc, p.lp, p.pb, p.dicSize) == (3, 0, 2, 65536)
    assert L.lib.LzmaProps_Decode(ctypes.byref(p), b"\x00\x00\x01\x00\x00", 5) == 0
    assert (p.lc, p.lp, p.pb, p.dicSize) == (0, 0, 0, 4096)
    assert L.lib.LzmaProps_Decode(ctypes.byref(p), b"\xe1\x00\x00\x01\x00", 5) == 4
    assert L.lib.LzmaProps_Decode(ctypes.byref(p), b"\x5d\x00\x00\x01", 4) == 4


def test_no_device_fails_loudly():
    import lzmagpu as L
    if L.device_count() > 0:
        pytest.skip("a HIP device is present")
    res, st, dl, sl, out = L.LzmaDecode(b"\x00" * 32, b"\x5d\x00\x00\x01\x00", 100)
    assert res == L.SZ_ERROR_FAIL and dl == 0
    assert "no HIP device" in L.last_error()
    # CRC drop-ins have no error channel: 0 (never a silently CPU-computed value)
    assert L.CrcCalc(b"123456789") == 0


def test_lzma2_split_blocks_matches_reference_layout():
    import lzmagpu as L
    if not os.path.exists(native.REF_SO):
        pytest.skip("reference build absent (fixture generation only)")
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "mg", os.path.join(ROOT, "tests", "golden", "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    data = native.gen("text", 5, 300000) + native.gen("random", 6, 70000)
    prop, comp = mg.lzma2_multiblock(data, 100000, 1 << 16)
    blocks = L.split_lzma2_blocks(comp)
    assert len(blocks) == 4
    assert [b[2] for b in blocks] == [100000, 100000, 100000, 70000]
    assert blocks[0][0] == 0
    for a, b in zip(blocks, blocks[1:]):
        assert a[0] + a[1] == b[0]
    assert blocks[-1][0] + blocks[-1][1] == len(comp) - 1  # trailing EOS byte
    # each block decodes standalone with the reference to its slice
    off = 0
    for so, sl, u in blocks:
        r = native.lzma2_decode(native.ref(), "ref", comp[so:so + sl], prop, u, 0)
        assert r[0] == 0 and r[2] == u and r[3] == sl
        assert r[4] == data[off:off + u]
        off += u


def test_plan_batch_workspace_and_order():
    import lzmagpu as L
    items = [dict(src_off=0, src_len=10, dst_off=0, dst_cap=c, props=p)
             for c, p in ((100, b"\x5d\x00\x00\x01\x00"), (5000, b"\x00\x00\x10\x00\x00"),
                          (300, b"\xe1\x00\x00\x01\x00"))]
    descs = L.make_descs(items)
    order = (ctypes.c_uint32 * 3)()
    ws = L.plan(descs, order)
    # compact device layout: lo = 56 * 2^pb + 438 + 0x300 << (lc+lp), hi = 512 cells
    def cells(lc, lp, pb):
        return 56 * (1 << pb) + 438 + (768 << (lc + lp)) + 512
    assert descs[0].probs_off == 0
    assert descs[1].probs_off == (cells(3, 0, 2) + 7) // 8 * 8
    assert ws == 2 * (descs[1].probs_off + (cells(0, 0, 0) + 7) // 8 * 8)
    assert list(order) == [1, 2, 0]
    # compact table never exceeds what LzmaDec_AllocateProbs allocates (numProbs)
    for lc in range(9):
        for lp in range(5):
            for pb in range(5):
                assert cells(lc, lp, pb) <= 1846 + (768 << (lc + lp))
    plan, order2 = L.plan_ex(descs)
    assert plan.n == 3 and plan.n_lds == 2 and list(order2) == [1, 0, 2]
    # one LDS launch per table-width class, in the lane order.  A one-stream class
    # is in the latency regime on the cooperative kernel with the whole table in
    # LDS (placement 0x7FF: 56 * 2^pb + 950 + 0x300 << (lc+lp) cells); with
    # LZMA_GPU_PLAN_COOP_LAT the latency placement 0x1BF (all but SpecPos,
    # matched-literal and LenHigh trees) = 56 * 2^pb + 324 + 0x100 << (lc+lp)
    assert plan.n_classes == 2
    c0, c1 = plan.classes[0], plan.classes[1]
    COOP = 0x80000000  # one stream per workgroup: the wave-cooperative kernel

    def odd_dwords(cells):  # per-lane slices: an odd number of dwords (LDS banks)
        return ((cells + 1) & ~1) | 2

    assert (c0.n, c0.lds_cells_per_lane, c0.lds_mask) == (1, odd_dwords(56 + 950 + 768), 0x7FF | COOP)
    assert (c1.n, c1.lds_cells_per_lane, c1.lds_mask) == (1, odd_dwords(56 * 4 + 950 + (768 << 3)),
                                                          0x7FF | COOP)
    assert (c0.lanes_per_group, c0.groups_per_cu) == (1, 16)
    pl, _ = L.plan_ex(descs, L.plan_options("auto", flags=4))
    assert (pl.classes[0].lds_cells_per_lane, pl.classes[0].lds_mask) == \
        (odd_dwords(56 + 324 + 256), 0x1BF | COOP)
    assert (pl.classes[1].lds_cells_per_lane, pl.classes[1].lds_mask) == \
        (odd_dwords(56 * 4 + 324 + (256 << 3)), 0x1BF | COOP)
    # a full-size batch is in the throughput regime: placement 0x105 (IsMatch,
    # IsRep/G0/G1/G2, plain literal tree) = 12 * 2^pb + 48 + 0x100 << (lc+lp) cells
    big = L.make_descs([dict(src_off=0, src_len=1000, dst_off=4096 * i, dst_cap=4096,
                             props=b"\x00\x00\x10\x00\x00") for i in range(65536)])
    pb_, _ = L.plan_ex(big)
    cb = pb_.classes[0]
    assert (pb_.n_classes, cb.n, cb.lds_cells_per_lane, cb.lds_mask) == \
        (1, 65536, 318, 0x105 | ILV)
    # global sections lane-interleaved in the class's slot area: 8 groups x 256
    # CUs of 32 lanes, one column each of the lc0/pb0 global rows (LitM 0x200,
    # Len + RepLen 2 x 18, PosSlot 256, SpecPos 114, Align 16, LenHigh 512, IsRep0Long 12)
    assert (cb.slot_groups, cb.slot_cells) == (2048, 512 + 36 + 256 + 114 + 16 + 512 + 12)
    assert cb.slot_off % 64 == 0
    assert pb_.workspace_bytes >= 2 * (cb.slot_off + 2048 * 32 * cb.slot_cells)
    # every stream of the class draws on the slot area: no per-stream slices
    assert cb.slot_off == 0
    ps, _ = L.plan_ex(big, L.plan_options("auto", flags=16))  # LZMA_GPU_PLAN_NO_ILV
    assert ps.classes[0].lds_mask == 0x105 and ps.classes[0].slot_cells == 0
    assert (cb.lanes_per_group, cb.groups_per_cu, cb.waves_per_simd) == (32, 8, 2)
    assert (cb.lds_cells_per_lane // 2) % 2 == 1  # 159 dwords: 32 lanes, 32 banks
    # LZMA_GPU_PLAN_SLICE_ALIGN8: the round-1 8-byte aligned slices (158 dwords)
    pa, _ = L.plan_ex(big, L.plan_options("auto", flags=1))
    assert pa.classes[0].lds_cells_per_lane == 316
    # 0x80 was LZMA_GPU_PLAN_STEP (removed); a caller still setting
    # it is refused, not silently given LZMA_GPU_PLAN_NO_SLOTG (now 0x100)
    order = (ctypes.c_uint32 * len(big))()
    for bad in (0x80, 0x200, 0x80000000):
        assert L.lib.LzmaGpu_PlanBatchOpt(big, len(big), order, ctypes.byref(L.Plan()),
                                          ctypes.byref(L.plan_options("auto", flags=bad))) == 5
    pn, _ = L.plan_ex(big, L.plan_options("auto", flags=0x100))  # NO_SLOTG: accepted
    assert pn.n_classes == 1
    assert plan.queue_offset % 64 == 0 and plan.workspace_bytes >= plan.queue_offset + 256


def test_plan_options_force_each_instantiation():
    """LzmaGpu_PlanBatchOpt forces the kernel per call (no process environment):
    the tests use it to run the goldens through every instantiation."""
    import lzmagpu as L
    items = [dict(src_off=0, src_len=100, dst_off=4096 * i, dst_cap=4096,
                  props=b"\x00\x00\x10\x00\x00" if i % 3 else b"\x5d\x00\x00\x01\x00")
             for i in range(300)]
    items.append(dict(src_off=0, src_len=100, dst_off=0, dst_cap=100, props=bytes([16]), kind=1))
    descs = L.make_descs(items)
    COOP = 0x80000000
    masks = {}
    for k in ("auto", "throughput", "latency", "coop", "global"):
        p, order = L.plan_ex(descs, L.plan_options(k, cus=4))
        assert sorted(order[i] for i in range(len(items))) == list(range(len(items)))
        masks[k] = [p.classes[c].lds_mask for c in range(p.n_classes)]
        lanes = [p.classes[c].lanes_per_group for c in range(p.n_classes)]
        if k == "throughput":
            # interleaved global rows for the 32-lane classes, slices for narrower ones
            assert all(m == (0x105 | ILV if ln in (32, 64) else 0x105)
                       for m, ln in zip(masks[k], lanes)) and max(lanes) == 32
        elif k == "latency":
            # 0x19F: the slot trees global where the widest slice (here the
            # LZMA2 item's lc + lp <= 4 reservation) would cost workgroups per CU
            assert set(masks[k]) <= {0x1BF, 0x19F} and set(lanes) == {1}
        elif k == "coop":
            assert set(masks[k]) <= {0x1BF | COOP, 0x7FF | COOP} and 0x7FF | COOP in masks[k]
        elif k == "global":
            assert p.n_lds == 0 and p.n_classes == 0
    # 200 narrow streams over 4 CUs = 50 per CU: latency regime by the planner
    assert masks["auto"] and 0x105 not in masks["auto"] and 0x105 | ILV not in masks["auto"]
    # more CUs: <= 8 streams per CU, the cooperative kernel
    p, _ = L.plan_ex(descs, L.plan_options("auto", cus=256))
    assert all(p.classes[c].lds_mask & COOP for c in range(p.n_classes))
    p, _ = L.plan_ex(descs, L.plan_options("auto", cus=256, coop=2))
    assert not any(p.classes[c].lds_mask & COOP for c in range(p.n_classes))
    # round 6: the cooperative gate counts the whole batch per CU, not one
    # width bucket -- four widths x 1,024 streams on 256 CUs (16 per CU in all,
    # ~4 per bucket) run as one merged one-stream class, not four cooperative
    # classes that would share the CUs' LDS
    props4 = [b"\x00\x00\x00\x01\x00", b"\x5d\x00\x00\x01\x00", b"\x02\x00\x00\x01\x00",
              b"\xb8\x00\x00\x01\x00"]  # lc0, lc3 pb2, lc2, lc4 pb4
    mix = L.make_descs([dict(src_off=0, src_len=3000, dst_off=65536 * i, dst_cap=65536,
                             props=props4[i % 4]) for i in range(4096)])
    pm, _ = L.plan_ex(mix, L.plan_options("auto", cus=256))
    assert pm.n_classes == 1 and not pm.classes[0].lds_mask & COOP and pm.classes[0].lanes_per_group == 1
    # ... while few streams per CU in all still go cooperative
    pf, _ = L.plan_ex(L.make_descs([dict(src_off=0, src_len=3000, dst_off=65536 * i, dst_cap=65536,
                                         props=props4[i % 4]) for i in range(1024)]),
                      L.plan_options("auto", cus=256))
    assert all(pf.classes[c].lds_mask & COOP for c in range(pf.n_classes))
    bad = L.plan_options("auto")
    bad.kernel = 9
    order = (ctypes.c_uint32 * len(items))()
    assert L.lib.LzmaGpu_PlanBatchOpt(descs, len(items), order, ctypes.byref(L.Plan()),
                                      ctypes.byref(bad)) == L.SZ_ERROR_PARAM

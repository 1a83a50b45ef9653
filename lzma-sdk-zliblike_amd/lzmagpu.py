"""lzmagpu -- Python mirror of liblzmagpu.so (include/lzma_gpu.h) over ctypes.

The product is the C ABI; this module only binds it for the test-suite and
bench.py.  Function names and argument meaning follow the reference C API
(LzmaDec.h / LzmaLib.h / Lzma2Dec.h): ``LzmaDecode`` returns the same
``(res, status, destLen, srcLen)`` the reference returns through its
out-parameters, plus the output bytes.

There is no fallback: if lib/liblzmagpu.so is missing this module raises at
import time, and on a machine without a HIP device every decode returns
SZ_ERROR_FAIL (``LzmaGpu_LastError`` says why).
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# LZGPU_LIB may name a code-shape variant build (lib/variants/, A/B runs only)
LIB_PATH = os.environ.get("LZGPU_LIB") or os.path.join(HERE, "lib", "liblzmagpu.so")

if not os.path.exists(LIB_PATH):
    raise ImportError(f"liblzmagpu.so not built ({LIB_PATH}); run __graft_entry__.build()")

SZ_OK, SZ_ERROR_DATA, SZ_ERROR_MEM, SZ_ERROR_UNSUPPORTED = 0, 1, 2, 4
SZ_ERROR_PARAM, SZ_ERROR_INPUT_EOF, SZ_ERROR_FAIL = 5, 6, 11
LZMA_FINISH_ANY, LZMA_FINISH_END = 0, 1
KIND_LZMA, KIND_LZMA2 = 0, 1

_lib = ctypes.CDLL(LIB_PATH)
_sp = ctypes.POINTER(ctypes.c_size_t)
_ip = ctypes.POINTER(ctypes.c_int)


class ISzAlloc(ctypes.Structure):
    _fields_ = [("Alloc", ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)),
                ("Free", ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p))]


class CLzmaProps(ctypes.Structure):
    _fields_ = [("lc", ctypes.c_uint), ("lp", ctypes.c_uint), ("pb", ctypes.c_uint),
                ("dicSize", ctypes.c_uint32)]


class CLzmaDec(ctypes.Structure):
    """Public layout of LzmaDec.h:50-69."""
    _fields_ = [("prop", CLzmaProps), ("probs", ctypes.c_void_p), ("dic", ctypes.c_void_p),
                ("buf", ctypes.c_void_p), ("range", ctypes.c_uint32), ("code", ctypes.c_uint32),
                ("dicPos", ctypes.c_size_t), ("dicBufSize", ctypes.c_size_t),
                ("processedPos", ctypes.c_uint32), ("checkDicSize", ctypes.c_uint32),
                ("state", ctypes.c_uint), ("reps", ctypes.c_uint32 * 4),
                ("remainLen", ctypes.c_uint), ("needFlush", ctypes.c_int),
                ("needInitState", ctypes.c_int), ("numProbs", ctypes.c_uint32),
                ("tempBufSize", ctypes.c_uint), ("tempBuf", ctypes.c_ubyte * 20)]


class CLzma2Dec(ctypes.Structure):
    _fields_ = [("decoder", CLzmaDec), ("packSize", ctypes.c_uint32),
                ("unpackSize", ctypes.c_uint32), ("state", ctypes.c_int),
                ("control", ctypes.c_ubyte), ("needInitDic", ctypes.c_int),
                ("needInitState", ctypes.c_int), ("needInitProp", ctypes.c_int)]


class StreamDesc(ctypes.Structure):
    _fields_ = [("src_off", ctypes.c_uint64), ("src_len", ctypes.c_uint64),
                ("dst_off", ctypes.c_uint64), ("dst_cap", ctypes.c_uint64),
                ("probs_off", ctypes.c_uint64), ("props", ctypes.c_ubyte * 5),
                ("props_size", ctypes.c_ubyte), ("finish_mode", ctypes.c_ubyte),
                ("kind", ctypes.c_ubyte)]


class Result(ctypes.Structure):
    _fields_ = [("res", ctypes.c_int32), ("status", ctypes.c_int32),
                ("dest_len", ctypes.c_uint64), ("src_len", ctypes.c_uint64)]


class LdsClass(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint64), ("lanes_per_group", ctypes.c_uint32),
                ("lds_cells_per_lane", ctypes.c_uint32), ("groups_per_cu", ctypes.c_uint32),
                ("waves_per_simd", ctypes.c_uint32), ("lds_mask", ctypes.c_uint32),
                ("flags", ctypes.c_uint32), ("slot_off", ctypes.c_uint64),
                ("slot_cells", ctypes.c_uint32), ("slot_groups", ctypes.c_uint32)]


class Plan(ctypes.Structure):
    _fields_ = [("workspace_bytes", ctypes.c_uint64), ("n", ctypes.c_uint64),
                ("n_lds", ctypes.c_uint64), ("lanes_per_group", ctypes.c_uint32),
                ("lds_cells_per_lane", ctypes.c_uint32), ("groups_per_cu", ctypes.c_uint32),
                ("waves_per_simd", ctypes.c_uint32), ("queue_offset", ctypes.c_uint64),
                ("persistent", ctypes.c_uint32), ("n_classes", ctypes.c_uint32),
                ("classes", LdsClass * 4)]


class PlanOptions(ctypes.Structure):
    """LzmaGpuPlanOptions (include/lzma_gpu.h): per-call planner overrides."""
    _fields_ = [("kernel", ctypes.c_uint32), ("cus", ctypes.c_uint32),
                ("lanes_per_group", ctypes.c_uint32), ("groups_per_cu", ctypes.c_uint32),
                ("waves_per_simd", ctypes.c_uint32), ("persistent", ctypes.c_uint32),
                ("coop", ctypes.c_uint32), ("one_class", ctypes.c_uint32),
                ("flags", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


KERNELS = {"auto": 0, "throughput": 1, "latency": 2, "coop": 3, "global": 4}


def plan_options(kernel="auto", **kw):
    """PlanOptions from a kernel name ('auto', 'throughput', 'latency', 'coop',
    'global') and any other LzmaGpuPlanOptions field by name."""
    o = PlanOptions()
    o.kernel = KERNELS[kernel]
    for k, v in kw.items():
        setattr(o, k, v)
    return o


class SlicedPlan(ctypes.Structure):
    """LzmaGpuSlicedPlan (include/lzma_gpu.h): a time-sliced batch."""
    _fields_ = [("workspace_bytes", ctypes.c_uint64), ("n", ctypes.c_uint64),
                ("slice_bytes", ctypes.c_uint64), ("rounds", ctypes.c_uint32),
                ("kernel", ctypes.c_uint32), ("table_cells", ctypes.c_uint32),
                ("groups_per_cu", ctypes.c_uint32), ("max_groups", ctypes.c_uint32),
                ("lds_mask", ctypes.c_uint32), ("sess_off", ctypes.c_uint64),
                ("list_off", ctypes.c_uint64), ("ctr_off", ctypes.c_uint64),
                ("n_inplace", ctypes.c_uint64)]


SLICED_KERNELS = {"auto": 0, "lane": 1, "coop": 2, "global": 3}


class Session(ctypes.Structure):
    """LzmaGpuSession: a device-resident decoder (include/lzma_gpu.h)."""
    _fields_ = [("lc", ctypes.c_uint32), ("lp", ctypes.c_uint32), ("pb", ctypes.c_uint32),
                ("dict_size", ctypes.c_uint32), ("probs", ctypes.c_void_p),
                ("dic", ctypes.c_void_p), ("in_", ctypes.c_void_p),
                ("dic_buf_size", ctypes.c_uint64), ("dic_pos", ctypes.c_uint64),
                ("dic_limit", ctypes.c_uint64), ("in_len", ctypes.c_uint64),
                ("in_used", ctypes.c_uint64), ("range", ctypes.c_uint32),
                ("code", ctypes.c_uint32), ("processed_pos", ctypes.c_uint32),
                ("check_dic_size", ctypes.c_uint32), ("state", ctypes.c_uint32),
                ("reps", ctypes.c_uint32 * 4), ("remain_len", ctypes.c_uint32),
                ("need_flush", ctypes.c_uint32), ("need_init_state", ctypes.c_uint32),
                ("temp_buf_size", ctypes.c_uint32), ("finish_mode", ctypes.c_int32),
                ("res", ctypes.c_int32), ("status", ctypes.c_int32), ("mode", ctypes.c_int32),
                ("temp_buf", ctypes.c_ubyte * 20), ("_pad", ctypes.c_ubyte * 4),
                ("out", ctypes.c_void_p), ("out_len", ctypes.c_uint64)]


class XzBlock(ctypes.Structure):
    """LzmaGpuXzBlock (include/lzma_gpu.h): one block of an indexed xz file."""
    _fields_ = [("header_off", ctypes.c_uint64), ("data_off", ctypes.c_uint64),
                ("pack_size", ctypes.c_uint64), ("unpack_size", ctypes.c_uint64),
                ("dst_off", ctypes.c_uint64), ("check_off", ctypes.c_uint64),
                ("check_type", ctypes.c_uint32), ("check_size", ctypes.c_uint32),
                ("lzma2_prop", ctypes.c_uint32), ("x86", ctypes.c_uint32),
                ("x86_ip", ctypes.c_uint32), ("stream", ctypes.c_uint32),
                ("num_filters", ctypes.c_uint32), ("filter_id", ctypes.c_uint32 * 3),
                ("filter_prop", ctypes.c_uint32 * 3)]


class Bcj2Job(ctypes.Structure):
    """Bcj2GpuJob (include/lzma_gpu.h): one BCJ2 decode, device pointers."""
    _fields_ = [("buf0", ctypes.c_void_p), ("buf1", ctypes.c_void_p), ("buf2", ctypes.c_void_p),
                ("buf3", ctypes.c_void_p), ("size0", ctypes.c_uint64), ("size1", ctypes.c_uint64),
                ("size2", ctypes.c_uint64), ("size3", ctypes.c_uint64), ("out", ctypes.c_void_p),
                ("out_size", ctypes.c_uint64)]


class SzFolder(ctypes.Structure):
    """LzmaGpu7zFolder (include/lzma_gpu.h): one folder of an opened 7z archive."""
    _fields_ = [("pack_off", ctypes.c_uint64), ("pack_size", ctypes.c_uint64),
                ("unpack_size", ctypes.c_uint64), ("dst_off", ctypes.c_uint64),
                ("method", ctypes.c_uint64), ("x86", ctypes.c_uint32),
                ("supported", ctypes.c_uint32), ("crc_defined", ctypes.c_uint32),
                ("crc", ctypes.c_uint32), ("first_file", ctypes.c_uint32),
                ("num_files", ctypes.c_uint32), ("num_coders", ctypes.c_uint32),
                ("props_size", ctypes.c_uint32), ("props", ctypes.c_ubyte * 8)]


class SzFile(ctypes.Structure):
    """LzmaGpu7zFile (include/lzma_gpu.h): one file entry of an opened 7z archive."""
    _fields_ = [("size", ctypes.c_uint64), ("dst_off", ctypes.c_uint64),
                ("folder", ctypes.c_uint32), ("crc", ctypes.c_uint32),
                ("crc_defined", ctypes.c_uint32), ("has_stream", ctypes.c_uint32),
                ("is_dir", ctypes.c_uint32), ("name_off", ctypes.c_uint32),
                ("name_len", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


assert ctypes.sizeof(XzBlock) == 104 and ctypes.sizeof(Bcj2Job) == 80
assert ctypes.sizeof(SzFolder) == 80 and ctypes.sizeof(SzFile) == 48
assert ctypes.sizeof(StreamDesc) == 48 and ctypes.sizeof(Result) == 24
assert ctypes.sizeof(Session) == 192 and ctypes.sizeof(Plan) == 248
assert ctypes.sizeof(PlanOptions) == 40
assert ctypes.sizeof(CLzmaDec) == 136

_P = ctypes.c_void_p
_sig = {
    "LzmaProps_Decode": (ctypes.c_int, [ctypes.POINTER(CLzmaProps), ctypes.c_char_p, ctypes.c_uint]),
    "LzmaDec_AllocateProbs": (ctypes.c_int, [ctypes.POINTER(CLzmaDec), ctypes.c_char_p, ctypes.c_uint, ctypes.POINTER(ISzAlloc)]),
    "LzmaDec_FreeProbs": (None, [ctypes.POINTER(CLzmaDec), ctypes.POINTER(ISzAlloc)]),
    "LzmaDec_Allocate": (ctypes.c_int, [ctypes.POINTER(CLzmaDec), ctypes.c_char_p, ctypes.c_uint, ctypes.POINTER(ISzAlloc)]),
    "LzmaDec_Free": (None, [ctypes.POINTER(CLzmaDec), ctypes.POINTER(ISzAlloc)]),
    "LzmaDec_Init": (None, [ctypes.POINTER(CLzmaDec)]),
    "LzmaDec_InitDicAndState": (None, [ctypes.POINTER(CLzmaDec), ctypes.c_int, ctypes.c_int]),
    "LzmaDec_DecodeToDic": (ctypes.c_int, [ctypes.POINTER(CLzmaDec), ctypes.c_size_t, _P, _sp, ctypes.c_int, _ip]),
    "LzmaDec_DecodeToBuf": (ctypes.c_int, [ctypes.POINTER(CLzmaDec), _P, _sp, _P, _sp, ctypes.c_int, _ip]),
    "LzmaGpu_DecoderRelease": (None, [ctypes.POINTER(CLzmaDec)]),
    "LzmaGpu_DropinTransferStats": (None, [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]),
    "LzmaGpu_CoalesceStats": (None, [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]),
    "LzmaDecode": (ctypes.c_int, [_P, _sp, _P, _sp, ctypes.c_char_p, ctypes.c_uint, ctypes.c_int, _ip, ctypes.POINTER(ISzAlloc)]),
    "LzmaUncompress": (ctypes.c_int, [_P, _sp, _P, _sp, ctypes.c_char_p, ctypes.c_size_t]),
    "Lzma2Dec_AllocateProbs": (ctypes.c_int, [ctypes.POINTER(CLzma2Dec), ctypes.c_ubyte, ctypes.POINTER(ISzAlloc)]),
    "Lzma2Dec_Allocate": (ctypes.c_int, [ctypes.POINTER(CLzma2Dec), ctypes.c_ubyte, ctypes.POINTER(ISzAlloc)]),
    "Lzma2Dec_Init": (None, [ctypes.POINTER(CLzma2Dec)]),
    "Lzma2Dec_DecodeToDic": (ctypes.c_int, [ctypes.POINTER(CLzma2Dec), ctypes.c_size_t, _P, _sp, ctypes.c_int, _ip]),
    "Lzma2Dec_DecodeToBuf": (ctypes.c_int, [ctypes.POINTER(CLzma2Dec), _P, _sp, _P, _sp, ctypes.c_int, _ip]),
    "Lzma2Decode": (ctypes.c_int, [_P, _sp, _P, _sp, ctypes.c_ubyte, ctypes.c_int, _ip, ctypes.POINTER(ISzAlloc)]),
    "LzmaGpu_PlanBatch": (ctypes.c_size_t, [ctypes.POINTER(StreamDesc), ctypes.c_size_t, _P]),
    "LzmaGpu_DecodeBatch": (ctypes.c_int, [_P, _P, ctypes.c_size_t, _P, _P, _P, ctypes.c_size_t, _P, _P]),
    "LzmaGpu_PlanBatchEx": (ctypes.c_int, [ctypes.POINTER(StreamDesc), ctypes.c_size_t, _P, ctypes.POINTER(Plan)]),
    "LzmaGpu_DecodeBatchEx": (ctypes.c_int, [ctypes.POINTER(Plan), _P, _P, _P, _P, _P, _P, _P]),
    "LzmaGpu_DecodeBatchHost": (ctypes.c_int, [ctypes.POINTER(StreamDesc), ctypes.c_size_t, _P, ctypes.c_size_t, _P, ctypes.c_size_t, ctypes.POINTER(Result)]),
    "LzmaGpu_PlanBatchOpt": (ctypes.c_int, [ctypes.POINTER(StreamDesc), ctypes.c_size_t, _P, ctypes.POINTER(Plan), ctypes.POINTER(PlanOptions)]),
    "LzmaGpu_DecodeBatchHostOpt": (ctypes.c_int, [ctypes.POINTER(StreamDesc), ctypes.c_size_t, _P, ctypes.c_size_t, _P, ctypes.c_size_t, ctypes.POINTER(Result), ctypes.POINTER(PlanOptions), ctypes.POINTER(Plan)]),
    "Lzma2Gpu_SplitBlocks": (ctypes.c_size_t, [_P, ctypes.c_size_t, _P, _P, _P, ctypes.c_size_t]),
    "LzmaGpu_SessionProbsBytes": (ctypes.c_size_t, [ctypes.c_char_p, ctypes.c_uint]),
    "LzmaGpu_SessionInit": (ctypes.c_int, [ctypes.POINTER(Session), ctypes.c_char_p, ctypes.c_uint, _P, _P, ctypes.c_size_t]),
    "LzmaGpu_SessionDecodeBatch": (ctypes.c_int, [_P, ctypes.c_size_t, _P]),
    "LzmaGpu_PlanSliced": (ctypes.c_int, [ctypes.POINTER(StreamDesc), ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint, _P, ctypes.POINTER(SlicedPlan)]),
    "LzmaGpu_DecodeBatchSliced": (ctypes.c_int, [ctypes.POINTER(SlicedPlan), _P, _P, _P, _P, _P, _P, ctypes.c_uint, ctypes.c_uint, _P]),
    "LzmaGpu_SlicedActive": (ctypes.c_int, [ctypes.POINTER(SlicedPlan), _P, ctypes.c_uint, _sp, _P]),
    "LzmaGpu_DecodeBatchSlicedHost": (ctypes.c_int, [ctypes.POINTER(StreamDesc), ctypes.c_size_t, _P, ctypes.c_size_t, _P, ctypes.c_size_t, ctypes.POINTER(Result), ctypes.c_uint64, ctypes.c_uint, ctypes.POINTER(SlicedPlan)]),
    "CrcGenerateTable": (None, []),
    "CrcUpdate": (ctypes.c_uint32, [ctypes.c_uint32, _P, ctypes.c_size_t]),
    "CrcCalc": (ctypes.c_uint32, [_P, ctypes.c_size_t]),
    "CrcGpu_PlanChunks": (ctypes.c_size_t, [_P, ctypes.c_size_t, _P, _P]),
    "CrcGpu_Batch": (ctypes.c_int, [_P, _P, _P, ctypes.c_size_t, _P, _P, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32, _P, _P, _P]),
    "LzmaGpu_Crc32Plan": (ctypes.c_size_t, [ctypes.POINTER(StreamDesc), ctypes.c_size_t, _P, _P]),
    "LzmaGpu_Crc32Batch": (ctypes.c_int, [_P, _P, ctypes.c_size_t, _P, _P, _P, ctypes.c_size_t, _P, _P, _P]),
    "x86_Convert": (ctypes.c_size_t, [_P, ctypes.c_size_t, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32), ctypes.c_int]),
    "BcjGpu_X86Batch": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, ctypes.c_size_t, ctypes.c_int, _P]),
    "ARM_Convert": (ctypes.c_size_t, [_P, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int]),
    "ARMT_Convert": (ctypes.c_size_t, [_P, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int]),
    "PPC_Convert": (ctypes.c_size_t, [_P, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int]),
    "SPARC_Convert": (ctypes.c_size_t, [_P, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int]),
    "IA64_Convert": (ctypes.c_size_t, [_P, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int]),
    "Delta_Init": (None, [_P]),
    "Delta_Encode": (None, [_P, ctypes.c_uint, _P, ctypes.c_size_t]),
    "Delta_Decode": (None, [_P, ctypes.c_uint, _P, ctypes.c_size_t]),
    "BraGpu_Batch": (ctypes.c_int, [ctypes.c_uint, _P, _P, _P, _P, _P, ctypes.c_size_t, ctypes.c_int, _P]),
    "DeltaGpu_Batch": (ctypes.c_int, [_P, _P, _P, _P, _P, ctypes.c_size_t, ctypes.c_int, _P]),
    "Bcj2_Decode": (ctypes.c_int, [_P, ctypes.c_size_t, _P, ctypes.c_size_t, _P, ctypes.c_size_t, _P, ctypes.c_size_t, _P, ctypes.c_size_t]),
    "Bcj2Gpu_Batch": (ctypes.c_int, [_P, ctypes.c_size_t, _P, _P]),
    "Crc64Calc": (ctypes.c_uint64, [_P, ctypes.c_size_t]),
    "Crc64Gpu_Batch": (ctypes.c_int, [_P, _P, _P, ctypes.c_size_t, _P, _P, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64, _P, _P, _P]),
    "LzmaGpu_XzIndex": (ctypes.c_int, [_P, ctypes.c_size_t, ctypes.POINTER(XzBlock), ctypes.c_size_t, _sp, ctypes.POINTER(ctypes.c_uint64)]),
    "LzmaGpu_XzDecode": (ctypes.c_int, [_P, _sp, _P, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int64)]),
    "LzmaGpu_7zOpen": (ctypes.c_int, [_P, ctypes.c_size_t, _P, ctypes.c_size_t, _sp, _P,
                                      ctypes.c_size_t, _sp, _P, ctypes.c_size_t, _sp,
                                      ctypes.POINTER(ctypes.c_uint64)]),
    "LzmaGpu_7zExtract": (ctypes.c_int, [_P, _sp, _P, ctypes.c_size_t, _P, ctypes.c_size_t]),
    "LzmaGpu_DeviceCount": (ctypes.c_int, []),
    "LzmaGpu_LastError": (ctypes.c_char_p, []),
    "LzmaGpu_Version": (ctypes.c_char_p, []),
}
for _name, (_rt, _at) in _sig.items():
    _f = getattr(_lib, _name)
    _f.restype = _rt
    _f.argtypes = _at

EXPORTED = tuple(_sig)
lib = _lib

_libc = ctypes.CDLL(None)
_libc.malloc.restype = ctypes.c_void_p
_libc.malloc.argtypes = [ctypes.c_size_t]
_libc.free.argtypes = [ctypes.c_void_p]


@ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)
def _py_alloc(_p, n):
    return _libc.malloc(n if n else 1)


@ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p)
def _py_free(_p, a):
    _libc.free(a)


g_alloc = ISzAlloc(_py_alloc, _py_free)


def transfer_stats(reset=False):
    """(h2d_bytes, d2h_bytes, calls) of the drop-in entry points
    (LzmaGpu_DropinTransferStats); reset zeroes the counters after reading."""
    h, d, c = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
    _lib.LzmaGpu_DropinTransferStats(ctypes.byref(h), ctypes.byref(d), ctypes.byref(c),
                                     1 if reset else 0)
    return h.value, d.value, c.value


def last_error():
    return _lib.LzmaGpu_LastError().decode()


def device_count():
    return _lib.LzmaGpu_DeviceCount()


def _buf(data):
    return ctypes.create_string_buffer(bytes(data), max(len(data), 1))


# ---------------------------------------------------------------- one-call API

def coalesce_stats(reset=False):
    """(batches, calls, largest batch) of the one-call coalescer
    (LzmaGpu_CoalesceStats); reset zeroes the counters after reading."""
    b, c, m = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    _lib.LzmaGpu_CoalesceStats(ctypes.byref(b), ctypes.byref(c), ctypes.byref(m),
                               1 if reset else 0)
    return b.value, c.value, m.value


def LzmaDecode(src, props, dest_cap, finish=LZMA_FINISH_END):
    """LzmaDecode (LzmaDec.c:972). Returns (res, status, destLen, srcLen, out)."""
    s = _buf(src)
    d = ctypes.create_string_buffer(max(dest_cap, 1))
    dl = ctypes.c_size_t(dest_cap)
    sl = ctypes.c_size_t(len(src))
    st = ctypes.c_int(-1)
    res = _lib.LzmaDecode(d, ctypes.byref(dl), s, ctypes.byref(sl), bytes(props), len(props),
                          finish, ctypes.byref(st), ctypes.byref(g_alloc))
    return res, st.value, dl.value, sl.value, d.raw[:dl.value]


def LzmaUncompress(src, props, dest_cap):
    """LzmaUncompress (LzmaLib.c:41). Returns (res, destLen, srcLen, out)."""
    s = _buf(src)
    d = ctypes.create_string_buffer(max(dest_cap, 1))
    dl = ctypes.c_size_t(dest_cap)
    sl = ctypes.c_size_t(len(src))
    res = _lib.LzmaUncompress(d, ctypes.byref(dl), s, ctypes.byref(sl), bytes(props), len(props))
    return res, dl.value, sl.value, d.raw[:dl.value]


def Lzma2Decode(src, prop, dest_cap, finish=LZMA_FINISH_END):
    s = _buf(src)
    d = ctypes.create_string_buffer(max(dest_cap, 1))
    dl = ctypes.c_size_t(dest_cap)
    sl = ctypes.c_size_t(len(src))
    st = ctypes.c_int(-1)
    res = _lib.Lzma2Decode(d, ctypes.byref(dl), s, ctypes.byref(sl), prop, finish,
                           ctypes.byref(st), ctypes.byref(g_alloc))
    return res, st.value, dl.value, sl.value, d.raw[:dl.value]


# ---------------------------------------------------------------- streaming API

def stream_decode(src, props, out_total, in_chunk, out_chunk, finish, max_calls=100000):
    """zlib-like loop over LzmaDec_DecodeToBuf with bounded chunks -- the same
    contract as the oracle's orc_lzma_stream_decode / the fork's
    SzDecodeLzmaToFileWithBuf (7zDec.c:567-648).
    Returns (calls, trace[(res, status, srcLen, destLen)], out, in_used)."""
    dec = CLzmaDec()
    dec.dic = None
    dec.probs = None
    r = _lib.LzmaDec_Allocate(ctypes.byref(dec), bytes(props), 5, ctypes.byref(g_alloc))
    if r != SZ_OK:
        return -r, [], b"", 0
    _lib.LzmaDec_Init(ctypes.byref(dec))
    sbuf = _buf(src)
    out = ctypes.create_string_buffer(max(out_total, 1))
    base_s = ctypes.addressof(sbuf)
    base_o = ctypes.addressof(out)
    in_pos = out_pos = 0
    trace = []
    try:
        while len(trace) < max_calls:
            sl = ctypes.c_size_t(min(len(src) - in_pos, in_chunk))
            dl = ctypes.c_size_t(min(out_total - out_pos, out_chunk))
            st = ctypes.c_int(-1)
            res = _lib.LzmaDec_DecodeToBuf(ctypes.byref(dec), base_o + out_pos, ctypes.byref(dl),
                                           base_s + in_pos, ctypes.byref(sl), finish,
                                           ctypes.byref(st))
            trace.append((res, st.value, sl.value, dl.value))
            in_pos += sl.value
            out_pos += dl.value
            if res != SZ_OK or st.value == 1 or out_pos == out_total:
                break
            if sl.value == 0 and dl.value == 0:
                break
    finally:
        _lib.LzmaDec_Free(ctypes.byref(dec), ctypes.byref(g_alloc))
    return len(trace), trace, out.raw[:out_pos], in_pos


def dic_decode(src, props, out_total, win, max_calls=100000, out=None, between=None):
    """The 7zDec.c:127-171 (SzDecodeLzma) loop over LzmaDec_DecodeToDic:
    LzmaDec_AllocateProbs, dic = the whole output buffer (dicBufSize =
    out_total), LzmaDec_Init, then DecodeToDic(out_total, FINISH_END) over look
    windows of at most `win` input bytes -- the same contract as the oracle's
    orc_lzma_dic_decode.  `out` (optional): a ctypes buffer of >= out_total bytes
    to decode into.  `between` (optional): called with (call index, the
    CLzmaDec) after every call.  Returns (calls, trace[(res, status, srcLen,
    dicPos)], out bytes, in_used)."""
    dec = CLzmaDec()
    dec.dic = None
    dec.probs = None
    r = _lib.LzmaDec_AllocateProbs(ctypes.byref(dec), bytes(props), 5, ctypes.byref(g_alloc))
    if r != SZ_OK:
        return -r, [], b"", 0
    sbuf = _buf(src)
    if out is None:
        out = ctypes.create_string_buffer(max(out_total, 1))
    dec.dic = ctypes.addressof(out)
    dec.dicBufSize = out_total
    _lib.LzmaDec_Init(ctypes.byref(dec))
    base_s = ctypes.addressof(sbuf)
    in_pos = 0
    trace = []
    try:
        while len(trace) < max_calls:
            sl = ctypes.c_size_t(min(len(src) - in_pos, win))
            pos0 = dec.dicPos
            st = ctypes.c_int(-1)
            res = _lib.LzmaDec_DecodeToDic(ctypes.byref(dec), out_total, base_s + in_pos,
                                           ctypes.byref(sl), LZMA_FINISH_END, ctypes.byref(st))
            trace.append((res, st.value, sl.value, dec.dicPos))
            in_pos += sl.value
            if res != SZ_OK:
                break
            if dec.dicPos == out_total or (sl.value == 0 and dec.dicPos == pos0):
                break
            if between is not None:
                between(len(trace) - 1, dec)
    finally:
        _lib.LzmaDec_FreeProbs(ctypes.byref(dec), ctypes.byref(g_alloc))
    return len(trace), trace, out.raw[:dec.dicPos], in_pos


# ---------------------------------------------------------------- batch API

def make_descs(items):
    """items: list of dicts with src_off, src_len, dst_off, dst_cap, props(bytes),
    finish, kind.  Returns a ctypes StreamDesc array."""
    arr = (StreamDesc * len(items))()
    for i, it in enumerate(items):
        d = arr[i]
        d.src_off, d.src_len = it["src_off"], it["src_len"]
        d.dst_off, d.dst_cap = it["dst_off"], it["dst_cap"]
        p = bytes(it["props"])
        for k in range(min(len(p), 5)):
            d.props[k] = p[k]
        d.props_size = it.get("props_size", len(p))
        d.finish_mode = it.get("finish", LZMA_FINISH_END)
        d.kind = it.get("kind", KIND_LZMA)
    return arr


def decode_batch_host(descs, src, dst_bytes, opts=None, plan_out=None):
    """Decode a batch from host buffers.  Returns (res, results[ctypes], dst bytes).
    opts: PlanOptions (None = the planner's defaults); plan_out: a Plan to receive
    the plan that ran."""
    n = len(descs)
    res = (Result * max(n, 1))()
    s = _buf(src)
    d = ctypes.create_string_buffer(max(dst_bytes, 1))
    if opts is None and plan_out is None:
        r = _lib.LzmaGpu_DecodeBatchHost(descs, n, s, len(src), d, dst_bytes, res)
    else:
        r = _lib.LzmaGpu_DecodeBatchHostOpt(descs, n, s, len(src), d, dst_bytes, res,
                                            ctypes.byref(opts) if opts is not None else None,
                                            ctypes.byref(plan_out) if plan_out is not None
                                            else None)
    return r, res, d.raw[:dst_bytes]


def plan(descs, order=None):
    """Fill probs_off (and the lane order, a ctypes uint32 array). Returns workspace bytes."""
    return _lib.LzmaGpu_PlanBatch(descs, len(descs), order)


def plan_ex(descs, opts=None):
    """LzmaGpu_PlanBatchEx (or LzmaGpu_PlanBatchOpt when opts is a PlanOptions):
    returns (Plan, order[ctypes uint32 array])."""
    n = len(descs)
    order = (ctypes.c_uint32 * max(n, 1))()
    p = Plan()
    if opts is None:
        r = _lib.LzmaGpu_PlanBatchEx(descs, n, order, ctypes.byref(p))
    else:
        r = _lib.LzmaGpu_PlanBatchOpt(descs, n, order, ctypes.byref(p), ctypes.byref(opts))
    if r != SZ_OK:
        raise RuntimeError(f"LzmaGpu_PlanBatchEx failed: {r}")
    return p, order


def decode_batch_device_ex(plan, d_descs, d_order, d_src, d_dst, d_ws, d_results, stream=0):
    """LzmaGpu_DecodeBatchEx over raw device pointers (ints)."""
    return _lib.LzmaGpu_DecodeBatchEx(ctypes.byref(plan), d_descs, d_order, d_src, d_dst, d_ws,
                                      d_results, stream or None)


def decode_batch_device(d_descs, d_order, n, d_src, d_dst, d_ws, ws_bytes, d_results, stream=0):
    """All arguments are raw device pointers (ints); stream is a hipStream_t (int)."""
    return _lib.LzmaGpu_DecodeBatch(d_descs, d_order, n, d_src, d_dst, d_ws, ws_bytes, d_results,
                                    stream or None)


def plan_sliced(descs, slice_bytes, kernel="auto"):
    """LzmaGpu_PlanSliced: fills descs' probs_off; returns (SlicedPlan, order)."""
    n = len(descs)
    order = (ctypes.c_uint32 * max(n, 1))()
    p = SlicedPlan()
    r = _lib.LzmaGpu_PlanSliced(descs, n, slice_bytes, SLICED_KERNELS[kernel], order,
                                ctypes.byref(p))
    if r != SZ_OK:
        raise RuntimeError(f"LzmaGpu_PlanSliced failed: {r}")
    return p, order


def decode_batch_sliced_device(plan, d_descs, d_order, d_src, d_dst, d_ws, d_results,
                               first_round=0, n_rounds=0, stream=0):
    """LzmaGpu_DecodeBatchSliced over raw device pointers (ints)."""
    return _lib.LzmaGpu_DecodeBatchSliced(ctypes.byref(plan), d_descs, d_order, d_src, d_dst,
                                          d_ws, d_results, first_round, n_rounds, stream or None)


def sliced_active(plan, d_ws, round_, stream=0):
    """Streams still unfinished entering round `round_` (synchronises `stream`)."""
    v = ctypes.c_size_t(0)
    r = _lib.LzmaGpu_SlicedActive(ctypes.byref(plan), d_ws, round_, ctypes.byref(v), stream or None)
    if r != SZ_OK:
        raise RuntimeError(f"LzmaGpu_SlicedActive failed: {r}")
    return v.value


def decode_batch_sliced_host(descs, src, dst_bytes, slice_bytes, kernel="auto", plan_out=None):
    """Time-sliced batch from host buffers: (res, results[ctypes], dst bytes)."""
    n = len(descs)
    res = (Result * max(n, 1))()
    s = _buf(src)
    d = ctypes.create_string_buffer(max(dst_bytes, 1))
    r = _lib.LzmaGpu_DecodeBatchSlicedHost(descs, n, s, len(src), d, dst_bytes, res, slice_bytes,
                                           SLICED_KERNELS[kernel],
                                           ctypes.byref(plan_out) if plan_out is not None else None)
    return r, res, d.raw[:dst_bytes]


def split_lzma2_blocks(src):
    """Lzma2Gpu_SplitBlocks: list of (src_off, src_len, unpack) per dict-reset block."""
    cap = max(16, len(src) // 16)
    s = _buf(src)
    while True:
        o = (ctypes.c_uint64 * cap)()
        ln = (ctypes.c_uint64 * cap)()
        u = (ctypes.c_uint64 * cap)()
        nb = _lib.Lzma2Gpu_SplitBlocks(s, len(src), o, ln, u, cap)
        if nb == ctypes.c_size_t(-1).value:
            raise ValueError("malformed LZMA2 chunk headers")
        if nb <= cap:
            return [(o[i], ln[i], u[i]) for i in range(nb)]
        cap = nb


# ---------------------------------------------------------------- CRC-32 (7zCrc.h)

CRC_CHUNK = 2048  # kCrcChunk in csrc/crc32_device.h


def CrcCalc(data):
    """7zCrc.c CrcCalc on the GPU (host buffer in, CRC out)."""
    return _lib.CrcCalc(_buf(data), len(data))


def CrcUpdate(crc, data):
    """7zCrc.c CrcUpdate (raw register, no final XOR) on the GPU."""
    return _lib.CrcUpdate(crc, _buf(data), len(data))


def crc_plan(caps):
    """CrcGpu_PlanChunks: (chunk_base[n], chunk_range[n_chunks]) as ctypes arrays."""
    n = len(caps)
    c = (ctypes.c_uint64 * max(n, 1))(*caps)
    total = _lib.CrcGpu_PlanChunks(c, n, None, None)
    if total == ctypes.c_size_t(-1).value:
        raise ValueError("too many CRC chunks")
    base = (ctypes.c_uint32 * max(n, 1))()
    rng = (ctypes.c_uint32 * max(total, 1))()
    _lib.CrcGpu_PlanChunks(c, n, base, rng)
    return base, rng, total


def crc32_plan_decoded(descs):
    """LzmaGpu_Crc32Plan over planned decode descriptors (host)."""
    n = len(descs)
    total = _lib.LzmaGpu_Crc32Plan(descs, n, None, None)
    base = (ctypes.c_uint32 * max(n, 1))()
    rng = (ctypes.c_uint32 * max(total, 1))()
    _lib.LzmaGpu_Crc32Plan(descs, n, base, rng)
    return base, rng, total


def crc_batch_device(d_data, d_off, d_len, n, d_base, d_range, n_chunks, init, xorout,
                     d_chunk_crc, d_crc, stream=0):
    """CrcGpu_Batch over raw device pointers (ints)."""
    return _lib.CrcGpu_Batch(d_data, d_off, d_len, n, d_base, d_range, n_chunks, init, xorout,
                             d_chunk_crc, d_crc, stream or None)


def crc32_batch_decoded(d_descs, d_results, n, d_dst, d_base, d_range, n_chunks, d_chunk_crc,
                        d_crc, stream=0):
    """LzmaGpu_Crc32Batch over raw device pointers (ints)."""
    return _lib.LzmaGpu_Crc32Batch(d_descs, d_results, n, d_dst, d_base, d_range, n_chunks,
                                   d_chunk_crc, d_crc, stream or None)


# ---------------------------------------------------------------- xz, x86 BCJ, CRC-64

def x86_Convert(data, ip=0, state=0, encoding=0):
    """Bra86.c x86_Convert on the GPU: (processed, state, converted bytes)."""
    b = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
    st = ctypes.c_uint32(state)
    n = _lib.x86_Convert(b, len(data), ip, ctypes.byref(st), encoding)
    return n, st.value, b.raw[:len(data)]


BRA_KINDS = {"PPC": 5, "IA64": 6, "ARM": 7, "ARMT": 8, "SPARC": 9}


def bra_convert(kind, data, ip=0, encoding=0):
    """Bra.c / BraIA64.c <kind>_Convert on the GPU: (processed, converted bytes)."""
    b = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
    n = getattr(_lib, kind + "_Convert")(b, len(data), ip, encoding)
    return n, b.raw[:len(data)]


def delta_convert(data, delta, state=b"", encoding=0):
    """Delta.c Delta_Decode (encoding 0) / Delta_Encode on the GPU: (state, bytes)."""
    st = ctypes.create_string_buffer(bytes(state).ljust(256, b"\0")[:256], 256)
    b = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
    (_lib.Delta_Encode if encoding else _lib.Delta_Decode)(st, delta, b, len(data))
    return st.raw, b.raw[:len(data)]


def bra_batch_device(kind, d_data, d_off, d_len, d_ip, d_done, n, encoding=0, stream=0):
    """BraGpu_Batch over raw device pointers (ints)."""
    return _lib.BraGpu_Batch(kind, d_data, d_off, d_len, d_ip, d_done, n, encoding, stream or None)


def delta_batch_device(d_data, d_off, d_len, d_delta, d_state, n, encoding=0, stream=0):
    """DeltaGpu_Batch over raw device pointers (ints)."""
    return _lib.DeltaGpu_Batch(d_data, d_off, d_len, d_delta, d_state, n, encoding, stream or None)


def Bcj2_Decode(main, call, jump, rc, out_size, overlap=False, fill=0xA5):
    """Bcj2.c Bcj2_Decode on the GPU over host buffers: (res, output buffer).
    The output buffer starts as `fill` bytes; overlap: the main stream sits at
    its tail (the 7zDec.c:367-372 layout)."""
    out = ctypes.create_string_buffer(bytes([fill]) * max(out_size, 1), max(out_size, 1))
    bufs = [_buf(x) for x in (call, jump, rc)]
    if overlap:
        at = out_size - len(main)
        ctypes.memmove(ctypes.addressof(out) + at, bytes(main), len(main))
        m = ctypes.addressof(out) + at
    else:
        mb = _buf(main)
        m = ctypes.addressof(mb)
    r = _lib.Bcj2_Decode(m, len(main), bufs[0], len(call), bufs[1], len(jump), bufs[2], len(rc),
                         out, out_size)
    return r, out.raw[:out_size]


def bcj2_batch_device(d_jobs, n, d_res, stream=0):
    """Bcj2Gpu_Batch over a device array of n Bcj2Job."""
    return _lib.Bcj2Gpu_Batch(d_jobs, n, d_res, stream or None)


def Crc64Calc(data):
    """XzCrc64.c Crc64Calc on the GPU."""
    return _lib.Crc64Calc(_buf(data), len(data))


def bcj_x86_batch_device(d_data, d_off, d_len, d_ip, d_state, d_done, n, encoding=0, stream=0):
    """BcjGpu_X86Batch over raw device pointers (ints)."""
    return _lib.BcjGpu_X86Batch(d_data, d_off, d_len, d_ip, d_state, d_done, n, encoding,
                                stream or None)


def crc64_batch_device(d_data, d_off, d_len, n, d_base, d_range, n_chunks, init, xorout,
                       d_chunk_crc, d_crc, stream=0):
    """Crc64Gpu_Batch over raw device pointers (ints)."""
    return _lib.Crc64Gpu_Batch(d_data, d_off, d_len, n, d_base, d_range, n_chunks, init, xorout,
                               d_chunk_crc, d_crc, stream or None)


def xz_index(data):
    """LzmaGpu_XzIndex: (res, [XzBlock...], unpack_total).  Host only."""
    n = ctypes.c_size_t(0)
    tot = ctypes.c_uint64(0)
    src = _buf(data)
    r = _lib.LzmaGpu_XzIndex(src, len(data), None, 0, ctypes.byref(n), ctypes.byref(tot))
    if r != SZ_OK:
        return r, [], 0
    arr = (XzBlock * max(n.value, 1))()
    r = _lib.LzmaGpu_XzIndex(src, len(data), arr, n.value, ctypes.byref(n), ctypes.byref(tot))
    return r, list(arr)[:n.value], tot.value


def XzDecode(data, dest_cap):
    """LzmaGpu_XzDecode: (res, output bytes, bad_block)."""
    out = ctypes.create_string_buffer(max(dest_cap, 1))
    dl = ctypes.c_size_t(dest_cap)
    bad = ctypes.c_int64(-1)
    r = _lib.LzmaGpu_XzDecode(out, ctypes.byref(dl), _buf(data), len(data), ctypes.byref(bad))
    return r, out.raw[:dl.value], bad.value


def sz_open(data):
    """LzmaGpu_7zOpen: (res, [SzFolder...], [SzFile...], names (UTF-16LE bytes),
    unpack_total).  A packed header is decoded on the GPU."""
    nfo, nfi, nn = ctypes.c_size_t(0), ctypes.c_size_t(0), ctypes.c_size_t(0)
    tot = ctypes.c_uint64(0)
    src = _buf(data)
    r = _lib.LzmaGpu_7zOpen(src, len(data), None, 0, ctypes.byref(nfo), None, 0,
                            ctypes.byref(nfi), None, 0, ctypes.byref(nn), ctypes.byref(tot))
    if r != SZ_OK:
        return r, [], [], b"", 0
    fo = (SzFolder * max(nfo.value, 1))()
    fi = (SzFile * max(nfi.value, 1))()
    names = (ctypes.c_uint16 * max(nn.value, 1))()
    r = _lib.LzmaGpu_7zOpen(src, len(data), fo, nfo.value, ctypes.byref(nfo), fi, nfi.value,
                            ctypes.byref(nfi), names, nn.value, ctypes.byref(nn),
                            ctypes.byref(tot))
    raw = bytes(bytearray(ctypes.string_at(names, 2 * nn.value)))
    return r, list(fo)[:nfo.value], list(fi)[:nfi.value], raw, tot.value


def SzExtract(data, dest_cap, max_files=1 << 16):
    """LzmaGpu_7zExtract: (res, extraction buffer, [per-file SRes])."""
    out = ctypes.create_string_buffer(max(dest_cap, 1))
    dl = ctypes.c_size_t(dest_cap)
    fres = (ctypes.c_int * max_files)()
    r = _lib.LzmaGpu_7zExtract(out, ctypes.byref(dl), _buf(data), len(data), fres, max_files)
    return r, out.raw[:dl.value], list(fres)


# ---------------------------------------------------------------- streaming sessions

def session_probs_bytes(props):
    return _lib.LzmaGpu_SessionProbsBytes(bytes(props), len(props))


def session_init(props, d_probs, d_dic, dic_buf_size):
    """Host-side LzmaDec_Allocate + LzmaDec_Init on a fresh Session (device pointers in)."""
    s = Session()
    r = _lib.LzmaGpu_SessionInit(ctypes.byref(s), bytes(props), len(props), d_probs, d_dic,
                                 dic_buf_size)
    return r, s


def session_decode_batch(d_sessions, n, stream=0):
    """LzmaGpu_SessionDecodeBatch over a device array of n Sessions."""
    return _lib.LzmaGpu_SessionDecodeBatch(d_sessions, n, stream or None)

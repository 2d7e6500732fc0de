"""redrock_old_amd — MI355X-native batch serialize/deserialize engine for RedRock value blobs.

The product is the C-ABI library ``redrock_old_amd/librr_serdes.so`` (include/rr_serdes.h):
hand-written gfx950 HIP kernels behind a plain-C host layer.  This module is a thin ctypes
binding used by the tests, ``bench.py`` and ``__graft_entry__``; it adds no compute of its own
and has no CPU fallback: if the library is missing or no GPU is present, calls raise.

Reference interface it mirrors (src/rock_serdes.h:47-49): ``serObject`` / ``desObject`` turn
one Redis object into a blob and back; here ``Engine.encode*`` / ``Engine.decode*`` do the same
for whole batches in the flat form of include/rr_format.h.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# RR_LIB selects an alternative in-tree build (e.g. the probe build librr_serdes_probe.so).
LIB_PATH = os.path.join(_HERE, os.environ.get("RR_LIB", "librr_serdes.so"))

# --- flat form dtypes (include/rr_format.h) ---------------------------------------------
VALUE_DT = np.dtype([("type", "u1"), ("enc", "u1"), ("status", "<u2"), ("lru", "<u4"),
                     ("n_elems", "<u4"), ("elem_base", "<u4")])
ELEM_DT = np.dtype([("data", "<u8"), ("len", "<u4"), ("kind", "u1"), ("zenc", "u1"), ("rsv", "<u2")])
assert VALUE_DT.itemsize == 16 and ELEM_DT.itemsize == 16

T_STRING, T_SET_HT, T_HASH_HT, T_ZSET_SKIPLIST = 0, 2, 4, 5
T_SET_INTSET, T_ZSET_ZIPLIST, T_HASH_ZIPLIST, T_LIST_QUICKLIST = 11, 12, 13, 14
K_STR, K_INT, K_SCORE, K_ZLRAW = 0, 1, 2, 3
STATUS_NAMES = {0: "OK", 1: "SHORT", 2: "TYPE", 3: "STR_ENC", 4: "STR_INTLEN", 5: "EMBSTR_LEN",
                6: "TRUNC", 7: "COUNT", 8: "INTSET", 9: "ZL_LEN", 10: "ZL_CORRUPT", 11: "CAPACITY",
                12: "ENCODE", 13: "DUP", 14: "NAN"}

CONFIG_MIXED = 4
CTX_NO_SMALL = 1          # rr_ctx_set_options: no one-launch small-batch kernels
SMALL_N, SMALL_BYTES = 4096, 128 * 1024   # the one-launch kernels' limits (rr_serdes.h)


class RRError(RuntimeError):
    pass


class Totals(C.Structure):
    _fields_ = [("n_elems", C.c_uint64), ("bytes", C.c_uint64), ("n_bad", C.c_uint64),
                ("payload", C.c_uint64)]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


class BlobBatch(C.Structure):
    _fields_ = [("data", C.c_void_p), ("offsets", C.c_void_p), ("n", C.c_uint64), ("data_cap", C.c_uint64)]


class FlatBatch(C.Structure):
    _fields_ = [("values", C.c_void_p), ("elems", C.c_void_p), ("arena", C.c_void_p), ("n", C.c_uint64),
                ("elem_cap", C.c_uint64), ("arena_cap", C.c_uint64)]


class Shard(C.Structure):
    _fields_ = [("v0", C.c_uint64), ("v1", C.c_uint64), ("b0", C.c_uint64), ("b1", C.c_uint64)]


class Xfer(C.Structure):
    _fields_ = [("peer", C.c_int32), ("dir", C.c_int32), ("buf", C.c_int32), ("rsv", C.c_int32),
                ("offset", C.c_uint64), ("bytes", C.c_uint64)]


# rr_xfer directions and buffers (include/rr_serdes.h)
XFER_SEND, XFER_RECV = 0, 1
BUF_WHOLE_DATA, BUF_WHOLE_OFFSETS, BUF_MINE_DATA, BUF_MINE_OFFSETS = 0, 1, 2, 3
BUF_MINE_VALUES, BUF_MINE_ELEMS, BUF_WHOLE_VALUES, BUF_WHOLE_ELEMS = 4, 5, 6, 7


class HostBatch(C.Structure):
    _fields_ = [("data", C.POINTER(C.c_uint8)), ("offsets", C.POINTER(C.c_uint64)), ("n", C.c_uint64),
                ("bytes", C.c_uint64)]


# Every symbol include/rr_serdes.h declares (the ABI test checks they are all exported).
EXPORTS = ["rr_ctx_create", "rr_ctx_destroy", "rr_ctx_reserve", "rr_last_error", "rr_decode_batch",
           "rr_encode_batch", "rr_decode_elem_bound", "rr_decode_batch_host", "rr_encode_batch_host",
           "rr_gen_batch", "rr_host_batch_free", "rr_gen_default_seed", "rr_shard_plan", "rr_flat_rebase",
           "rr_comm_get_id", "rr_comm_init", "rr_comm_destroy", "rr_split_plan", "rr_split", "rr_gather",
           "rr_flat_rebase_host", "rr_gather_layout", "rr_copy_device", "rr_gen_sizes", "rr_gen_range",
           "rr_split_schedule", "rr_gather_schedule", "rr_ctx_set_options"]
COMM_ID_BYTES = 128
# include/rr_snappy.h (GPU block compression)
SNAPPY_EXPORTS = ["rr_snappy_max_compressed_length", "rr_snappy_compress_bound", "rr_snappy_compress_batch",
                  "rr_snappy_decompress_batch", "rr_snappy_compress_batch_host", "rr_snappy_decompress_batch_host"]
# include/rr_rdb.h (batched snapshot restore over the fork-child pipes, row f4; used from C)
RDB_EXPORTS = ["rr_rdb_request_batch", "rr_rdb_blobs_free", "rr_rdb_request_flat", "rr_rdb_flat_free", "rr_rdb_serve"]
# include/rr_kv.h (batched store I/O around the GPU path, row f2; used from C)
KV_EXPORTS = ["rr_kv_dump_batch", "rr_kv_restore_batch"]
# include/rr_host.h (the host codec: RedRock's per-key call sites through the compat shim, row f1)
HOST_EXPORTS = ["rr_host_reserve", "rr_host_decode_value", "rr_host_check_value", "rr_host_decode_batch",
                "rr_host_encode_size", "rr_host_encode_value", "rr_host_encode_batch"]
SNAPPY_STATUS = {0: "OK", 1: "HEADER", 2: "TRUNC", 3: "OFFSET", 4: "OVERFLOW", 5: "LENGTH", 6: "CAPACITY"}

_lib = None


def lib():
    """Load the in-tree engine library (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RRError(f"{LIB_PATH} not built: run __graft_entry__.build()")
    # torch (used for device buffers and streams) ships its own libamdhip64.so.7; load it first
    # so this library binds to the same HIP runtime instead of a second copy from /opt/rocm.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    vp, u64 = C.c_void_p, C.c_uint64
    L.rr_ctx_create.argtypes = [C.c_int, C.POINTER(vp)]
    L.rr_ctx_destroy.argtypes = [vp]
    L.rr_ctx_destroy.restype = None
    L.rr_ctx_reserve.argtypes = [vp, u64, u64]
    if hasattr(L, "rr_ctx_set_options"):   # (RR_LIB: an older build for A/B timing may predate it)
        L.rr_ctx_set_options.argtypes = [vp, C.c_uint]
    if hasattr(L, "rr_debug_fail_second"):   # test hook, not in rr_serdes.h
        L.rr_debug_fail_second.argtypes = [vp]
    if hasattr(L, "rr_debug_one_help"):   # test hook, not in rr_serdes.h
        L.rr_debug_one_help.argtypes = [vp]
    L.rr_last_error.restype = C.c_char_p
    L.rr_decode_batch.argtypes = [vp, C.POINTER(BlobBatch), C.POINTER(FlatBatch), vp, vp]
    L.rr_encode_batch.argtypes = [vp, C.POINTER(FlatBatch), C.POINTER(BlobBatch), vp, vp]
    L.rr_decode_elem_bound.argtypes = [u64, u64]
    L.rr_decode_elem_bound.restype = u64
    L.rr_decode_batch_host.argtypes = [vp, vp, vp, u64, vp, vp, u64, vp, C.POINTER(Totals)]
    L.rr_encode_batch_host.argtypes = [vp, vp, vp, u64, vp, u64, u64, vp, u64, vp, C.POINTER(Totals)]
    L.rr_gen_batch.argtypes = [C.c_int, u64, u64, C.POINTER(HostBatch)]
    L.rr_host_batch_free.argtypes = [C.POINTER(HostBatch)]
    L.rr_host_batch_free.restype = None
    L.rr_gen_sizes.argtypes = [C.c_int, u64, u64, u64, vp, vp, C.c_int]
    L.rr_gen_range.argtypes = [C.c_int, u64, u64, u64, C.POINTER(HostBatch), C.c_int]
    L.rr_gen_default_seed.argtypes = [C.c_int]
    L.rr_gen_default_seed.restype = u64
    L.rr_shard_plan.argtypes = [vp, u64, C.c_uint32, C.POINTER(Shard)]
    L.rr_flat_rebase.argtypes = [vp, vp, u64, vp, u64, u64, u64, vp]
    L.rr_flat_rebase_host.argtypes = [vp, u64, vp, u64, u64, u64]
    L.rr_gather_layout.argtypes = [vp, C.c_int, vp]
    if hasattr(L, "rr_split_schedule"):   # (RR_LIB: an older build for A/B timing may predate them)
        L.rr_split_schedule.argtypes = [C.POINTER(Shard), C.c_int, C.c_int, C.c_int, C.POINTER(Xfer)]
        L.rr_gather_schedule.argtypes = [C.POINTER(Shard), vp, C.c_int, C.c_int, C.c_int, C.POINTER(Xfer)]
    L.rr_gather_layout.restype = u64
    L.rr_copy_device.argtypes = [vp, vp, vp, u64, vp]
    L.rr_comm_get_id.argtypes = [vp]
    L.rr_comm_init.argtypes = [vp, C.c_int, C.c_int, vp, C.POINTER(vp)]
    L.rr_comm_destroy.argtypes = [vp]
    L.rr_comm_destroy.restype = None
    L.rr_split_plan.argtypes = [vp, C.POINTER(BlobBatch), C.c_int, C.POINTER(Shard), vp]
    L.rr_split.argtypes = [vp, C.POINTER(BlobBatch), C.POINTER(Shard), C.c_int, C.POINTER(BlobBatch), vp]
    L.rr_gather.argtypes = [vp, C.POINTER(FlatBatch), u64, C.POINTER(Shard), C.c_int, C.POINTER(FlatBatch), vp]
    L.rr_snappy_max_compressed_length.argtypes = [u64]
    L.rr_snappy_max_compressed_length.restype = u64
    L.rr_snappy_compress_bound.argtypes = [u64, u64]
    L.rr_snappy_compress_bound.restype = u64
    L.rr_snappy_compress_batch.argtypes = [vp, C.POINTER(BlobBatch), C.POINTER(BlobBatch), vp]
    L.rr_snappy_decompress_batch.argtypes = [vp, C.POINTER(BlobBatch), C.POINTER(BlobBatch), vp, vp]
    L.rr_snappy_compress_batch_host.argtypes = [vp, vp, vp, u64, vp, u64, vp]
    L.rr_snappy_decompress_batch_host.argtypes = [vp, vp, vp, u64, vp, u64, vp, vp]
    if hasattr(L, "rr_host_decode_batch"):   # (RR_LIB: an older build for A/B timing may predate it)
        L.rr_host_reserve.argtypes = [vp, u64]
        L.rr_host_reserve.restype = u64
        L.rr_host_decode_value.argtypes = [vp, u64, u64, vp, vp, u64, C.POINTER(C.c_uint64)]
        L.rr_host_decode_batch.argtypes = [vp, vp, u64, vp, vp, u64, vp, C.POINTER(Totals)]
        L.rr_host_check_value.argtypes = [vp, u64, vp]
        L.rr_host_encode_size.argtypes = [vp, vp, u64, u64, C.POINTER(C.c_uint64)]
        L.rr_host_encode_value.argtypes = [vp, vp, vp, vp]
        L.rr_host_encode_value.restype = None
        L.rr_host_encode_batch.argtypes = [vp, vp, u64, vp, u64, u64, vp, u64, vp, C.POINTER(Totals)]
    _lib = L
    return L


def _check(rc):
    if rc != 0:
        raise RRError(f"rr call failed ({rc}): {lib().rr_last_error().decode()}")


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p) if a is not None and a.size else None


def gen_batch(config: int, n: int, seed: int | None = None):
    """Synthetic blob batch: returns (data uint8 padded to 16, offsets uint64)."""
    L = lib()
    if seed is None:
        seed = L.rr_gen_default_seed(config)
    hb = HostBatch()
    _check(L.rr_gen_batch(config, n, seed, C.byref(hb)))
    try:
        nbytes = int(hb.bytes)
        padded = (nbytes + 15) & ~15
        data = np.ctypeslib.as_array(hb.data, shape=(max(padded, 1),))[:padded].copy() if padded else \
            np.zeros(0, np.uint8)
        offs = np.ctypeslib.as_array(hb.offsets, shape=(n + 1,)).copy()
    finally:
        L.rr_host_batch_free(C.byref(hb))
    return data, offs


def gen_sizes(config: int, v0: int, v1: int, seed: int | None = None, nthreads: int = 8):
    """Config 5 (seekable): (blob bytes uint64, descriptor counts uint32) of values [v0, v1)."""
    L = lib()
    if seed is None:
        seed = L.rr_gen_default_seed(config)
    nb = np.zeros(max(v1 - v0, 1), np.uint64)
    nd = np.zeros(max(v1 - v0, 1), np.uint32)
    _check(L.rr_gen_sizes(config, v0, v1, seed, _ptr(nb), _ptr(nd), nthreads))
    return nb[:v1 - v0], nd[:v1 - v0]


def gen_range(config: int, v0: int, v1: int, seed: int | None = None, nthreads: int = 8):
    """Config 5 (seekable): (data uint8 padded to 16, offsets relative to v0) of values [v0, v1)."""
    L = lib()
    if seed is None:
        seed = L.rr_gen_default_seed(config)
    hb = HostBatch()
    _check(L.rr_gen_range(config, v0, v1, seed, C.byref(hb), nthreads))
    try:
        n, nbytes = v1 - v0, int(hb.bytes)
        padded = (nbytes + 15) & ~15
        data = np.ctypeslib.as_array(hb.data, shape=(max(padded, 1),))[:padded].copy() if padded else \
            np.zeros(0, np.uint8)
        offs = np.ctypeslib.as_array(hb.offsets, shape=(n + 1,)).copy()
    finally:
        L.rr_host_batch_free(C.byref(hb))
    return data, offs


def shard_plan(offsets: np.ndarray, g: int) -> np.ndarray:
    """The C library's byte-balanced plan (rr_shard_plan): (g, 4) uint64 rows v0, v1, b0, b1."""
    offsets = np.ascontiguousarray(offsets, np.uint64)
    plan = (Shard * g)()
    _check(lib().rr_shard_plan(_ptr(offsets), len(offsets) - 1, g, plan))
    return np.array([[p.v0, p.v1, p.b0, p.b1] for p in plan], np.uint64).reshape(g, 4)


def flat_rebase_host(values: np.ndarray, elems: np.ndarray, elem_add: int, byte_add: int):
    """In place on host records (rr_flat_rebase_host): the placement rr_gather makes on the device."""
    assert values.dtype == VALUE_DT and elems.dtype == ELEM_DT and values.flags.c_contiguous and elems.flags.c_contiguous
    _check(lib().rr_flat_rebase_host(_ptr(values), len(values), _ptr(elems), len(elems), elem_add, byte_add))


def gather_layout(shard_elems) -> tuple[np.ndarray, int]:
    """(elem_at per shard, total) of the C library's gather placement (rr_gather_layout)."""
    ne = np.ascontiguousarray(shard_elems, np.uint64)
    at = np.zeros(max(len(ne), 1), np.uint64)
    tot = int(lib().rr_gather_layout(_ptr(ne), len(ne), _ptr(at)))
    if tot == 2 ** 64 - 1:
        raise RRError("gather layout past 2^32 - 1 descriptors")
    return at[:len(ne)], tot


def _plan_arg(plan):
    plan = np.ascontiguousarray(plan, np.uint64).reshape(-1, 4)
    arr = (Shard * len(plan))()
    for k, (v0, v1, b0, b1) in enumerate(plan):
        arr[k] = Shard(int(v0), int(v1), int(b0), int(b1))
    return arr, len(plan)


def _xfers(out, m):
    if m < 0:
        raise RRError("bad schedule arguments")
    return [(int(x.peer), int(x.dir), int(x.buf), int(x.offset), int(x.bytes)) for x in out[:m]]


def split_schedule(plan, rank: int, root: int = 0):
    """The transfers rr_split posts on `rank` (rr_split_schedule): [(peer, dir, buf, offset, bytes)]."""
    arr, g = _plan_arg(plan)
    out = (Xfer * (2 * g))()
    return _xfers(out, lib().rr_split_schedule(arr, g, rank, root, out))


def gather_schedule(plan, shard_elems, rank: int, root: int = 0):
    """The transfers rr_gather posts on `rank` (rr_gather_schedule)."""
    arr, g = _plan_arg(plan)
    ne = np.ascontiguousarray(shard_elems, np.uint64)
    out = (Xfer * (2 * g))()
    return _xfers(out, lib().rr_gather_schedule(arr, _ptr(ne), g, rank, root, out))


# ---- the host codec (include/rr_host.h) ------------------------------------------------------
# The CPU routing target of the compat shim for RedRock's per-key calls: explicit functions, never
# reached from Engine (the GPU entry points have no CPU fallback).
def host_decode(data: np.ndarray, offsets: np.ndarray, elem_cap: int | None = None):
    """rr_host_decode_batch: (values, elems, arena, totals) with rr_decode_batch_host's contract."""
    n = len(offsets) - 1
    nbytes = int(offsets[-1])
    if elem_cap is None:
        elem_cap = elem_bound(n, nbytes)
    data = np.ascontiguousarray(data, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    values = np.zeros(n, VALUE_DT)
    elems = np.zeros(max(elem_cap, 1), ELEM_DT)
    arena = np.zeros(max(nbytes, 1), np.uint8)
    t = Totals()
    _check(lib().rr_host_decode_batch(_ptr(data), _ptr(offsets), n, _ptr(values), _ptr(elems), elem_cap,
                                      _ptr(arena), C.byref(t)))
    ne = min(int(t.n_elems), elem_cap)
    return values, elems[:ne], arena[:nbytes], t.as_dict()


def host_decode_value(blob: bytes, base: int = 0, cap: int = 64):
    """rr_host_decode_value: (status, record, descriptors, need) of one blob."""
    b = np.frombuffer(bytes(blob) or b"\0", np.uint8)
    v = np.zeros(1, VALUE_DT)
    e = np.zeros(max(cap, 1), ELEM_DT)
    need = C.c_uint64()
    st = lib().rr_host_decode_value(_ptr(b), len(blob), base, _ptr(v), _ptr(e), cap, C.byref(need))
    return int(st), v[0], e[:min(int(v[0]["n_elems"]), cap)], int(need.value)


def host_check(data: np.ndarray, offsets: np.ndarray) -> np.ndarray:
    """rr_host_check_value per blob: the records (elem_base 0) rr_host_decode_value gives."""
    data = np.ascontiguousarray(data, np.uint8)
    n = len(offsets) - 1
    out = np.zeros(n, VALUE_DT)
    L = lib()
    base = data.ctypes.data
    for i in range(n):
        o, ln = int(offsets[i]), int(offsets[i + 1] - offsets[i])
        L.rr_host_check_value(C.c_void_p(base + o), ln, C.c_void_p(out.ctypes.data + 16 * i))
    return out


def host_encode(values: np.ndarray, elems: np.ndarray, arena: np.ndarray, data_cap: int | None = None):
    """rr_host_encode_batch: (data, offsets, totals) with rr_encode_batch_host's contract."""
    n = len(values)
    values = np.ascontiguousarray(values, VALUE_DT)
    elems = np.ascontiguousarray(elems, ELEM_DT)
    arena = np.ascontiguousarray(arena, np.uint8)
    if data_cap is None:
        data_cap = encode_bound(values, elems)
    data = np.zeros(max(data_cap, 1), np.uint8)
    offsets = np.zeros(n + 1, np.uint64)
    t = Totals()
    _check(lib().rr_host_encode_batch(_ptr(values), _ptr(elems), len(elems), _ptr(arena), arena.size, n, _ptr(data),
                                      data_cap, _ptr(offsets), C.byref(t)))
    return data[:int(offsets[-1])], offsets, t.as_dict()


def elem_bound(n: int, nbytes: int) -> int:
    return int(lib().rr_decode_elem_bound(n, nbytes))


class Engine:
    """One engine context (one per host thread) on a HIP device."""

    def __init__(self, device: int = 0):
        self._L = lib()
        self._ctx = C.c_void_p()
        _check(self._L.rr_ctx_create(device, C.byref(self._ctx)))

    def close(self):
        if self._ctx:
            self._L.rr_ctx_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_options(self, flags: int):
        """RR_CTX_* flags (CTX_NO_SMALL: every call takes the batch pipeline)."""
        _check(self._L.rr_ctx_set_options(self._ctx, flags))

    def debug_fail_second(self):
        """Test hook: the next pipeline call launches only its first kernel and fails."""
        _check(self._L.rr_debug_fail_second(self._ctx))

    def debug_one_help(self):
        """Test hook: the next one-launch decode sums every earlier window itself (the look-back's
        help for windows whose workgroups have not started)."""
        _check(self._L.rr_debug_one_help(self._ctx))

    def reserve(self, n: int, nbytes: int = 0):
        _check(self._L.rr_ctx_reserve(self._ctx, n, nbytes))

    # ---- host entry points ------------------------------------------------------------
    def decode_host(self, data: np.ndarray, offsets: np.ndarray, elem_cap: int | None = None):
        n = len(offsets) - 1
        nbytes = int(offsets[-1])
        if elem_cap is None:
            elem_cap = elem_bound(n, nbytes)
        data = np.ascontiguousarray(data, np.uint8)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        values = np.zeros(n, VALUE_DT)
        elems = np.zeros(max(elem_cap, 1), ELEM_DT)
        arena = np.zeros(max(nbytes, 1), np.uint8)
        t = Totals()
        _check(self._L.rr_decode_batch_host(self._ctx, _ptr(data), _ptr(offsets), n, _ptr(values), _ptr(elems),
                                            elem_cap, _ptr(arena), C.byref(t)))
        ne = min(int(t.n_elems), elem_cap)
        return values, elems[:ne], arena[:nbytes], t.as_dict()

    def encode_host(self, values: np.ndarray, elems: np.ndarray, arena: np.ndarray, data_cap: int | None = None):
        n = len(values)
        values = np.ascontiguousarray(values, VALUE_DT)
        elems = np.ascontiguousarray(elems, ELEM_DT)
        arena = np.ascontiguousarray(arena, np.uint8)
        if data_cap is None:
            data_cap = encode_bound(values, elems)
        data = np.zeros(max(data_cap, 1), np.uint8)
        offsets = np.zeros(n + 1, np.uint64)
        t = Totals()
        _check(self._L.rr_encode_batch_host(self._ctx, _ptr(values), _ptr(elems), len(elems), _ptr(arena),
                                            arena.size, n, _ptr(data), data_cap, _ptr(offsets), C.byref(t)))
        return data[:int(offsets[-1])], offsets, t.as_dict()

    # ---- device entry points (torch tensors on the engine's device) ----------------------
    def decode_device(self, data, offsets, values, elems, arena, totals, stream=None):
        """All arguments are torch CUDA tensors; no host sync.  stream: torch stream or None."""
        n = offsets.numel() - 1
        inb = BlobBatch(data.data_ptr(), offsets.data_ptr(), n, data.numel())
        outb = FlatBatch(values.data_ptr(), elems.data_ptr(), arena.data_ptr(), n, elems.numel() // 16,
                         arena.numel())
        s = stream.cuda_stream if stream is not None else None
        _check(self._L.rr_decode_batch(self._ctx, C.byref(inb), C.byref(outb), C.c_void_p(totals.data_ptr()),
                                       C.c_void_p(s) if s else None))

    def flat_rebase(self, values, elems, elem_add: int, byte_add: int, stream=None):
        """In place on torch CUDA tensors (uint8 views of the flat records): rr_flat_rebase."""
        _check(self._L.rr_flat_rebase(self._ctx, C.c_void_p(values.data_ptr()), values.numel() // 16,
                                      C.c_void_p(elems.data_ptr()), elems.numel() // 16, elem_add, byte_add,
                                      _sp(stream)))

    def copy_device(self, dst, src, nbytes: int | None = None, stream=None):
        """The engine's streaming copy (rr_copy_device) between torch CUDA tensors."""
        nb = src.numel() * src.element_size() if nbytes is None else nbytes
        _check(self._L.rr_copy_device(self._ctx, C.c_void_p(dst.data_ptr()), C.c_void_p(src.data_ptr()), nb,
                                      _sp(stream)))

    # ---- snappy block compression (include/rr_snappy.h) -----------------------------------
    def snappy_compress_host(self, data: np.ndarray, offsets: np.ndarray):
        """Blocks [offsets[i], offsets[i+1]) of data -> (packed compressed bytes, offsets)."""
        data = np.ascontiguousarray(data, np.uint8)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        n = len(offsets) - 1
        cap = int(self._L.rr_snappy_compress_bound(n, int(offsets[-1])))
        out = np.zeros(max(cap, 1), np.uint8)
        oo = np.zeros(n + 1, np.uint64)
        _check(self._L.rr_snappy_compress_batch_host(self._ctx, _ptr(data), _ptr(offsets), n, _ptr(out), cap, _ptr(oo)))
        return out[:int(oo[-1])], oo

    def snappy_decompress_host(self, comp: np.ndarray, offsets: np.ndarray, out_cap: int):
        """(out bytes, out offsets, per-block status) of snappy blocks."""
        comp = np.ascontiguousarray(comp, np.uint8)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        n = len(offsets) - 1
        out = np.zeros(max(out_cap, 1), np.uint8)
        oo = np.zeros(n + 1, np.uint64)
        st = np.zeros(max(n, 1), np.uint8)
        _check(self._L.rr_snappy_decompress_batch_host(self._ctx, _ptr(comp), _ptr(offsets), n, _ptr(out), out_cap,
                                                       _ptr(oo), _ptr(st)))
        return out[:int(oo[-1])], oo, st[:n]

    def snappy_compress_device(self, data, offsets, out, out_offsets, stream=None):
        n = offsets.numel() - 1
        inb = BlobBatch(data.data_ptr(), offsets.data_ptr(), n, data.numel())
        outb = BlobBatch(out.data_ptr(), out_offsets.data_ptr(), n, out.numel())
        _check(self._L.rr_snappy_compress_batch(self._ctx, C.byref(inb), C.byref(outb), _sp(stream)))

    def snappy_decompress_device(self, comp, offsets, out, out_offsets, status, stream=None):
        n = offsets.numel() - 1
        inb = BlobBatch(comp.data_ptr(), offsets.data_ptr(), n, comp.numel())
        outb = BlobBatch(out.data_ptr(), out_offsets.data_ptr(), n, out.numel())
        _check(self._L.rr_snappy_decompress_batch(self._ctx, C.byref(inb), C.byref(outb),
                                                  C.c_void_p(status.data_ptr()), _sp(stream)))

    def encode_device(self, values, elems, arena, out_data, out_offsets, totals, stream=None):
        n = out_offsets.numel() - 1
        inb = FlatBatch(values.data_ptr(), elems.data_ptr(), arena.data_ptr(), n, elems.numel() // 16,
                        arena.numel())
        outb = BlobBatch(out_data.data_ptr(), out_offsets.data_ptr(), n, out_data.numel())
        s = stream.cuda_stream if stream is not None else None
        _check(self._L.rr_encode_batch(self._ctx, C.byref(inb), C.byref(outb), C.c_void_p(totals.data_ptr()),
                                       C.c_void_p(s) if s else None))


class Comm:
    """An RCCL communicator over one engine's device (include/rr_serdes.h multi-GPU calls).
    Every rank builds one with the same 128-byte id (``Comm.new_id()`` on one rank, handed to
    the others by any means).  Device arguments are torch CUDA tensors."""

    def __init__(self, engine: Engine, nranks: int, rank: int, cid: bytes):
        self._L = lib()
        self.nranks, self.rank = nranks, rank
        self._c = C.c_void_p()
        buf = (C.c_uint8 * COMM_ID_BYTES).from_buffer_copy(cid)
        _check(self._L.rr_comm_init(engine._ctx, nranks, rank, buf, C.byref(self._c)))

    @staticmethod
    def new_id() -> bytes:
        buf = (C.c_uint8 * COMM_ID_BYTES)()
        _check(lib().rr_comm_get_id(buf))
        return bytes(buf)

    def close(self):
        if self._c:
            self._L.rr_comm_destroy(self._c)
            self._c = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def split_plan(self, data=None, offsets=None, root=0, stream=None):
        whole = BlobBatch(data.data_ptr(), offsets.data_ptr(), offsets.numel() - 1, data.numel()) \
            if offsets is not None else BlobBatch()
        plan = (Shard * self.nranks)()
        _check(self._L.rr_split_plan(self._c, C.byref(whole), root, plan, _sp(stream)))
        return plan

    def split(self, plan, data, offsets, mine_data, mine_offsets, root=0, stream=None):
        whole = BlobBatch(data.data_ptr(), offsets.data_ptr(), offsets.numel() - 1, data.numel()) \
            if offsets is not None else BlobBatch()
        mine = BlobBatch(mine_data.data_ptr(), mine_offsets.data_ptr(), 0, mine_data.numel())
        _check(self._L.rr_split(self._c, C.byref(whole), plan, root, C.byref(mine), _sp(stream)))
        return int(mine.n)

    def gather(self, plan, values, elems, mine_elems, whole_values=None, whole_elems=None, root=0, stream=None):
        mine = FlatBatch(values.data_ptr(), elems.data_ptr(), None, values.numel() // 16, elems.numel() // 16, 0)
        whole = FlatBatch(whole_values.data_ptr(), whole_elems.data_ptr(), None, whole_values.numel() // 16,
                          whole_elems.numel() // 16, 0) if whole_values is not None else FlatBatch()
        _check(self._L.rr_gather(self._c, C.byref(mine), mine_elems, plan, root, C.byref(whole), _sp(stream)))


def _sp(stream):
    return C.c_void_p(stream.cuda_stream) if stream is not None else None


def encode_bound(values: np.ndarray, elems: np.ndarray) -> int:
    """Upper bound on encoded bytes for a flat batch (decimal ints <= 20 chars + 4-byte prefix;
    every other element costs <= 16 + len)."""
    return int(len(values) * 13 + len(elems) * 24 + int(elems["len"].astype(np.uint64).sum()) + 16)

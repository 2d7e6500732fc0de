"""ctypes binding of oracle/librr_oracle.so — TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() (as the checker) and bench.py's cpu_baseline
leg.  The engine (redrock_old_amd) never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import time

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "librr_oracle.so")

_lib = None


class _Totals(C.Structure):
    _fields_ = [("n_elems", C.c_uint64), ("bytes", C.c_uint64), ("n_bad", C.c_uint64),
                ("payload", C.c_uint64)]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} not built (make -C oracle)")
        L = C.CDLL(LIB_PATH)
        vp, u64 = C.c_void_p, C.c_uint64
        L.rro_decode.argtypes = [vp, vp, u64, vp, vp, u64, vp, C.POINTER(_Totals), C.c_int]
        L.rro_encode.argtypes = [vp, vp, u64, vp, u64, u64, vp, u64, vp, C.POINTER(_Totals), C.c_int]
        L.rro_string2ll.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_longlong)]
        L.rro_ll2str.argtypes = [C.c_char_p, C.c_longlong]
        L.rro_parse_ziplist.argtypes = [vp, u64, u64, vp, u64, C.POINTER(C.c_uint64)]
        L.rro_faithful_decode.argtypes = [vp, vp, u64, C.POINTER(C.c_uint64)]
        L.rro_faithful_decode.restype = vp
        L.rro_faithful_encode.argtypes = [vp, vp, u64, vp]
        L.rro_faithful_encode.restype = u64
        L.rro_store_free.argtypes = [vp]
        L.rro_store_free.restype = None
        L.rro_nprocs.restype = C.c_int
        L.rrs_max_compressed.argtypes = [u64]
        L.rrs_max_compressed.restype = u64
        L.rrs_compress.argtypes = [vp, u64, vp]
        L.rrs_compress.restype = u64
        L.rrs_uncompressed_length.argtypes = [vp, u64, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        L.rrs_uncompress.argtypes = [vp, u64, vp, u64, C.POINTER(C.c_uint64)]
        L.rrs_compress_batch.argtypes = [vp, vp, u64, vp, vp, vp, C.c_int]
        L.rrs_compress_batch.restype = None
        L.rrs_uncompress_batch.argtypes = [vp, vp, u64, vp, vp, vp, C.c_int]
        L.rrs_uncompress_batch.restype = None
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None and a.size else None


def _tot(t):
    return {k: int(getattr(t, k)) for k, _ in t._fields_}


def decode(data, offsets, elem_cap=None, nthreads=1):
    from redrock_old_amd import VALUE_DT, ELEM_DT
    n = len(offsets) - 1
    nbytes = int(offsets[-1])
    if elem_cap is None:
        elem_cap = n + nbytes // 2
    data = np.ascontiguousarray(data, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    values = np.zeros(n, VALUE_DT)
    elems = np.zeros(max(elem_cap, 1), ELEM_DT)
    arena = np.zeros(max(nbytes, 1), np.uint8)
    t = _Totals()
    lib().rro_decode(_p(data), _p(offsets), n, _p(values), _p(elems), elem_cap, _p(arena), C.byref(t), nthreads)
    ne = min(int(t.n_elems), elem_cap)
    return values, elems[:ne], arena[:nbytes], _tot(t)


def encode(values, elems, arena, data_cap=None, nthreads=1):
    from redrock_old_amd import encode_bound
    n = len(values)
    if data_cap is None:
        data_cap = encode_bound(values, elems)
    data = np.zeros(max(data_cap, 1), np.uint8)
    offsets = np.zeros(n + 1, np.uint64)
    t = _Totals()
    values = np.ascontiguousarray(values)
    elems = np.ascontiguousarray(elems)
    arena = np.ascontiguousarray(arena, np.uint8)
    lib().rro_encode(_p(values), _p(elems), len(elems), _p(arena), arena.size, n, _p(data), data_cap,
                     _p(offsets), C.byref(t), nthreads)
    return data[:int(offsets[-1])], offsets, _tot(t)


def string2ll(b: bytes):
    v = C.c_longlong()
    ok = lib().rro_string2ll(b, len(b), C.byref(v))
    return v.value if ok else None


def ll2str(v: int) -> bytes:
    buf = C.create_string_buffer(32)
    n = lib().rro_ll2str(buf, v)
    return buf.raw[:n]


def parse_ziplist(zl: bytes, base: int = 0):
    from redrock_old_amd import ELEM_DT
    a = np.frombuffer(zl, np.uint8).copy()
    out = np.zeros(max(len(zl), 1), ELEM_DT)
    cnt = C.c_uint64()
    st = lib().rro_parse_ziplist(_p(a), len(zl), base, _p(out), len(out), C.byref(cnt))
    return st, out[:cnt.value]


def nprocs() -> int:
    return int(lib().rro_nprocs())


def faithful_roundtrip(data, offsets):
    """Reference-faithful desObject over the batch, then serObject of every object.
    Returns (out_bytes, out_offsets, n_bad, t_decode_s, t_encode_s)."""
    L = lib()
    n = len(offsets) - 1
    data = np.ascontiguousarray(data, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    bad = C.c_uint64()
    t0 = time.perf_counter()
    st = L.rro_faithful_decode(_p(data), _p(offsets), n, C.byref(bad))
    t1 = time.perf_counter()
    out = np.zeros(int(offsets[-1]) + 16, np.uint8)
    ooff = np.zeros(n + 1, np.uint64)
    t2 = time.perf_counter()
    L.rro_faithful_encode(st, _p(out), out.size, _p(ooff))
    t3 = time.perf_counter()
    L.rro_store_free(st)
    return out[:int(ooff[-1])], ooff, int(bad.value), t1 - t0, t3 - t2


# ---- snappy raw format (oracle/rr_snappy.c) ---------------------------
def snappy_compress(data: bytes) -> bytes:
    src = np.frombuffer(bytes(data), np.uint8)
    out = np.zeros(int(lib().rrs_max_compressed(len(src))) + 8, np.uint8)
    n = lib().rrs_compress(_p(src), len(src), _p(out))
    return out[:n].tobytes()


def snappy_uncompress(comp: bytes, cap: int | None = None):
    """(status, bytes or None); cap defaults to the preamble's length."""
    src = np.frombuffer(bytes(comp), np.uint8)
    ln, hdr = C.c_uint32(), C.c_uint32()
    st = lib().rrs_uncompressed_length(_p(src), len(src), C.byref(ln), C.byref(hdr))
    if st:
        return st, None
    if cap is None:
        cap = ln.value
    out = np.zeros(max(cap, 1), np.uint8)
    got = C.c_uint64()
    st = lib().rrs_uncompress(_p(src), len(src), _p(out), cap, C.byref(got))
    return st, (out[:got.value].tobytes() if st == 0 else None)


def snappy_length(comp: bytes):
    """(status, announced uncompressed length) of a snappy stream's preamble."""
    src = np.frombuffer(bytes(comp), np.uint8)
    ln, hdr = C.c_uint32(), C.c_uint32()
    st = lib().rrs_uncompressed_length(_p(src), len(src), C.byref(ln), C.byref(hdr))
    return st, (ln.value if st == 0 else 0)


def snappy_compress_blocks(data, offs, nthreads=1):
    """Every block [offs[i], offs[i+1]) compressed: (packed bytes, offsets, seconds)."""
    L = lib()
    offs = np.ascontiguousarray(offs, np.uint64)
    n = len(offs) - 1
    bounds = np.array([L.rrs_max_compressed(int(offs[i + 1] - offs[i])) for i in range(n)], np.uint64)
    slot = np.zeros(n + 1, np.uint64)
    np.cumsum(bounds, out=slot[1:])
    out = np.zeros(int(slot[-1]) + 16, np.uint8)
    sizes = np.zeros(max(n, 1), np.uint64)
    data = np.ascontiguousarray(data, np.uint8)
    t0 = time.perf_counter()
    L.rrs_compress_batch(_p(data), _p(offs), n, _p(out), _p(slot), _p(sizes), nthreads)
    dt = time.perf_counter() - t0
    coffs = np.zeros(n + 1, np.uint64)
    np.cumsum(sizes[:n], out=coffs[1:])
    packed = np.concatenate([out[int(slot[i]):int(slot[i] + sizes[i])] for i in range(n)]) if n else np.zeros(0, np.uint8)
    return packed, coffs, dt


def snappy_uncompress_blocks(comp, coffs, out_offs, nthreads=1):
    """Blocks of comp into slots [out_offs[i], out_offs[i+1]): (out, status, seconds)."""
    L = lib()
    coffs = np.ascontiguousarray(coffs, np.uint64)
    out_offs = np.ascontiguousarray(out_offs, np.uint64)
    n = len(coffs) - 1
    out = np.zeros(int(out_offs[-1]) + 16, np.uint8)
    st = np.zeros(max(n, 1), np.uint8)
    comp = np.ascontiguousarray(comp, np.uint8)
    t0 = time.perf_counter()
    L.rrs_uncompress_batch(_p(comp), _p(coffs), n, _p(out), _p(out_offs), _p(st), nthreads)
    return out[:int(out_offs[-1])], st[:n], time.perf_counter() - t0

"""Pure-Python restatement of RedRock's value serdes format — TEST INFRASTRUCTURE ONLY.

This module is one of the two CPU oracles (the other is ``oracle/rr_oracle.c``).  It is
written independently of the C restatement and of the HIP kernels, from the source text of
the reference (read as text, never built or imported — SURVEY.md §8c denial record):

  blob header        rock_serdes.c:512-518 (write), :538-544 (read); rock.h:50-63 tags
  String             rock_serdes.c:114-158
  List               rock_serdes.c:162-214  (+ zipTryEncoding ziplist.c:480-503,
                                              string2ll util.c:360-424, sdsll2str sds.c:450-479)
  Set                rock_serdes.c:217-311  (intset.h:34-38)
  Hash               rock_serdes.c:314-414
  ZSet               rock_serdes.c:417-508
  ziplist entries    ziplist.c:55-106, :300-447, :507-566

It decodes blobs into the flat form of include/rr_format.h (values, element descriptors,
mirror arena) and encodes that form back.  Only tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py may use anything under oracle/; the product never does.

Parity pins: SURVEY.md §8c known-answer vectors K1-K9 (tests/golden), the ziplist byte
example of ziplist.c:114-149, util.c:754-897 string2ll/ll2string vectors and intset.c:361-375
encoding boundaries.
"""
from __future__ import annotations

import struct

T_STRING, T_SET_HT, T_HASH_HT, T_ZSET_SKIPLIST = 0, 2, 4, 5
T_SET_INTSET, T_ZSET_ZIPLIST, T_HASH_ZIPLIST, T_LIST_QUICKLIST = 11, 12, 13, 14
ENC_RAW, ENC_INT, ENC_EMBSTR = 0, 1, 8
K_STR, K_INT, K_SCORE, K_ZLRAW = 0, 1, 2, 3

OK, E_SHORT, E_TYPE, E_STR_ENC, E_STR_INTLEN, E_EMBSTR_LEN = 0, 1, 2, 3, 4, 5
E_TRUNC, E_COUNT, E_INTSET, E_ZL_LEN, E_ZL_CORRUPT, E_CAPACITY, E_ENCODE = 6, 7, 8, 9, 10, 11, 12
E_DUP, E_NAN = 13, 14

LLONG_MIN, LLONG_MAX = -(1 << 63), (1 << 63) - 1


class DecodeError(Exception):
    def __init__(self, code):
        super().__init__(code)
        self.code = code


def string2ll(b: bytes):
    """Strict decimal parse, util.c:360-424. Returns int or None."""
    if len(b) == 0:
        return None
    if b == b"0":
        return 0
    i, neg = 0, False
    if b[0:1] == b"-":
        neg, i = True, 1
        if i == len(b):
            return None
    if not (0x31 <= b[i] <= 0x39):
        return None
    v = b[i] - 0x30
    i += 1
    while i < len(b) and 0x30 <= b[i] <= 0x39:
        v = v * 10 + (b[i] - 0x30)
        if v > (1 << 64) - 1:
            return None
        i += 1
    if i < len(b):
        return None
    if neg:
        if v > (1 << 63):
            return None
        return -v
    if v > LLONG_MAX:
        return None
    return v


def ll2str(v: int) -> bytes:
    """sdsll2str, sds.c:450-479 (same digits as ll2string util.c:294)."""
    return str(v).encode()


def zip_try_encoding(b: bytes):
    """ziplist.c:480-503 (entrylen >= 32 or 0 -> not an integer)."""
    if len(b) >= 32 or len(b) == 0:
        return None
    return string2ll(b)


def _u32(b, p):
    return struct.unpack_from("<I", b, p)[0]


def _u64(b, p):
    return struct.unpack_from("<Q", b, p)[0]


_INT_SIZES = {0xC0: 2, 0xD0: 4, 0xE0: 8, 0xF0: 3, 0xFE: 1}


def parse_ziplist(zl: bytes, base: int = 0):
    """Walk a ziplist (ziplist.c:300-447). Returns list of element tuples
    (kind, data, len, zenc) where STR data is base+offset of the string bytes."""
    L = len(zl)
    if L < 11 or _u32(zl, 0) != L:
        raise DecodeError(E_ZL_CORRUPT)
    zltail, zllen = _u32(zl, 4), struct.unpack_from("<H", zl, 8)[0]
    p, prev_raw, last, out = 10, 0, 10, []
    while True:
        if p >= L:
            raise DecodeError(E_ZL_CORRUPT)
        if zl[p] == 0xFF:
            break
        if zl[p] < 254:
            pl, pls = zl[p], 1
        else:
            if p + 5 > L - 1:
                raise DecodeError(E_ZL_CORRUPT)
            pl, pls = _u32(zl, p + 1), 5
        if pl != prev_raw:
            raise DecodeError(E_ZL_CORRUPT)
        q = p + pls
        if q >= L - 1:
            raise DecodeError(E_ZL_CORRUPT)
        enc = zl[q]
        if enc < 0xC0:
            cls = enc & 0xC0
            if cls == 0x00:
                ls, sl = 1, enc & 0x3F
            elif cls == 0x40:
                if q + 2 > L - 1:
                    raise DecodeError(E_ZL_CORRUPT)
                ls, sl = 2, ((enc & 0x3F) << 8) | zl[q + 1]
            else:
                if q + 5 > L - 1:
                    raise DecodeError(E_ZL_CORRUPT)
                ls, sl = 5, struct.unpack_from(">I", zl, q + 1)[0]
            d = q + ls
            end = d + sl
            if end > L - 1:
                raise DecodeError(E_ZL_CORRUPT)
            out.append((K_STR, base + d, sl, cls))
        else:
            if enc in _INT_SIZES:
                isz = _INT_SIZES[enc]
            elif 0xF1 <= enc <= 0xFD:
                isz = 0
            else:
                raise DecodeError(E_ZL_CORRUPT)
            d = q + 1
            end = d + isz
            if end > L - 1:
                raise DecodeError(E_ZL_CORRUPT)
            if isz == 0:
                v = (enc & 0x0F) - 1
            elif isz == 3:
                v = int.from_bytes(zl[d:d + 3], "little", signed=True)
            else:
                v = int.from_bytes(zl[d:d + isz], "little", signed=True)
            out.append((K_INT, v, 0, enc))
        prev_raw = end - p
        last = p
        p = end
    if p != L - 1:
        raise DecodeError(E_ZL_CORRUPT)
    if zllen != 0xFFFF and zllen != len(out):
        raise DecodeError(E_ZL_CORRUPT)
    if zltail != last:
        raise DecodeError(E_ZL_CORRUPT)
    return out


def decode_one(blob: bytes, off: int = 0):
    """Decode one blob located at batch offset `off`.
    Returns (value_dict, elems) where value_dict has type/enc/status/lru/n_elems and elems is a
    list of (kind, data, len, zenc)."""
    val = {"type": blob[0] if len(blob) else 0, "enc": 0, "status": OK,
           "lru": (_u32(blob, 1) & 0xFFFFFF) if len(blob) >= 5 else 0}
    try:
        elems = _decode_body(blob, off, val)
    except DecodeError as e:
        val["status"] = e.code
        elems = []
    val["n_elems"] = len(elems)
    val.setdefault("n_slots", len(elems))
    if val["status"] != OK:
        val["n_slots"] = 0
    return val, elems


def _decode_body(b, off, val):
    n = len(b)
    if n < 5:
        raise DecodeError(E_SHORT)
    t = b[0]
    p, rem, out = 5, n - 5, []
    if t == T_STRING:
        if n < 6:
            raise DecodeError(E_SHORT)
        enc = b[5]
        val["enc"] = enc
        rest = n - 6
        if enc == ENC_INT:
            if rest != 8:
                raise DecodeError(E_STR_INTLEN)
            out.append((K_INT, struct.unpack_from("<q", b, 6)[0], 0, 0))
        elif enc == ENC_RAW or enc == ENC_EMBSTR:
            if enc == ENC_EMBSTR and rest > 44:
                raise DecodeError(E_EMBSTR_LEN)
            out.append((K_STR, off + 6, rest, 0))
        else:
            raise DecodeError(E_STR_ENC)
    elif t == T_LIST_QUICKLIST:
        while rem:
            if rem < 4:
                raise DecodeError(E_TRUNC)
            ln = _u32(b, p)
            p += 4
            rem -= 4
            if ln > rem:
                raise DecodeError(E_TRUNC)
            v = zip_try_encoding(b[p:p + ln])
            if v is None:
                out.append((K_STR, off + p, ln, 0))
            else:
                out.append((K_INT, v, 0, 0))
            p += ln
            rem -= ln
    elif t == T_SET_INTSET:
        if rem < 8:
            raise DecodeError(E_SHORT)
        w, cnt = _u32(b, p), _u32(b, p + 4)
        p += 8
        rem -= 8
        if w not in (2, 4, 8) or rem != w * cnt:
            raise DecodeError(E_INTSET)
        val["enc"] = w
        for i in range(cnt):
            out.append((K_INT, int.from_bytes(b[p + i * w:p + (i + 1) * w], "little", signed=True), 0, 0))
    elif t in (T_SET_HT, T_HASH_HT):
        if rem < 8:
            raise DecodeError(E_SHORT)
        cnt = _u64(b, p)
        p += 8
        rem -= 8
        per = 1 if t == T_SET_HT else 2
        got = 0
        members = []   # (batch offset, length) in blob order
        while rem:
            for _ in range(per):
                if rem < 8:
                    raise DecodeError(E_TRUNC)
                ln = _u64(b, p)
                p += 8
                rem -= 8
                if ln > rem:
                    raise DecodeError(E_TRUNC)
                members.append((off + p, ln, bytes(b[p:p + ln])))
                p += ln
                rem -= ln
            got += 1
        if got != cnt:
            raise DecodeError(E_COUNT)
        val["n_slots"] = len(members)
        seen = set()
        for i, (o, ln, key) in enumerate(members):
            if per == 2 and i % 2:            # hash values are not keys
                out.append((K_STR, o, ln, 0))
                continue
            if key in seen:                   # dictAdd != DICT_OK
                if per == 2:
                    raise DecodeError(E_DUP)  # rock_serdes.c:399-400 serverAssert
                continue                      # desSet ignores it (rock_serdes.c:297)
            seen.add(key)
            out.append((K_STR, o, ln, 0))
    elif t in (T_HASH_ZIPLIST, T_ZSET_ZIPLIST):
        if rem < 8:
            raise DecodeError(E_SHORT)
        L = _u64(b, p)
        p += 8
        rem -= 8
        if rem != L:
            raise DecodeError(E_ZL_LEN)
        ents = parse_ziplist(b[p:p + L], off + p)
        if len(ents) % 2:
            raise DecodeError(E_ZL_CORRUPT)
        out.append((K_ZLRAW, off + p, L, 0))
        out.extend(ents)
    elif t == T_ZSET_SKIPLIST:
        if rem < 8:
            raise DecodeError(E_SHORT)
        cnt = _u64(b, p)
        p += 8
        rem -= 8
        pairs = []
        for _ in range(cnt):
            if rem < 8:
                raise DecodeError(E_TRUNC)
            ln = _u64(b, p)
            p += 8
            rem -= 8
            if ln > rem:
                raise DecodeError(E_TRUNC)
            mo, ele = off + p, bytes(b[p:p + ln])
            p += ln
            rem -= ln
            if rem < 8:
                raise DecodeError(E_TRUNC)
            bits = _u64(b, p)
            pairs.append((struct.unpack_from("<d", b, p)[0], ele, mo, ln, bits))
            p += 8
            rem -= 8
        if rem != 0:
            raise DecodeError(E_COUNT)
        if any(x[0] != x[0] for x in pairs):  # zslInsert serverAssert(!isnan(score)) t_zset.c:137
            raise DecodeError(E_NAN)
        # desZset rebuilds a skiplist ascending by (score, member) and serZset writes it tail to
        # head: descending, equal keys kept in blob order (Python's sort is stable, also with
        # reverse=True; -0.0 == 0.0 as in zslInsert's double compares)
        pairs.sort(key=lambda x: (x[0], x[1]), reverse=True)
        for sc, ele, mo, ln, bits in pairs:
            out.append((K_STR, mo, ln, 0))
            out.append((K_SCORE, bits, 0, 0))
    else:
        raise DecodeError(E_TYPE)
    return out


def encode_one(val: dict, elems, arena: bytes) -> bytes:
    """Inverse of decode_one: flat value -> blob (serObject, rock_serdes.c:512-535)."""
    t = val["type"]
    out = bytearray([t]) + struct.pack("<I", val["lru"] & 0xFFFFFF)

    def s(e):
        assert e[0] == K_STR
        return bytes(arena[e[1]:e[1] + e[2]])

    if t == T_STRING:
        out.append(val["enc"])
        e = elems[0]
        if val["enc"] == ENC_INT:
            out += struct.pack("<q", e[1])
        else:
            out += s(e)
    elif t == T_LIST_QUICKLIST:
        for e in elems:
            x = ll2str(e[1]) if e[0] == K_INT else s(e)
            out += struct.pack("<I", len(x)) + x
    elif t == T_SET_INTSET:
        w = val["enc"]
        out += struct.pack("<II", w, len(elems))
        for e in elems:
            out += int(e[1]).to_bytes(w, "little", signed=True)
    elif t in (T_SET_HT,):
        out += struct.pack("<Q", len(elems))
        for e in elems:
            out += struct.pack("<Q", e[2]) + s(e)
    elif t == T_HASH_HT:
        out += struct.pack("<Q", len(elems) // 2)
        for e in elems:
            out += struct.pack("<Q", e[2]) + s(e)
    elif t in (T_HASH_ZIPLIST, T_ZSET_ZIPLIST):
        e = elems[0]
        assert e[0] == K_ZLRAW
        out += struct.pack("<Q", e[2]) + bytes(arena[e[1]:e[1] + e[2]])
    elif t == T_ZSET_SKIPLIST:
        out += struct.pack("<Q", len(elems) // 2)
        for i in range(0, len(elems), 2):
            m, sc = elems[i], elems[i + 1]
            out += struct.pack("<Q", m[2]) + s(m) + struct.pack("<Q", sc[1])
    else:
        raise ValueError("type")
    return bytes(out)


def reserve(b: bytes) -> int:
    """Descriptor slots a value owns in the flat batch, from its header alone (plus the length
    chain of a List, which has no count field).  For every valid blob this equals the number of
    descriptors decode emits; a malformed value keeps its slots, zero-filled.  It lets the GPU
    size every value's output before parsing it (include/rr_format.h, "descriptor slots")."""
    L = len(b)
    if L < 5:
        return 0
    t = b[0]
    if t == T_STRING:
        return 1 if L >= 6 else 0
    if t == T_LIST_QUICKLIST:
        p, n = 5, 0
        while p < L:
            if L - p < 4:
                break
            ln = _u32(b, p)
            if ln > L - p - 4:
                break
            n += 1
            p += 4 + ln
        return n
    if L < 13:
        return 0
    if t == T_SET_INTSET:
        w, c = _u32(b, 5), _u32(b, 9)
        return c if (w in (2, 4, 8) and L - 13 == w * c) else 0
    if t == T_SET_HT:
        return min(_u64(b, 5), (L - 13) // 8)
    if t == T_HASH_HT:
        return min(2 * _u64(b, 5), (L - 13) // 8)
    if t == T_ZSET_SKIPLIST:
        return 2 * min(_u64(b, 5), (L - 13) // 16)
    if t in (T_HASH_ZIPLIST, T_ZSET_ZIPLIST):
        Lz = _u64(b, 5)
        if Lz != L - 13 or Lz < 11:
            return 0
        zllen = struct.unpack_from("<H", b, 13 + 8)[0]
        if zllen != 0xFFFF:
            return 1 + min(zllen, (Lz - 11) // 2)
        return 1 + _zl_walk_count(b[13:])
    return 0


def _zl_walk_count(zl: bytes) -> int:
    """Entries of a ziplist whose zllen saturated at 0xFFFF: walk until the end byte or the
    first entry that does not parse (ziplist.c:300-447)."""
    L, p, n = len(zl), 10, 0
    while p < L - 1 and zl[p] != 0xFF:
        pls = 1 if zl[p] < 254 else 5
        q = p + pls
        if q >= L - 1:
            break
        enc = zl[q]
        if enc < 0xC0:
            cls = enc & 0xC0
            if cls == 0x00:
                e = q + 1 + (enc & 0x3F)
            elif cls == 0x40:
                if q + 2 > L - 1:
                    break
                e = q + 2 + (((enc & 0x3F) << 8) | zl[q + 1])
            else:
                if q + 5 > L - 1:
                    break
                e = q + 5 + struct.unpack_from(">I", zl, q + 1)[0]
        elif enc in _INT_SIZES:
            e = q + 1 + _INT_SIZES[enc]
        elif 0xF1 <= enc <= 0xFD:
            e = q + 1
        else:
            break
        if e > L - 1:
            break
        n += 1
        p = e
    return n


def decode_batch(blobs):
    """Decode a list of blobs as one batch: returns (data, offsets, values, elems, arena).
    Value i owns descriptor slots [elem_base, elem_base + reserve(blob i)); a malformed value
    leaves its slots as zero descriptors (K_STR, 0, 0, 0)."""
    offsets = [0]
    for b in blobs:
        offsets.append(offsets[-1] + len(b))
    data = b"".join(blobs)
    values, elems = [], []
    for i, b in enumerate(blobs):
        v, es = decode_one(b, offsets[i])
        r = reserve(b)
        if v["status"] == OK and v["n_slots"] != r:
            v["status"], v["n_elems"], es = E_COUNT, 0, []
        v["elem_base"] = len(elems)
        values.append(v)
        # a malformed value keeps its slots zero-filled; a de-duplicated set zero-fills its tail
        elems.extend(es if v["status"] == OK else [])
        elems.extend([(K_STR, 0, 0, 0)] * (r - (len(es) if v["status"] == OK else 0)))
    return data, offsets, values, elems, data  # mirror arena == blob bytes


# ---- ziplist / intset builders used by the golden-fixture script ------------------------

def zl_entry(prev_raw: int, item, big_prevlen: bool = False) -> bytes:
    """One ziplist entry for a tail push (__ziplistInsert, ziplist.c:743-839)."""
    if prev_raw < 254 and not big_prevlen:
        pre = bytes([prev_raw])
    else:
        pre = b"\xfe" + struct.pack("<I", prev_raw)
    if isinstance(item, int):
        v = item
        enc_v = v
    else:
        enc_v = zip_try_encoding(item)
    if enc_v is not None:
        v = enc_v
        if 0 <= v <= 12:
            return pre + bytes([0xF1 + v])
        for lo, hi, enc, sz in ((-128, 127, 0xFE, 1), (-32768, 32767, 0xC0, 2),
                                (-(1 << 23), (1 << 23) - 1, 0xF0, 3),
                                (-(1 << 31), (1 << 31) - 1, 0xD0, 4)):
            if lo <= v <= hi:
                return pre + bytes([enc]) + v.to_bytes(sz, "little", signed=True)
        return pre + b"\xe0" + v.to_bytes(8, "little", signed=True)
    s = item
    n = len(s)
    if n <= 0x3F:
        hdr = bytes([n])
    elif n <= 0x3FFF:
        hdr = bytes([0x40 | (n >> 8), n & 0xFF])
    else:
        hdr = b"\x80" + struct.pack(">I", n)
    return pre + hdr + s


def build_ziplist(items, big_prevlen_at=()) -> bytes:
    body, prev, last = b"", 0, 10
    for i, it in enumerate(items):
        e = zl_entry(prev, it, i in big_prevlen_at)
        last = 10 + len(body)
        body += e
        prev = len(e)
    L = 10 + len(body) + 1
    n = len(items) if len(items) < 0xFFFF else 0xFFFF
    return struct.pack("<IIH", L, last, n) + body + b"\xff"

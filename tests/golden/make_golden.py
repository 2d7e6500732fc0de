"""Generates tests/golden/kat.json — committed golden vectors for the serdes path.

No expected value in this file is computed by an oracle's decoder:

  * KAT  — known-answer vectors hand-derived from the reference's source text (SURVEY.md §8c
           table K1-K9): blob bytes and flat form are both literals.
  * EDGE — edge and malformed cases (SURVEY.md §8c list, plus the reference's abort sites and
           the reconstruction rules of desSet / desZset).  Each blob is written by the small
           RECORDING writers below, which note where they place every member (byte offset in
           the blob, length, ziplist encoding byte) — the writer's record, not a parse of the
           bytes.  Every decision the reference makes is a hand-written literal next to the
           input, with the reference line it follows:
             - integer-or-string of each List element (zipTryEncoding / string2ll),
             - the ziplist encoding byte of each integer entry (zipTryEncoding widths),
             - which members of a set survive desSet's dictAdd (first occurrence kept),
             - the order serZset writes a skiplist desZset rebuilt (zslInsert),
             - the status code (the serverAssert / serverPanic site, or a documented
               [stricter] deviation — DESIGN.md "Deviations"),
             - the descriptor slots the value owns (rr_format.h reservation rule).

The script finally CHECKS (it does not produce) that the Python restatement oracle/pyoracle
agrees with every literal, and refuses to write the file otherwise.  The reference itself is
never built or run (SURVEY.md §8c denial).   Run:  python tests/golden/make_golden.py
"""
import json
import math
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kat.json")

K_STR, K_INT, K_SCORE, K_ZLRAW = 0, 1, 2, 3
M24, M64 = 0xFFFFFF, (1 << 64) - 1
# status codes (include/rr_format.h)
OK, SHORT, TYPE, STR_ENC, STR_INTLEN, EMBSTR_LEN, TRUNC, COUNT, INTSET, ZL_LEN, ZL_CORRUPT = range(11)
DUP, NAN = 13, 14


def h(s):
    return bytes.fromhex(s.replace(" ", ""))


K3_LITERAL = b"aadfcrghsdgggggggggggadbAFWEdsar4dadsrd423FASFASXASDFASR3ADFASDFASFASR34RFADSFSADFSAFXEEdsdec"[:60]

# Hand-derived KATs.  elems: [kind, data, len, zenc]; STR data = byte offset in blob.
KATS = [
    dict(name="K1_string_int_134123", cite="rock_serdes.c:832 (createStringObjectFromLongLongForValue)",
         blob="00 00000000 01 EB0B020000000000",
         value=dict(type=0, enc=1, lru=0), elems=[[K_INT, 134123, 0, 0]]),
    dict(name="K2_string_embstr_abc", cite="rock_serdes.c:847", blob="00 00000000 08 616263",
         value=dict(type=0, enc=8, lru=0), elems=[[K_STR, 6, 3, 0]]),
    dict(name="K3_string_raw_60", cite="rock_serdes.c:864", blob="00 00000000 00 " + K3_LITERAL.hex(),
         value=dict(type=0, enc=0, lru=0), elems=[[K_STR, 6, 60, 0]]),
    dict(name="K4_list_xxx_-1234567", cite="rock_serdes.c:815-819 (ZIP_INT_24B re-rendered by sdsll2str)",
         blob="0E 00000000 03000000 787878 08000000 2D31323334353637",
         value=dict(type=14, enc=0, lru=0), elems=[[K_STR, 9, 3, 0], [K_INT, -1234567 & M64, 0, 0]]),
    dict(name="K5_zset_ziplist_2_5", cite="ziplist.c:114-149 worked example, rock_serdes.c:420-423",
         blob="0C 00000000 0F00000000000000 0F000000 0C000000 0200 00F3 02F6 FF",
         value=dict(type=12, enc=0, lru=0),
         elems=[[K_ZLRAW, 13, 15, 0], [K_INT, 2, 0, 0xF3], [K_INT, 5, 0, 0xF6]]),
    dict(name="K6_set_intset_123", cite="intset.c:45-52 (INT16), rock_serdes.c:220-226",
         blob="0B 00000000 02000000 03000000 010002000300",
         value=dict(type=11, enc=2, lru=0),
         elems=[[K_INT, 1, 0, 0], [K_INT, 2, 0, 0], [K_INT, 3, 0, 0]]),
    dict(name="K7_hash_ht_f_v", cite="rock_serdes.c:322-339",
         blob="04 00000000 0100000000000000 0100000000000000 66 0100000000000000 76",
         value=dict(type=4, enc=0, lru=0), elems=[[K_STR, 21, 1, 0], [K_STR, 30, 1, 0]]),
    dict(name="K8_zset_skiplist_a1_b2", cite="rock_serdes.c:425-440 (tail->head = descending)",
         blob="05 00000000 0200000000000000 0100000000000000 62 0000000000000040 "
              "0100000000000000 61 000000000000F03F",
         value=dict(type=5, enc=0, lru=0),
         elems=[[K_STR, 21, 1, 0], [K_SCORE, 0x4000000000000000, 0, 0],
                [K_STR, 38, 1, 0], [K_SCORE, 0x3FF0000000000000, 0, 0]]),
    dict(name="K9_set_ht_x", cite="rock_serdes.c:227-239",
         blob="02 00000000 0100000000000000 0100000000000000 78",
         value=dict(type=2, enc=0, lru=0), elems=[[K_STR, 21, 1, 0]]),
]

# string2ll / ll2string vectors of the reference's own self-test (util.c:754-897)
STRING2LL = [["+1", None], [" 1", None], ["1 ", None], ["01", None], ["-1", -1], ["0", 0], ["1", 1],
             ["99", 99], ["-99", -99], ["-9223372036854775808", -(1 << 63)],
             ["-9223372036854775809", None], ["9223372036854775807", (1 << 63) - 1],
             ["9223372036854775808", None]]
LL2STRING = [[0, "0"], [-1, "-1"], [99, "99"], [-99, "-99"], [-2147483648, "-2147483648"],
             [-(1 << 63), "-9223372036854775808"], [(1 << 63) - 1, "9223372036854775807"]]
# ziplist.c:114-149: "2","5" then "Hello World" appended ([02][0b][48 65 6c 6c 6f 20 57 6f 72 6c 64])
ZIPLIST_EXAMPLE = {
    "two_five": "0f000000 0c000000 0200 00f3 02f6 ff",
    "hello_world_entry": "02 0b 48656c6c6f20576f726c64",
}
# intset.c:361-375 _intsetValueEncoding boundaries
INTSET_ENC = [[-32768, 2], [32767, 2], [-32769, 4], [32768, 4], [-2147483648, 4], [2147483647, 4],
              [-2147483649, 8], [2147483648, 8], [-(1 << 63), 8], [(1 << 63) - 1, 8]]


# ---------------------------------------------------------------- recording writers
def hdr(t, lru=0):
    return bytes([t]) + struct.pack("<I", lru)


def fx(name, cite, blob, t, enc, lru, status, reserve, elems):
    return dict(name=name, cite=cite, blob=blob.hex(),
                value=dict(type=t, enc=enc, lru=lru & M24, status=status,
                           n_elems=len(elems) if status == OK else 0, reserve=reserve),
                elems=elems if status == OK else [])


def w_string(name, cite, enc, payload, lru=0, status=OK):
    """STRING blob; payload bytes start at offset 6."""
    blob = hdr(0, lru) + bytes([enc]) + payload
    if enc == 1 and status == OK:
        el = [[K_INT, struct.unpack("<q", payload)[0] & M64, 0, 0]]
    else:
        el = [[K_STR, 6, len(payload), 0]]
    return fx(name, cite, blob, 0, enc, lru, status, 1, el)


def w_list(name, cite, items, lru=0):
    """items: (bytes, expected) with expected = the int quicklistPushTail stores (zipTryEncoding
    + string2ll said yes) or None (kept as a string).  The expectations are literals."""
    blob, el, p = bytearray(hdr(14, lru)), [], 5
    for s, want in items:
        blob += struct.pack("<I", len(s)) + s
        p += 4
        el.append([K_INT, want & M64, 0, 0] if want is not None else [K_STR, p, len(s), 0])
        p += len(s)
    return fx(name, cite, bytes(blob), 14, 0, lru, OK, len(items), el)


def w_intset(name, cite, width, vals, lru=0):
    blob = hdr(11, lru) + struct.pack("<II", width, len(vals)) + b"".join(
        v.to_bytes(width, "little", signed=True) for v in vals)
    return fx(name, cite, blob, 11, width, lru, OK, len(vals), [[K_INT, v & M64, 0, 0] for v in vals])


def w_ht(name, cite, t, members, count=None, keep=None, lru=0, status=OK, reserve=None):
    """SET_HT (t=2, members) / HASH_HT (t=4, field,value,...).  keep: literal indices of the
    members desSet's dictAdd keeps (default: all)."""
    per = 1 if t == 2 else 2
    n = len(members) // per if count is None else count
    blob, p, offs = bytearray(hdr(t, lru) + struct.pack("<Q", n)), 13, []
    for m in members:
        blob += struct.pack("<Q", len(m)) + m
        p += 8
        offs.append([K_STR, p, len(m), 0])
        p += len(m)
    f = fx(name, cite, bytes(blob), t, 0, lru, status, len(members) if reserve is None else reserve,
           [offs[i] for i in (range(len(members)) if keep is None else keep)])
    if keep is not None:   # what serObject writes for the set desSet built: the kept members
        f["reencoded"] = w_ht(name, cite, t, [members[i] for i in keep], lru=lru)["blob"]
    return f


def w_skiplist(name, cite, pairs, order=None, lru=0, status=OK, reserve=None):
    """pairs in blob order: (member bytes, score float or raw u64 bits).  order: literal indices
    of the pairs in the order serZset writes the rebuilt skiplist (default: blob order)."""
    blob, p, rec = bytearray(hdr(5, lru) + struct.pack("<Q", len(pairs))), 13, []
    for m, sc in pairs:
        bits = sc if isinstance(sc, int) else struct.unpack("<Q", struct.pack("<d", sc))[0]
        blob += struct.pack("<Q", len(m)) + m + struct.pack("<Q", bits)
        p += 8
        rec.append(([K_STR, p, len(m), 0], [K_SCORE, bits, 0, 0]))
        p += len(m) + 8
    el = [x for i in (range(len(pairs)) if order is None else order) for x in rec[i]]
    f = fx(name, cite, bytes(blob), 5, 0, lru, status, 2 * len(pairs) if reserve is None else reserve, el)
    if order is not None:   # what serZset writes for the skiplist desZset built
        f["reencoded"] = w_skiplist(name, cite, [pairs[i] for i in order], lru=lru)["blob"]
    return f


ZL_INT_SIZE = {0xFE: 1, 0xC0: 2, 0xF0: 3, 0xD0: 4, 0xE0: 8}


def zl_write(entries, big_prevlen_at=()):
    """A ziplist written entry by entry (__ziplistInsert tail pushes, ziplist.c:743-839).
    entries: ("s", bytes) strings, ("i", value, encoding byte) integers with the encoding the
    fixture states.  Returns (bytes, records) with records = [kind, offset in ziplist, len, zenc]
    for strings / [K_INT, value, 0, enc] for integers."""
    body, rec, prev, last = bytearray(), [], 0, 10
    for i, e in enumerate(entries):
        start = 10 + len(body)
        ent = bytearray(bytes([prev]) if prev < 254 and i not in big_prevlen_at else b"\xfe" + struct.pack("<I", prev))
        if e[0] == "s":
            s = e[1]
            if len(s) <= 0x3F:
                ent += bytes([len(s)]); cls = 0x00
            elif len(s) <= 0x3FFF:
                ent += bytes([0x40 | (len(s) >> 8), len(s) & 0xFF]); cls = 0x40
            else:
                ent += b"\x80" + struct.pack(">I", len(s)); cls = 0x80
            rec.append([K_STR, start + len(ent), len(s), cls])
            ent += s
        else:
            v, enc = e[1], e[2]
            ent += bytes([enc])
            if 0xF1 <= enc <= 0xFD:
                assert v == enc - 0xF1
            else:
                ent += v.to_bytes(ZL_INT_SIZE[enc], "little", signed=True)
            rec.append([K_INT, v & M64, 0, enc])
        body += ent
        last, prev = start, len(ent)
    zl = struct.pack("<IIH", 10 + len(body) + 1, last, min(len(entries), 0xFFFF)) + bytes(body) + b"\xff"
    return zl, rec


def w_ziplist(name, cite, t, entries, big_prevlen_at=(), lru=0):
    zl, rec = zl_write(entries, big_prevlen_at)
    blob = hdr(t, lru) + struct.pack("<Q", len(zl)) + zl
    el = [[K_ZLRAW, 13, len(zl), 0]] + [[k, d + 13 if k == K_STR else d, ln, z] for k, d, ln, z in rec]
    return fx(name, cite, blob, t, 0, lru, OK, 1 + len(entries), el)


def bad(name, cite, blob, status, reserve, enc=0):
    t = blob[0] if blob else 0
    lru = struct.unpack_from("<I", blob, 1)[0] if len(blob) >= 5 else 0
    return fx(name, cite, blob, t, enc, lru, status, reserve, [])


def S(x):
    return ("s", x)


def I(v, enc):
    return ("i", v, enc)


def edges():
    E = []
    I64 = lambda v: struct.pack("<q", v)  # noqa: E731
    for v in (0, -1, -(1 << 63), (1 << 63) - 1):
        E.append(w_string(f"string_int_{v}", "rock_serdes.c:144-146", 1, I64(v), lru=5))
    E.append(w_string("string_embstr_44", "rock_serdes.c:152 (limit 44)", 8, b"e" * 44, lru=1))
    E.append(w_string("string_embstr_0", "rock_serdes.c:151-153", 8, b"", lru=1))
    E.append(w_string("string_raw_44", "rock_serdes.c:149-150 (RAW may be short)", 0, b"r" * 44, lru=2))
    E.append(w_string("string_raw_45", "rock_serdes.c:149-150", 0, b"r" * 45, lru=2))
    E.append(w_string("string_raw_binary_nul", "rock_serdes.c:150 (HLL values are RAW binary)", 0,
                      bytes([0, 1, 0, 255, 0, 0, 7]), lru=3))
    E.append(w_string("lru_high_bits_masked", "server.h:592-599 (24-bit lru)", 8, b"ab", lru=0xFF123456))
    # List elements: the int each one becomes (zipTryEncoding ziplist.c:480 + string2ll util.c:360)
    E.append(w_list("list_all_int_widths", "rock_serdes.c:207 quicklistPushTail -> zipTryEncoding", [
        (b"0", 0), (b"12", 12), (b"13", 13), (b"-1", -1), (b"127", 127), (b"128", 128), (b"-128", -128),
        (b"-129", -129), (b"32767", 32767), (b"32768", 32768), (b"-32768", -32768), (b"-32769", -32769),
        (b"8388607", 8388607), (b"8388608", 8388608), (b"-8388608", -8388608), (b"-8388609", -8388609),
        (b"2147483647", 2147483647), (b"2147483648", 2147483648), (b"-2147483648", -2147483648),
        (b"-2147483649", -2147483649), (b"9223372036854775807", 9223372036854775807),
        (b"-9223372036854775808", -9223372036854775808)], lru=9))
    E.append(w_list("list_not_ints", "util.c:360-424 (strict), ziplist.c:480 (1..31 bytes)", [
        (b"99999999999999999999", None), (b"-0", None), (b"+1", None), (b"01", None), (b" 1", None),
        (b"", None), (b"9223372036854775808", None), (b"1234567890123456789012345678901", None),
        (b"12345678901234567890123456789012", None)], lru=9))
    E.append(w_list("list_empty", "rock_serdes.c:201 (no elements)", [], lru=9))
    E.append(w_intset("intset_w2", "intset.h:34-38, rock_serdes.c:255-276", 2, [-32768, 0, 32767]))
    E.append(w_intset("intset_w4", "intset.h:34-38", 4, [-2147483648, 1, 2147483647]))
    E.append(w_intset("intset_w8", "intset.h:34-38", 8, [-(1 << 63), 0, (1 << 63) - 1]))
    E.append(w_intset("intset_empty", "rock_serdes.c:274 (0 == 2*0)", 2, []))
    E.append(w_ht("set_ht_empty_member", "rock_serdes.c:291 (could be empty string)", 2, [b"", b"x"]))
    E.append(w_ziplist("hash_ziplist_14b_32b_prevlen5", "ziplist.c:55-106 (06/14/32-bit lengths, 5-byte prevlen)",
                       13, [S(b"f1"), S(b"a" * 63), S(b"f2"), S(b"b" * 64), S(b"f3"), S(b"c" * 253),
                            S(b"f4"), S(b"d" * 254), S(b"f5"), S(b"e" * 16383), S(b"f6"), S(b"g" * 16384)]))
    E.append(w_ziplist("zset_ziplist_nonminimal_prevlen", "ziplist.c:391-419 (5-byte prevlen kept after a cascade)",
                       12, [S(b"a"), I(1, 0xF2), S(b"bb"), I(-70000, 0xF0)], big_prevlen_at=(1, 2)))
    E.append(w_ziplist("zset_ziplist_special_scores", "util.c:517-552 d2string; '-0' is not string2ll-able",
                       12, [S(b"m0"), S(b"-inf"), S(b"m1"), S(b"-0"), S(b"m2"), I(0, 0xF1), S(b"m3"), S(b"1.5"),
                            S(b"m4"), S(b"inf")]))
    E.append(w_ziplist("hash_ziplist_int_values", "ziplist.c:480-566 integer widths",
                       13, [S(b"k"), I(300, 0xC0), S(b"k2"), I(-5, 0xFE), S(b"k3"), I(1 << 40, 0xE0),
                            S(b"k4"), I(-(1 << 20), 0xF0)]))
    E.append(w_ziplist("hash_ziplist_empty", "ziplist.c:193-256 (empty: 11 bytes)", 13, []))
    E.append(w_skiplist("zset_skiplist_inf_negzero_ties", "rock_serdes.c:430-440 (already descending)",
                        [(b"z", math.inf), (b"b", 2.0), (b"a", 2.0), (b"c", -0.0), (b"d", -math.inf)]))
    E.append(w_ht("hash_ht_empty_field_value", "rock_serdes.c:378-404", 4, [b"", b""]))
    # --- reconstruction rules of desSet / desHash / desZset (the flat form = what serObject
    #     would write for the object the reference builds) ---
    E.append(w_ht("hash_ht_repeated_values_ok", "rock_serdes.c:399 (values may repeat)", 4,
                  [b"a", b"v", b"b", b"v"]))
    E.append(w_ht("set_ht_dup_members", "rock_serdes.c:297 dictAdd keeps the first, ignores the rest", 2,
                  [b"x", b"yy", b"x", b"z", b"yy"], keep=[0, 1, 3]))
    E.append(w_ht("set_ht_dup_empty", "rock_serdes.c:297", 2, [b"", b""], keep=[0]))
    E.append(w_skiplist("zset_skiplist_unsorted", "zslInsert t_zset.c:132-180 re-sorts; serZset writes descending",
                        [(b"a", 1.0), (b"b", 2.0), (b"c", 0.0)], order=[1, 0, 2]))
    E.append(w_skiplist("zset_skiplist_negzero_dup_members", "t_zset.c:143-146 (-0.0 == 0.0: member order, "
                        "then blob order); rock_serdes.c:499 dictAdd ignores the repeat",
                        [(b"a", 0.0), (b"m", -0.0), (b"m", 0.0)], order=[1, 2, 0]))
    E.append(w_skiplist("zset_skiplist_same_score_members", "t_zset.c:143-146 sdscmp tie-break",
                        [(b"a", 1.0), (b"b", 1.0), (b"ab", 1.0)], order=[1, 2, 0]))
    E.append(w_skiplist("zset_skiplist_dup_member_two_scores", "rock_serdes.c:498-499 (both nodes kept)",
                        [(b"x", 1.0), (b"x", 2.0)], order=[1, 0]))
    # --- malformed blobs: each maps to the reference's assert site (or a [stricter] deviation) ---
    E.append(bad("bad_short_header", "rock_serdes.c:542", b"\x00\x00\x00", SHORT, 0))
    E.append(bad("bad_empty", "rock_serdes.c:539", b"", SHORT, 0))
    E.append(bad("bad_string_no_enc", "rock_serdes.c:134", hdr(0), SHORT, 0))
    E.append(bad("bad_unknown_type", "rock_serdes.c:561", hdr(7) + b"xx", TYPE, 0))
    E.append(bad("bad_string_enc", "rock_serdes.c:148", hdr(0) + b"\x05abc", STR_ENC, 1, enc=5))
    E.append(bad("bad_string_int_len", "rock_serdes.c:145", hdr(0) + b"\x01" + b"\x00" * 7, STR_INTLEN, 1, enc=1))
    E.append(bad("bad_embstr_45", "rock_serdes.c:152", hdr(0) + b"\x08" + b"x" * 45, EMBSTR_LEN, 1, enc=8))
    E.append(bad("bad_list_trunc_len", "rock_serdes.c:202", hdr(14) + b"\x05\x00", TRUNC, 0))
    E.append(bad("bad_list_trunc_body", "rock_serdes.c:206", hdr(14) + struct.pack("<I", 10) + b"abc", TRUNC, 0))
    E.append(bad("bad_intset_width", "[stricter] reference accepts width 3 (rock_serdes.c:274 only checks the length)",
                 hdr(11) + struct.pack("<II", 3, 1) + b"abc", INTSET, 0))
    E.append(bad("intset_u32_wrap", "[stricter] reference's u32 width*count wraps to 0 == len (rock_serdes.c:268,274)",
                 hdr(11) + struct.pack("<II", 8, 0x20000000), INTSET, 0))
    E.append(bad("bad_intset_len", "rock_serdes.c:274", hdr(11) + struct.pack("<II", 2, 2) + b"ab", INTSET, 0))
    # count 2, one member: reservation min(2, (22-13)/8) = 1
    E.append(bad("bad_set_ht_count", "rock_serdes.c:303", hdr(2) + struct.pack("<QQ", 2, 1) + b"x", COUNT, 1))
    E.append(bad("bad_hash_ht_missing_value", "rock_serdes.c:389",
                 hdr(4) + struct.pack("<QQ", 1, 1) + b"f", TRUNC, 1))
    # duplicate field: count 2, (49-13)/8 = 4 >= 2*2 -> reservation 4
    E.append(bad("hash_ht_dup_field", "rock_serdes.c:399-400 serverAssert(ret == DICT_OK)",
                 hdr(4) + struct.pack("<Q", 2) + b"".join(struct.pack("<Q", 1) + x for x in (b"f", b"1", b"f", b"2")),
                 DUP, 4))
    E.append(bad("hash_ht_dup_field_long", "rock_serdes.c:399-400 (fields compared as whole sds)",
                 hdr(4) + struct.pack("<Q", 3) + b"".join(struct.pack("<Q", len(x)) + x for x in (
                     b"field-0123456789abcdef", b"v1", b"field-0123456789abcdeX", b"v2", b"field-0123456789abcdef",
                     b"v3")), DUP, 6))
    # NaN score: reservation 2*min(1, (30-13)/16) = 2
    E.append(bad("zset_skiplist_nan", "t_zset.c:137 serverAssert(!isnan(score)) via rock_serdes.c:498",
                 hdr(5) + struct.pack("<QQ", 1, 1) + b"a" + struct.pack("<Q", 0x7FF8000000000000), NAN, 2))
    E.append(bad("zset_skiplist_nan_negative_payload", "t_zset.c:137",
                 hdr(5) + struct.pack("<Q", 2) + struct.pack("<Q", 1) + b"a" + struct.pack("<d", 1.0) +
                 struct.pack("<Q", 1) + b"b" + struct.pack("<Q", 0xFFF0000000000001), NAN, 4))
    # ziplist blobs: reservation 1 + min(zllen, (Lz-11)/2)
    E.append(bad("bad_ziplist_len", "rock_serdes.c:360", hdr(13) + struct.pack("<Q", 99) + zl_write([S(b"a"), S(b"b")])[0],
                 ZL_LEN, 0))
    zl = bytearray(zl_write([S(b"a"), S(b"b")])[0])   # Lz 17, zllen 2
    zl[11] = 0xC5                                       # entry 0's encoding: no such encoding (zipIntSize)
    E.append(bad("bad_ziplist_encoding", "[stricter] ziplist.c:300-447 (the reference copies it blind)",
                 hdr(13) + struct.pack("<Q", len(zl)) + bytes(zl), ZL_CORRUPT, 3))
    zl = zl_write([S(b"a"), S(b"b"), S(b"c")])[0]      # Lz 20, zllen 3: 1 + min(3, 4)
    E.append(bad("bad_ziplist_odd_entries", "[stricter] field without a value (t_hash.c:229-231 pairs)",
                 hdr(13) + struct.pack("<Q", len(zl)) + zl, ZL_CORRUPT, 4))
    zl = bytearray(zl_write([S(b"a"), S(b"b")])[0])
    zl[8] = 5                                           # zllen 5: 1 + min(5, 3)
    E.append(bad("bad_ziplist_zllen", "[stricter] zllen != entries (ziplist.c:193-256)",
                 hdr(12) + struct.pack("<Q", len(zl)) + bytes(zl), ZL_CORRUPT, 4))
    E.append(bad("bad_skiplist_trailing", "rock_serdes.c:501", hdr(5) + struct.pack("<Q", 0) + b"\x01", COUNT, 0))
    E.append(bad("bad_skiplist_trunc_score", "rock_serdes.c:493",
                 hdr(5) + struct.pack("<QQ", 1, 1) + b"a" + b"\x00" * 4, TRUNC, 0))
    return E


def shapes():
    """Values built the way the reference's own tests build them, expected flat forms written
    by the recording writers from the construction (every zipTryEncoding decision a literal):

      ziplist.c:1255-1281  createList / createIntList — the ziplists ziplist.c's self-test
                           builds by ziplistPush (HEAD pushes included), each as a hash ziplist;
      testredrock/test_redrock.py:76-111 (_warm_up_with_all_data_types) — the value of every
                           data type the E2E checker warms up, in the encoding Redis gives it
                           under the reference's config defaults (SURVEY.md §5 Config)."""
    E = []
    # createList: push "foo" T, "quux" T, "hello" H, "1024" T -> hello, foo, quux, 1024; "1024"
    # passes zipTryEncoding as a 16-bit integer (ziplist.c:486-498: > INT8_MAX, <= INT16_MAX)
    E.append(w_ziplist("ziplist_c_createList", "ziplist.c:1255-1262", 13,
                       [S(b"hello"), S(b"foo"), S(b"quux"), I(1024, 0xC0)]))
    # createIntList: "100" T, "128000" T, "-100" H, "4294967296" H, "non integer" T,
    # "much much longer non integer" T -> 4294967296, -100, 100, 128000, then the two strings;
    # widths: 2^32 > INT32_MAX -> 64-bit, -100 / 100 -> 8-bit, 128000 -> 24-bit
    E.append(w_ziplist("ziplist_c_createIntList", "ziplist.c:1264-1281", 13,
                       [I(4294967296, 0xE0), I(-100, 0xFE), I(100, 0xFE), I(128000, 0xF0), S(b"non integer"),
                        S(b"much much longer non integer")]))
    # String: "0123...1999" (6,890 bytes), RAW (longer than the 44-byte EMBSTR limit)
    s = "".join(str(i) for i in range(2000)).encode()
    assert len(s) == 6890
    E.append(w_string("redrock_py_string_0_1999", "test_redrock.py:82-84,96 r.set(i, string_val)", 0, s, lru=0x00ABCD))
    # List: lpush 0..99 -> 99, 98, ..., 0; every element an integer entry (serList renders it
    # by sdsll2str, desList's quicklistPushTail re-encodes it as that integer)
    E.append(w_list("redrock_py_list_lpush_100", "test_redrock.py:97-99 r.lpush(i, j)",
                    [(str(j).encode(), j) for j in range(99, -1, -1)], lru=0x00ABCD))
    # Set: sadd 0..999 -> past set-max-intset-entries (512, config.c:2262) the intset becomes a
    # hash table of decimal members (any dict order; this one ascending)
    E.append(w_ht("redrock_py_set_1000", "test_redrock.py:100-103 r.sadd(i, j), 1000 > 512 -> HT", 2,
                  [str(j).encode() for j in range(1000)], lru=0x00ABCD))
    # Hash: hset j -> "0123...99" (190 bytes) for 1000 fields -> HT (1000 > 512 entries, 190 > 64 bytes)
    hv = "".join(str(i) for i in range(100)).encode()
    assert len(hv) == 190
    E.append(w_ht("redrock_py_hash_1000x190", "test_redrock.py:104-107 r.hset(i, j, hash_field_val)", 4,
                  [x for j in range(1000) for x in (str(j).encode(), hv)], lru=0x00ABCD))
    # ZSet: zadd {j: j} for 100 members -> ziplist (100 <= 128 entries): member j and score
    # d2string(j) = "j" are both integer entries (0..12 immediate 0xF1+j, 13..99 8-bit), ascending
    zent = []
    for j in range(100):
        e = I(j, 0xF1 + j) if j <= 12 else I(j, 0xFE)
        zent += [e, e]
    E.append(w_ziplist("redrock_py_zset_ziplist_100", "test_redrock.py:108-111 r.zadd(i, {j: j}), t_zset.c:1029-1050",
                       12, zent))
    # Geo: a zset ziplist of members with integral 52-bit geohash scores (d2string -> ll2string ->
    # a 64-bit integer entry); scores in ascending order
    E.append(w_ziplist("redrock_py_geo_zset", "test_redrock.py:112-114 r.geoadd(...): zset of geohash scores", 12,
                       [S(b"Palermo"), I(3479099956230698, 0xE0), S(b"Catania"), I(3479447370796909, 0xE0)]))
    # HyperLogLog: a RAW binary string (sparse encoding header "HYLL", encoding 1, cached
    # cardinality, opcodes): NUL and high bytes in the payload
    hll = b"HYLL" + bytes([1, 0, 0, 0]) + bytes([7, 0, 0, 0, 0, 0, 0, 0]) + bytes(
        [0x7F, 0xFF, 0x80, 0x51, 0x7F, 0x3A, 0x84, 0x4C, 0x90, 0x7F, 0xFF, 0x7F, 0xFF, 0x5E, 0x10])
    E.append(w_string("redrock_py_hll_raw_binary", "test_redrock.py:115-117 r.pfadd(...): RAW binary", 0, hll))
    return E


def check_against_pyoracle(kats, edges_):
    """Consistency report: the Python restatement must agree with every literal."""
    from oracle import pyoracle as po
    bad_ = []
    for f in kats + edges_:
        blob = bytes.fromhex(f["blob"])
        v, es = po.decode_one(blob, 0)
        want = f["value"]
        got_el = [[e[0], e[1] & M64, e[2], e[3]] for e in es]
        if v["status"] != want.get("status", 0) or v["enc"] != want["enc"] or v["lru"] != want["lru"] or \
                got_el != f["elems"] or ("reserve" in want and po.reserve(blob) != want["reserve"]):
            bad_.append((f["name"], v, got_el[:6], want, f["elems"][:6]))
    return bad_


def main():
    kats = [dict(k, blob=h(k["blob"]).hex()) for k in KATS]
    ed = edges()
    names = [e["name"] for e in ed]
    assert len(names) == len(set(names))
    sh = shapes()
    assert not set(e["name"] for e in sh) & set(names)
    mism = check_against_pyoracle(kats, ed + sh)
    if mism:
        for m in mism:
            print("MISMATCH", *m, sep="\n  ")
        raise SystemExit(1)
    doc = dict(generator="tests/golden/make_golden.py", kats=kats, edges=ed, shapes=sh, string2ll=STRING2LL,
               ll2string=LL2STRING, ziplist_example=ZIPLIST_EXAMPLE, intset_encoding=INTSET_ENC)
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1)
    print(f"wrote {OUT}: {len(kats)} KATs, {len(ed)} edge fixtures, {len(sh)} reference-shaped values")


if __name__ == "__main__":
    main()

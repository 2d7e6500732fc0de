"""Generates tests/golden/kat.json — committed golden vectors for the serdes path.

Two kinds of fixture:
  * KAT  — known-answer vectors hand-derived from the reference's source text
           (SURVEY.md §8c table K1-K9).  Both the blob bytes and the flat form are written
           here by hand, NOT computed by an oracle: the tests require every oracle and the GPU
           to decode the blob into exactly this flat form and to encode it back into exactly
           these bytes.
  * EDGE — edge cases SURVEY.md §8c asks for (widths, 14/32-bit ziplist lengths, 5-byte
           prevlen, LLONG_MIN/MAX, empty members, ±inf/-0.0 scores, malformed blobs).  Blobs
           are built with the ziplist/intset writers of oracle/pyoracle.py; the expected flat
           form is the Python restatement's decode (the C oracle and GPU are checked against it).

The reference itself is not run (SURVEY.md §8c denial); this script only uses oracle/pyoracle.
Run:  python tests/golden/make_golden.py
"""
import json
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import pyoracle as po  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kat.json")


def h(s):
    return bytes.fromhex(s.replace(" ", ""))


K3_LITERAL = b"aadfcrghsdgggggggggggadbAFWEdsar4dadsrd423FASFASXASDFASR3ADFASDFASFASR34RFADSFSADFSAFXEEdsdec"[:60]

# Hand-derived KATs.  elems: [kind, data, len, zenc]; STR data = byte offset in blob.
KATS = [
    dict(name="K1_string_int_134123", cite="rock_serdes.c:832 (createStringObjectFromLongLongForValue)",
         blob="00 00000000 01 EB0B020000000000",
         value=dict(type=0, enc=1, lru=0), elems=[[po.K_INT, 134123, 0, 0]]),
    dict(name="K2_string_embstr_abc", cite="rock_serdes.c:847", blob="00 00000000 08 616263",
         value=dict(type=0, enc=8, lru=0), elems=[[po.K_STR, 6, 3, 0]]),
    dict(name="K3_string_raw_60", cite="rock_serdes.c:864", blob="00 00000000 00 " + K3_LITERAL.hex(),
         value=dict(type=0, enc=0, lru=0), elems=[[po.K_STR, 6, 60, 0]]),
    dict(name="K4_list_xxx_-1234567", cite="rock_serdes.c:815-819 (ZIP_INT_24B re-rendered by sdsll2str)",
         blob="0E 00000000 03000000 787878 08000000 2D31323334353637",
         value=dict(type=14, enc=0, lru=0), elems=[[po.K_STR, 9, 3, 0], [po.K_INT, -1234567, 0, 0]]),
    dict(name="K5_zset_ziplist_2_5", cite="ziplist.c:114-149 worked example, rock_serdes.c:420-423",
         blob="0C 00000000 0F00000000000000 0F000000 0C000000 0200 00F3 02F6 FF",
         value=dict(type=12, enc=0, lru=0),
         elems=[[po.K_ZLRAW, 13, 15, 0], [po.K_INT, 2, 0, 0xF3], [po.K_INT, 5, 0, 0xF6]]),
    dict(name="K6_set_intset_123", cite="intset.c:45-52 (INT16), rock_serdes.c:220-226",
         blob="0B 00000000 02000000 03000000 010002000300",
         value=dict(type=11, enc=2, lru=0),
         elems=[[po.K_INT, 1, 0, 0], [po.K_INT, 2, 0, 0], [po.K_INT, 3, 0, 0]]),
    dict(name="K7_hash_ht_f_v", cite="rock_serdes.c:322-339",
         blob="04 00000000 0100000000000000 0100000000000000 66 0100000000000000 76",
         value=dict(type=4, enc=0, lru=0), elems=[[po.K_STR, 21, 1, 0], [po.K_STR, 30, 1, 0]]),
    dict(name="K8_zset_skiplist_a1_b2", cite="rock_serdes.c:425-440 (tail->head = descending)",
         blob="05 00000000 0200000000000000 0100000000000000 62 0000000000000040 "
              "0100000000000000 61 000000000000F03F",
         value=dict(type=5, enc=0, lru=0),
         elems=[[po.K_STR, 21, 1, 0], [po.K_SCORE, 0x4000000000000000, 0, 0],
                [po.K_STR, 38, 1, 0], [po.K_SCORE, 0x3FF0000000000000, 0, 0]]),
    dict(name="K9_set_ht_x", cite="rock_serdes.c:227-239",
         blob="02 00000000 0100000000000000 0100000000000000 78",
         value=dict(type=2, enc=0, lru=0), elems=[[po.K_STR, 21, 1, 0]]),
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


def lru_hdr(t, lru=0):
    return bytes([t]) + struct.pack("<I", lru)


def edge_blobs():
    E = []
    I64 = lambda v: struct.pack("<q", v)  # noqa: E731
    for v in (0, -1, -(1 << 63), (1 << 63) - 1):
        E.append((f"string_int_{v}", lru_hdr(0, 5) + b"\x01" + I64(v)))
    E.append(("string_embstr_44", lru_hdr(0, 1) + b"\x08" + b"e" * 44))
    E.append(("string_embstr_0", lru_hdr(0, 1) + b"\x08"))
    E.append(("string_raw_44", lru_hdr(0, 2) + b"\x00" + b"r" * 44))
    E.append(("string_raw_45", lru_hdr(0, 2) + b"\x00" + b"r" * 45))
    E.append(("string_raw_binary_nul", lru_hdr(0, 3) + b"\x00" + bytes([0, 1, 0, 255, 0, 0, 7])))
    E.append(("lru_high_bits_masked", bytes([0]) + struct.pack("<I", 0xFF123456) + b"\x08ab"))
    ints = ["0", "12", "13", "-1", "127", "128", "-128", "-129", "32767", "32768", "-32768", "-32769",
            "8388607", "8388608", "-8388608", "-8388609", "2147483647", "2147483648", "-2147483648",
            "-2147483649", "9223372036854775807", "-9223372036854775808"]
    nonints = ["99999999999999999999", "-0", "+1", "01", " 1", "", "9223372036854775808",
               "1234567890123456789012345678901", "12345678901234567890123456789012"]

    def lst(items):
        b = lru_hdr(14, 9)
        for it in items:
            it = it.encode()
            b += struct.pack("<I", len(it)) + it
        return b
    E.append(("list_all_int_widths", lst(ints)))
    E.append(("list_not_ints", lst(nonints)))
    E.append(("list_empty", lst([])))
    for w, vals in ((2, [-32768, 0, 32767]), (4, [-2147483648, 1, 2147483647]),
                    (8, [-(1 << 63), 0, (1 << 63) - 1])):
        b = lru_hdr(11) + struct.pack("<II", w, len(vals)) + b"".join(v.to_bytes(w, "little", signed=True) for v in vals)
        E.append((f"intset_w{w}", b))
    E.append(("intset_empty", lru_hdr(11) + struct.pack("<II", 2, 0)))
    E.append(("set_ht_empty_member", lru_hdr(2) + struct.pack("<Q", 2) + struct.pack("<Q", 0) +
              struct.pack("<Q", 1) + b"x"))
    zl = po.build_ziplist([b"f1", b"a" * 63, b"f2", b"b" * 64, b"f3", b"c" * 253, b"f4", b"d" * 254,
                           b"f5", b"e" * 16383, b"f6", b"g" * 16384])
    E.append(("hash_ziplist_14b_32b_prevlen5", lru_hdr(13) + struct.pack("<Q", len(zl)) + zl))
    zl = po.build_ziplist([b"a", b"1", b"bb", b"-70000"], big_prevlen_at=(1, 2))
    E.append(("zset_ziplist_nonminimal_prevlen", lru_hdr(12) + struct.pack("<Q", len(zl)) + zl))
    zl = po.build_ziplist([b"m0", b"-inf", b"m1", b"-0", b"m2", b"0", b"m3", b"1.5", b"m4", b"inf"])
    E.append(("zset_ziplist_special_scores", lru_hdr(12) + struct.pack("<Q", len(zl)) + zl))
    zl = po.build_ziplist([b"k", 300, b"k2", -5, b"k3", 1 << 40, b"k4", -(1 << 20)])
    E.append(("hash_ziplist_int_values", lru_hdr(13) + struct.pack("<Q", len(zl)) + zl))
    zl = po.build_ziplist([])
    E.append(("hash_ziplist_empty", lru_hdr(13) + struct.pack("<Q", len(zl)) + zl))
    sk = lru_hdr(5) + struct.pack("<Q", 5)
    for m, s in ((b"z", float("inf")), (b"b", 2.0), (b"a", 2.0), (b"c", -0.0), (b"d", float("-inf"))):
        sk += struct.pack("<Q", len(m)) + m + struct.pack("<d", s)
    E.append(("zset_skiplist_inf_negzero_ties", sk))
    E.append(("hash_ht_empty_field_value", lru_hdr(4) + struct.pack("<Q", 1) + struct.pack("<Q", 0) +
              struct.pack("<Q", 0)))
    # --- malformed blobs: every serverAssert/serverPanic site maps to a status ---
    E.append(("bad_short_header", b"\x00\x00\x00"))
    E.append(("bad_empty", b""))
    E.append(("bad_string_no_enc", lru_hdr(0)))
    E.append(("bad_unknown_type", lru_hdr(7) + b"xx"))
    E.append(("bad_string_enc", lru_hdr(0) + b"\x05abc"))
    E.append(("bad_string_int_len", lru_hdr(0) + b"\x01" + b"\x00" * 7))
    E.append(("bad_embstr_45", lru_hdr(0) + b"\x08" + b"x" * 45))
    E.append(("bad_list_trunc_len", lru_hdr(14) + b"\x05\x00"))
    E.append(("bad_list_trunc_body", lru_hdr(14) + struct.pack("<I", 10) + b"abc"))
    E.append(("bad_intset_width", lru_hdr(11) + struct.pack("<II", 3, 1) + b"abc"))
    E.append(("bad_intset_len", lru_hdr(11) + struct.pack("<II", 2, 2) + b"ab"))
    E.append(("bad_set_ht_count", lru_hdr(2) + struct.pack("<Q", 2) + struct.pack("<Q", 1) + b"x"))
    E.append(("bad_hash_ht_missing_value", lru_hdr(4) + struct.pack("<Q", 1) + struct.pack("<Q", 1) + b"f"))
    E.append(("bad_ziplist_len", lru_hdr(13) + struct.pack("<Q", 99) + po.build_ziplist([b"a", b"b"])))
    zl = bytearray(po.build_ziplist([b"a", b"b"]))
    zl[11] = 0xC5  # invalid integer encoding byte of entry 0 (zipIntSize panics)
    E.append(("bad_ziplist_encoding", lru_hdr(13) + struct.pack("<Q", len(zl)) + bytes(zl)))
    zl = po.build_ziplist([b"a", b"b", b"c"])
    E.append(("bad_ziplist_odd_entries", lru_hdr(13) + struct.pack("<Q", len(zl)) + zl))
    zl = bytearray(po.build_ziplist([b"a", b"b"]))
    zl[8] = 5  # zllen mismatch
    E.append(("bad_ziplist_zllen", lru_hdr(12) + struct.pack("<Q", len(zl)) + bytes(zl)))
    E.append(("bad_skiplist_trailing", lru_hdr(5) + struct.pack("<Q", 0) + b"\x01"))
    E.append(("bad_skiplist_trunc_score", lru_hdr(5) + struct.pack("<Q", 1) + struct.pack("<Q", 1) + b"a" + b"\x00" * 4))
    return E


def main():
    kats = []
    for k in KATS:
        assert po.reserve(h(k["blob"])) == len(k["elems"])
        kats.append(dict(k, blob=h(k["blob"]).hex()))
    edges = []
    for name, blob in edge_blobs():
        v, es = po.decode_one(blob, 0)
        edges.append(dict(name=name, blob=blob.hex(),
                          value=dict(type=v["type"], enc=v["enc"], lru=v["lru"], status=v["status"],
                                     n_elems=v["n_elems"], reserve=po.reserve(blob)),
                          elems=[[e[0], e[1] & 0xFFFFFFFFFFFFFFFF, e[2], e[3]] for e in es]))
    doc = dict(generator="tests/golden/make_golden.py", kats=kats, edges=edges, string2ll=STRING2LL,
               ll2string=LL2STRING, ziplist_example=ZIPLIST_EXAMPLE, intset_encoding=INTSET_ENC)
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1)
    print(f"wrote {OUT}: {len(kats)} KATs, {len(edges)} edge fixtures")


if __name__ == "__main__":
    main()

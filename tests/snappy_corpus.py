"""Deterministic inputs for the snappy block-compression tests.

Synthetic stand-ins for the kinds of data snappy's own test corpus covers (text, markup,
protocol buffers, already-compressed bytes), RocksDB-sized data blocks of the engine's own
value blobs, the compressor's edge sizes, and hand-built compressed streams (literal / copy
tags written by hand from the format, format_description.txt in deps/snappy) with the status
the format gives each of them.
"""
import numpy as np

import redrock_old_amd as rr

WORDS = ("the of and to in a is that for it as was with be by on not he this are or his from at which "
         "but have an they you were her she there been one all we their has would when if so no what up "
         "said out its about who them into some could him time only other new more these two may first "
         "value key block table level cache snapshot evict restore rocks redis hash list set zset").split()


def text(n, seed):
    rng = np.random.default_rng(seed)
    out, size = [], 0
    while size < n:
        w = WORDS[int(rng.zipf(1.3)) % len(WORDS)]
        if rng.random() < 0.08:
            w = w.capitalize() + (". " if rng.random() < 0.5 else ", ")
        else:
            w += " "
        out.append(w)
        size += len(w)
    return "".join(out).encode()[:n]


def markup(n, seed):
    rng = np.random.default_rng(seed)
    parts, size = [], 0
    while size < n:
        t = ["div", "span", "a", "p", "li", "td"][int(rng.integers(6))]
        s = f'<{t} class="c{int(rng.integers(40))}" id="x{int(rng.integers(100000))}">{text(int(rng.integers(5, 80)), int(rng.integers(1 << 30))).decode()}</{t}>\n'
        parts.append(s)
        size += len(s)
    return "".join(parts).encode()[:n]


def protobuf_like(n, seed):
    rng = np.random.default_rng(seed)
    out = bytearray()
    while len(out) < n:
        field = int(rng.integers(1, 16))
        if rng.random() < 0.6:
            out += bytes([(field << 3) | 0]) + bytes([int(x) | 0x80 for x in rng.integers(0, 128, int(rng.integers(0, 3)))]) + bytes([int(rng.integers(0, 128))])
        else:
            s = text(int(rng.integers(1, 30)), int(rng.integers(1 << 30)))
            out += bytes([(field << 3) | 2, len(s)]) + s
    return bytes(out[:n])


def random_bytes(n, seed):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


def corpus():
    """name -> bytes (whole inputs of 0 .. ~200 KB: several 64 KiB fragments for the big ones)."""
    c = {
        "empty": b"", "one": b"a", "two": b"ab", "three": b"abc",
        "m14": text(14, 1), "m15": text(15, 2), "m16": text(16, 3), "m17": text(17, 4),
        "zeros_100k": b"\0" * 100000, "pattern_4": b"abcd" * 5000,
        "snappy_unittest_like": b"aaaaaaa" + b"b" * 2047 + b"aaaaa" + b"abc",
        "long_run": b"aaaaaaa" + b"b" * 65536 + b"aaaaa" + b"abc",
        "text_150k": text(150000, 10), "markup_100k": markup(100000, 11), "proto_120k": protobuf_like(120000, 12),
        "random_120k": random_bytes(120000, 13), "random_16k": random_bytes(16384, 14),
        "lit60": bytes(range(60)) + b"0123" * 8, "lit61": bytes(range(61)) + b"0123" * 8,
        "lit256": random_bytes(256, 15) + b"xyzw" * 10, "lit65536": random_bytes(65536, 16) + b"q" * 100,
    }
    data, offs = rr.gen_batch(4, 3000)
    c["blobs_cfg4_200k"] = data[:200000].tobytes()
    data3, _ = rr.gen_batch(3, 300)
    c["blobs_cfg3_64k"] = data3[:65536].tobytes()
    return c


def blocks(buf, size):
    """RocksDB-style data blocks: consecutive `size`-byte pieces (last one shorter)."""
    n = len(buf)
    cuts = list(range(0, n, size)) + [n]
    return cuts if n else [0, 0]


# ---- hand-built compressed streams (tags straight from the format) -------------------------
def varint(v):
    out = bytearray()
    while v >= 128:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def lit(b):
    n = len(b) - 1
    if n < 60:
        return bytes([n << 2]) + b
    cnt = (n.bit_length() + 7) // 8
    return bytes([(59 + cnt) << 2]) + n.to_bytes(cnt, "little") + b


def copy1(off, ln):
    return bytes([1 | ((ln - 4) << 2) | ((off >> 8) << 5), off & 0xFF])


def copy2(off, ln):
    return bytes([2 | ((ln - 1) << 2), off & 0xFF, off >> 8])


def copy4(off, ln):
    return bytes([3 | ((ln - 1) << 2)]) + off.to_bytes(4, "little")


def crafted():
    """(name, stream, status, expected output or None); statuses of rr_snappy.h."""
    frag1 = b"012345689abcdefghijklmnopqrstuvwxyz"
    frag2 = b"some other string"
    n2 = 100000 // len(frag2)
    src = frag1 * 2 + frag2 * n2   # snappy_unittest's FourByteOffset shape: a copy-4 reaching back
    four = varint(len(src)) + lit(frag1) + b"".join(lit(frag2) for _ in range(n2)) + copy4(len(frag1) + n2 * len(frag2), len(frag1))
    four_out = frag1 + frag2 * n2 + frag1
    four = varint(len(four_out)) + four[len(varint(len(src))):]
    rle = varint(1 + 63) + lit(b"z") + copy2(1, 63)                            # overlapping copy, offset 1
    ovl3 = varint(3 + 40) + lit(b"xyz") + copy2(3, 40)                         # offset 3 < length
    c1 = varint(4 + 11) + lit(b"abcd") + copy1(4, 11)                          # copy-1 at its longest
    return [
        ("four_byte_offset", four, 0, four_out),
        ("rle_offset1", rle, 0, b"z" * 64),
        ("overlap_offset3", ovl3, 0, b"xyz" * 14 + b"x"),
        ("copy1_len11", c1, 0, b"abcd" * 3 + b"abc"),
        ("long_literal_2byte_len", varint(300) + lit(bytes(range(256)) + bytes(44)), 0, bytes(range(256)) + bytes(44)),
        ("empty", varint(0), 0, b""),
        ("no_preamble", b"", 1, None),
        ("preamble_6_bytes", b"\x80\x80\x80\x80\x80\x01", 1, None),
        ("preamble_5th_byte_16", b"\x80\x80\x80\x80\x10" + lit(b"a"), 1, None),
        ("preamble_unterminated", b"\x85\x81", 1, None),
        ("truncated_tag", varint(5) + lit(b"abcd") + b"\x02\x04", 2, None),
        ("truncated_literal", varint(10) + bytes([9 << 2]) + b"abc", 2, None),
        ("truncated_litlen", varint(100) + bytes([61 << 2]), 2, None),
        ("offset_zero", varint(8) + lit(b"abcd") + copy2(0, 4), 3, None),
        ("offset_past_start", varint(8) + lit(b"abcd") + copy2(5, 4), 3, None),
        ("copy_first", varint(4) + copy1(1, 4), 3, None),
        ("overflow_literal", varint(3) + lit(b"abcd"), 4, None),
        ("overflow_copy", varint(6) + lit(b"abcd") + copy1(4, 4), 4, None),
        ("short_output", varint(9) + lit(b"abcd"), 5, None),
        ("literal_4byte_len", varint(5) + bytes([63 << 2]) + b"\x04\x00\x00\x00abcde", 0, b"abcde"),
        ("literal_len_2_32", varint(5) + bytes([63 << 2]) + b"\xff\xff\xff\xffabcde", 2, None),
    ]

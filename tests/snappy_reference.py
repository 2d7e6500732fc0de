"""The reference's own snappy test inputs (deps/snappy/snappy_unittest.cc of the vendored
snappy 1.1.8), as data for tests/test_snappy.py (oracle) and tests/test_gpu_snappy.py (GPU).

  tests/golden/snappy/*     data files the reference's tests read from deps/snappy/testdata,
                            copied byte for byte (SHA256SUMS): the three corrupt streams
                            baddata{1,2,3}.snappy (snappy_unittest.cc:583-597) and the corpus
                            files of its `files[]` table (:1239-1252) — html, fireworks.jpeg,
                            paper-100k.pdf, alice29.txt, geo.protodata, kppkn.gtb (the larger
                            text files of that table are left out: same kind as alice29.txt);
  corruption_cases()        the hand-built streams of snappy_unittest.cc:531-569 and
                            :888-965, each with the verdict the reference's test requires.

TEST INFRASTRUCTURE: no product code reads this.
"""
import hashlib
import os

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "snappy")
CORPUS = ("html", "fireworks.jpeg", "paper-100k.pdf", "alice29.txt", "geo.protodata", "kppkn.gtb")
BADDATA = ("baddata1.snappy", "baddata2.snappy", "baddata3.snappy")


def read(name):
    with open(os.path.join(HERE, name), "rb") as f:
        return f.read()


def check_sums():
    """Every fixture matches the checksum recorded when it was copied."""
    with open(os.path.join(HERE, "SHA256SUMS")) as f:
        for line in f:
            digest, name = line.split()
            assert hashlib.sha256(read(name)).hexdigest() == digest, name


def corpus():
    return {n: read(n) for n in CORPUS}


def baddata():
    return {n: read(n) for n in BADDATA}


def varint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def corruption_cases(compress):
    """(name, stream, valid, expected output or None).  `compress` is snappy::Compress (the
    oracle's restatement): the first cases corrupt its output, as VerifyCorrupted does."""
    src = b"making sure we don't crash with corrupted input"
    d = bytearray(compress(src))
    assert len(d) > 3
    d[1] = (d[1] - 1) & 0xFF   # dest[1]--; dest[3]++  (snappy_unittest.cc:541-543)
    d[3] = (d[3] + 1) & 0xFF
    cases = [("verify_corrupted", bytes(d), False, None)]
    big = bytearray(compress(b"A" * 100000))
    big[0:4] = b"\x00\x00\x00\x00"   # the header lies: 0 bytes announced (:549-555)
    cases.append(("lying_header_zero", bytes(big), False, None))
    two_mb = bytearray(big)
    two_mb[0:4] = b"\xff\xff\xff\x00"   # announces about 2 MB (:576-580)
    cases.append(("lying_header_2mb", bytes(two_mb), False, None))
    cases += [
        ("truncated_varint", b"\xf0", False, None),                                   # :893-902
        ("unterminated_varint", b"\x80\x80\x80\x80\x80\x0a", False, None),            # :904-918
        ("overflowing_varint", b"\xfb\xff\xff\xff\x7f", False, None),                 # :920-932
        ("read_past_end_literal", varint(1) + bytes([0 << 2]) + b"x", True, b"x"),    # :934-946
        ("zero_offset_copy", b"\x40\x12\x00\x00", False, None),                       # :949-955
        ("zero_offset_copy_validation", b"\x05\x12\x00\x00", False, None),            # :957-962
    ]
    return cases

"""CPU tests of the snappy block-compression oracle (oracle/rr_snappy.c).

Pinning: the reference vendors snappy 1.1.8 (deps/snappy) but cannot be built or run here
(SURVEY.md §8c).  Two things pin the oracle:
  - the reference's own snappy test inputs (tests/snappy_reference.py): baddata{1,2,3}.snappy,
    the corruption cases of snappy_unittest.cc and the corpus files of its benchmark table;
  - pyarrow's bundled snappy (an independent, later release), which pins the FORMAT: every
    stream either side writes, the other decompresses to the input, and both accept / reject
    the same hand-built and mutated streams.
The compressor's exact bytes follow snappy 1.1.8's CompressFragment as restated from its source
(rr_snappy.c cites the lines); later snappy releases changed the match finder, so pyarrow's
compressed bytes differ from 1.1.8's on some inputs and are not used as the expected bytes:
compression bit-exactness against a run of 1.1.8 itself is unpinned, and the GPU compressor is
held bit-exact to the restatement.
"""
import numpy as np
import pytest

from oracle import cpu
from snappy_corpus import blocks, corpus, crafted

pa = pytest.importorskip("pyarrow")


def pa_compress(b):
    return pa.compress(b, codec="snappy", asbytes=True)


def pa_decompress(b, n):
    return pa.decompress(b, decompressed_size=n, codec="snappy", asbytes=True)


@pytest.mark.parametrize("name", sorted(corpus()))
def test_oracle_roundtrip_and_pyarrow_interop(name):
    x = corpus()[name]
    z = cpu.snappy_compress(x)
    assert len(z) <= cpu.lib().rrs_max_compressed(len(x))
    st, y = cpu.snappy_uncompress(z)
    assert st == 0 and y == x
    assert pa_decompress(z, len(x)) == x                  # our stream is valid snappy
    st, y = cpu.snappy_uncompress(pa_compress(x))         # theirs decodes here
    assert st == 0 and y == x


@pytest.mark.parametrize("name,stream,status,expected", crafted(), ids=[c[0] for c in crafted()])
def test_crafted_streams(name, stream, status, expected):
    st, y = cpu.snappy_uncompress(stream)
    assert st == status, (name, st)
    if status == 0:
        assert y == expected
        assert pa_decompress(stream, len(expected)) == expected
    elif status != 1:   # pyarrow needs a parsable length to try
        with pytest.raises(Exception):
            pa_decompress(stream, 1 << 20)


def test_mutated_streams_accept_reject_like_pyarrow():
    """Random byte flips of valid streams: the oracle accepts exactly the streams pyarrow's
    snappy accepts, with the same output."""
    rng = np.random.default_rng(7)
    c = corpus()
    agree = 0
    for name in ("text_150k", "markup_100k", "proto_120k", "blobs_cfg4_200k", "pattern_4"):
        z = bytearray(cpu.snappy_compress(c[name][:6000]))
        for _ in range(60):
            m = bytearray(z)
            for _ in range(int(rng.integers(1, 4))):
                m[int(rng.integers(len(m)))] = int(rng.integers(256))
            st, y = cpu.snappy_uncompress(bytes(m))
            ln = cpu.lib().rrs_uncompressed_length
            try:
                ref = pa.decompress(bytes(m), decompressed_size=len(y) if st == 0 else 6000, codec="snappy", asbytes=True)
                ok = True
            except Exception:
                ok = False
            if st == 0:
                assert ok and ref == y, name
            else:
                # pyarrow is handed a size it cannot produce (6000 != announced) or a bad stream
                hdr_ok = st != 1
                if hdr_ok and ok:
                    # it decoded: then the announced length must be 6000 and our status is a real reject
                    raise AssertionError(f"{name}: oracle status {st} but pyarrow decoded")
            agree += 1
    assert agree == 300


def test_block_batches_match_single_calls():
    c = corpus()
    buf = c["text_150k"] + c["blobs_cfg4_200k"]
    cuts = np.array(blocks(buf, 16384), np.uint64)
    data = np.frombuffer(buf, np.uint8)
    packed, coffs, _ = cpu.snappy_compress_blocks(data, cuts, nthreads=4)
    for i in range(len(cuts) - 1):
        one = cpu.snappy_compress(buf[int(cuts[i]):int(cuts[i + 1])])
        assert packed[int(coffs[i]):int(coffs[i + 1])].tobytes() == one
    out, st, _ = cpu.snappy_uncompress_blocks(packed, coffs, cuts, nthreads=4)
    assert not st.any() and out.tobytes() == buf


def test_compressor_properties():
    """What CompressFragment guarantees whatever the data: 64 KiB fragments compress
    independently (no copy reaches across a fragment), copies never exceed 64 bytes, offsets
    stay below 65536 (no copy-4 tag), the output fits MaxCompressedLength."""
    c = corpus()
    for name in ("text_150k", "random_120k", "long_run", "zeros_100k"):
        x = c[name]
        z = cpu.snappy_compress(x)
        i = 0
        while z[i] & 0x80:
            i += 1
        i += 1
        pos = 0
        while i < len(z):
            t = z[i]
            if t & 3 == 0:
                n = (t >> 2) + 1
                if n >= 61:
                    k = n - 60
                    n = int.from_bytes(z[i + 1:i + 1 + k], "little") + 1
                    i += k
                i += 1 + n
                pos += n
            else:
                assert t & 3 != 3, "copy-4 tag"
                if t & 3 == 1:
                    ln, off = 4 + ((t >> 2) & 7), ((t >> 5) << 8) | z[i + 1]
                    i += 2
                else:
                    ln, off = (t >> 2) + 1, z[i + 1] | (z[i + 2] << 8)
                    i += 3
                assert ln <= 64 and 0 < off < 65536
                assert (pos - off) // 65536 == pos // 65536, "copy crosses a fragment"
                pos += ln
        assert pos == len(x)


# ---- the reference's own snappy test inputs (tests/snappy_reference.py) ---------------------
import snappy_reference as sref  # noqa: E402


def test_reference_fixture_checksums():
    sref.check_sums()


@pytest.mark.parametrize("name", sref.BADDATA)
def test_reference_baddata_rejected_with_sane_length(name):
    """snappy_unittest.cc:583-597: the length preamble either fails or stays under 1 MiB, and
    the stream is rejected (by the oracle and by pyarrow's independent snappy)."""
    z = sref.baddata()[name]
    st, ln = cpu.snappy_length(z)
    assert st != 0 or ln < (1 << 20)
    st, _ = cpu.snappy_uncompress(z)
    assert st != 0
    with pytest.raises(Exception):
        pa_decompress(z, ln if st == 0 or ln else 1 << 20)


def test_reference_corruption_cases():
    """snappy_unittest.cc:531-580 (VerifyCorrupted) and :888-965 (truncated, unterminated and
    overflowing varints, a literal ending the buffer, zero-offset copies): the verdict each
    test requires, from the oracle and from pyarrow."""
    for name, stream, valid, expected in sref.corruption_cases(cpu.snappy_compress):
        st, y = cpu.snappy_uncompress(stream)
        assert (st == 0) == valid, (name, st)
        if valid:
            assert y == expected, name
            assert pa_decompress(stream, len(expected)) == expected
        else:
            lst, ln = cpu.snappy_length(stream)
            with pytest.raises(Exception):
                pa_decompress(stream, ln if lst == 0 and ln < (1 << 24) else 1 << 20)


@pytest.mark.parametrize("name", sref.CORPUS)
def test_reference_corpus_roundtrip(name):
    """The files of snappy_unittest.cc's corpus table (:1239-1252): whole-file and RocksDB
    16 KiB block streams decompress to the input here and under pyarrow, and pyarrow's
    streams decompress here."""
    x = sref.corpus()[name]
    cuts = blocks(x, 16384)
    for part in [x] + [x[a:b] for a, b in zip(cuts[:-1], cuts[1:])]:
        z = cpu.snappy_compress(part)
        st, y = cpu.snappy_uncompress(z)
        assert st == 0 and y == part
        assert pa_decompress(z, len(part)) == part
        st, y = cpu.snappy_uncompress(pa_compress(part))
        assert st == 0 and y == part

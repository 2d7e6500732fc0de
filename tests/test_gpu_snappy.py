"""GPU parity of the snappy block compression (include/rr_snappy.h)
against the CPU restatement (oracle/rr_snappy.c), through the C-ABI: compressed bytes
bit-identical to the oracle's, decompressed bytes and per-block statuses identical, on the
synthetic corpus, RocksDB-sized 16 KiB blocks of the engine's own value blobs, blocks of every
edge size, blocks longer than the LDS paths, hand-built and mutated streams, and a full
1M-value batch."""
import numpy as np
import pytest
import torch

import redrock_old_amd as rr
from oracle import cpu
from snappy_corpus import blocks, corpus, crafted

pytestmark = pytest.mark.gpu


def pack(bufs):
    offs = np.zeros(len(bufs) + 1, np.uint64)
    for i, b in enumerate(bufs):
        offs[i + 1] = offs[i] + len(b)
    raw = b"".join(bufs)
    data = np.zeros(((len(raw) + 15) & ~15) or 16, np.uint8)
    data[:len(raw)] = np.frombuffer(raw, np.uint8) if raw else data[:0]
    return data, offs


def oracle_compress(bufs):
    return [cpu.snappy_compress(b) for b in bufs]


def check_compress(engine, bufs, what):
    data, offs = pack(bufs)
    got, goffs = engine.snappy_compress_host(data, offs)
    want = oracle_compress(bufs)
    for i, w in enumerate(want):
        g = got[int(goffs[i]):int(goffs[i + 1])].tobytes()
        assert g == w, f"{what}: block {i} ({len(bufs[i])} B) differs: {len(g)} vs {len(w)} bytes"
    return got, goffs


def check_decompress(engine, streams, what, cap=None):
    data, offs = pack(streams)
    want = [cpu.snappy_uncompress(s) for s in streams]
    total = sum(cpu.snappy_length(s)[1] for s in streams)
    out, ooffs, st = engine.snappy_decompress_host(data, offs, cap if cap is not None else total)
    for i, (wst, wout) in enumerate(want):
        assert int(st[i]) == wst, f"{what}: block {i} status {rr.SNAPPY_STATUS[int(st[i])]} vs {rr.SNAPPY_STATUS[wst]}"
        if wst == 0:
            assert out[int(ooffs[i]):int(ooffs[i + 1])].tobytes() == wout, f"{what}: block {i} output differs"
    return out, ooffs, st


def test_compress_corpus_bit_exact(engine):
    c = corpus()
    names = sorted(c)
    check_compress(engine, [c[k] for k in names], "corpus")


def test_compress_rocksdb_blocks_bit_exact(engine):
    c = corpus()
    for name in ("text_150k", "markup_100k", "proto_120k", "random_120k", "blobs_cfg4_200k", "zeros_100k"):
        buf = c[name]
        cuts = blocks(buf, 16384)
        check_compress(engine, [buf[cuts[i]:cuts[i + 1]] for i in range(len(cuts) - 1)], name)


def test_compress_edge_sizes(engine):
    """Every size around the compressor's thresholds: below / at kInputMarginBytes (15), the
    LDS stage limit of the GPU fragment path, the 64 KiB fragment size."""
    base = corpus()["text_150k"] + corpus()["random_120k"]
    sizes = list(range(0, 40)) + [255, 256, 257, 4095, 4096, 4097, 16383, 16384, 16385, 16439, 16440, 16441, 16448,
                                  16449, 32768, 65535, 65536, 65537, 131072, 131073]
    check_compress(engine, [base[:s] for s in sizes], "edge sizes")
    check_compress(engine, [base[1:1 + s] for s in sizes], "edge sizes, odd alignment")


def test_decompress_corpus_and_blocks(engine):
    c = corpus()
    streams = [cpu.snappy_compress(c[k]) for k in sorted(c)]
    import pyarrow as pa
    streams += [pa.compress(c[k], codec="snappy", asbytes=True) for k in sorted(c)]   # another snappy's streams
    check_decompress(engine, streams, "corpus")
    buf = c["blobs_cfg4_200k"] + c["text_150k"]
    cuts = blocks(buf, 16384)
    check_decompress(engine, [cpu.snappy_compress(buf[cuts[i]:cuts[i + 1]]) for i in range(len(cuts) - 1)], "blocks")


def test_decompress_crafted(engine):
    cases = crafted()
    check_decompress(engine, [s for _, s, _, _ in cases], "crafted")


def test_decompress_mutated(engine):
    """400 mutated streams a round (1-3 random bytes overwritten in five corpus streams): every
    status and output equal to the oracle's.  RR_FUZZ_ROUNDS=k runs k seeds (an extended run)."""
    import os
    for k in range(int(os.environ.get("RR_FUZZ_ROUNDS", "1"))):
        _mutated_round(engine, 11 + 7919 * k)


def _mutated_round(engine, seed):
    rng = np.random.default_rng(seed)
    c = corpus()
    streams = []
    for name in ("text_150k", "markup_100k", "blobs_cfg4_200k", "pattern_4", "zeros_100k"):
        z = cpu.snappy_compress(c[name][:40000])
        for _ in range(80):
            m = bytearray(z)
            for _ in range(int(rng.integers(1, 4))):
                m[int(rng.integers(len(m)))] = int(rng.integers(256))
            streams.append(bytes(m))
    # a preamble the mutation made huge would need gigabytes: cap the output and compare only
    # the blocks that fit (the rest must be CAPACITY)
    keep = []
    for s in streams:
        st, _ = cpu.snappy_uncompress(s, cap=1 << 20)
        ok = st != 6
        if ok:
            keep.append(s)
    check_decompress(engine, keep, "mutated")


def test_decompress_capacity(engine):
    c = corpus()
    streams = [cpu.snappy_compress(c["text_150k"][:10000]) for _ in range(4)]
    data, offs = pack(streams)
    d_data = torch.from_numpy(data).cuda()
    d_offs = torch.from_numpy(offs.view(np.int64)).cuda()
    d_out = torch.zeros(25000, dtype=torch.uint8, device="cuda")
    d_oo = torch.zeros(5, dtype=torch.int64, device="cuda")
    d_st = torch.zeros(4, dtype=torch.uint8, device="cuda")
    engine.snappy_decompress_device(d_data, d_offs, d_out, d_oo, d_st)
    torch.cuda.synchronize()
    assert d_st.cpu().tolist() == [0, 0, 6, 6]
    assert d_out[:20000].cpu().numpy().tobytes() == c["text_150k"][:10000] * 2


def test_large_blocks_global_paths(engine):
    """Blocks whose output exceeds the 32 KiB LDS window decompress straight to global memory
    (copies read back through the L2); the copy-4 stream reaches back 100 KB."""
    c = corpus()
    streams = [cpu.snappy_compress(c[k]) for k in ("text_150k", "markup_100k", "long_run", "zeros_100k")]
    streams.append([s for n, s, _, _ in crafted() if n == "four_byte_offset"][0])
    check_decompress(engine, streams, "large blocks")


def test_device_entry_full_batch_roundtrip(engine):
    """The 1M-value config-4 batch as 16 KiB blocks through the device entry points:
    compressed bytes equal the oracle's (multi-threaded), decompression restores the blobs."""
    data, offs = rr.gen_batch(4, 1_000_000)
    nb = int(offs[-1])
    cuts = np.arange(0, nb, 16384, dtype=np.uint64)
    cuts = np.append(cuts, np.uint64(nb))
    n = len(cuts) - 1
    want, woffs, _ = cpu.snappy_compress_blocks(data[:nb], cuts, nthreads=min(16, cpu.nprocs()))
    d_data = torch.from_numpy(data).cuda()
    d_offs = torch.from_numpy(cuts.view(np.int64)).cuda()
    cap = int(rr.lib().rr_snappy_compress_bound(n, d_data.numel()))
    d_comp = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    d_coffs = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    engine.snappy_compress_device(d_data, d_offs, d_comp, d_coffs)
    torch.cuda.synchronize()
    coffs = d_coffs.cpu().numpy().view(np.uint64)
    assert np.array_equal(coffs, woffs)
    assert np.array_equal(d_comp[:int(coffs[-1])].cpu().numpy(), want)
    d_back = torch.zeros(((nb + 15) & ~15), dtype=torch.uint8, device="cuda")
    d_boffs = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    d_st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    engine.snappy_decompress_device(d_comp, d_coffs, d_back, d_boffs, d_st)
    torch.cuda.synchronize()
    assert int(d_st.max().item()) == 0
    assert np.array_equal(d_boffs.cpu().numpy().view(np.uint64), cuts)
    assert torch.equal(d_back[:nb], d_data[:nb])


# ---- the reference's own snappy test inputs (tests/snappy_reference.py) ---------------------
import snappy_reference as sref  # noqa: E402


def test_reference_corpus_files(engine):
    """The files of snappy_unittest.cc's corpus table (:1239-1252), whole and as RocksDB 16 KiB
    blocks: GPU compression bit-exact with the 1.1.8 restatement, GPU decompression of those
    streams and of pyarrow's restores the files."""
    import pyarrow as pa
    c = sref.corpus()
    whole = [c[k] for k in sref.CORPUS]
    check_compress(engine, whole, "reference corpus")
    parts = []
    for x in whole:
        cuts = blocks(x, 16384)
        parts += [x[a:b] for a, b in zip(cuts[:-1], cuts[1:])]
    check_compress(engine, parts, "reference corpus blocks")
    streams = [cpu.snappy_compress(x) for x in whole + parts]
    streams += [pa.compress(x, codec="snappy", asbytes=True) for x in whole]
    check_decompress(engine, streams, "reference corpus streams")


def test_reference_baddata_and_corruption(engine):
    """baddata{1,2,3}.snappy (snappy_unittest.cc:583-597) and the corruption cases
    (:531-580, :888-965): the GPU decompressor gives the oracle's status for every stream (a
    rejection wherever the reference's test requires one) and the literal case's bytes."""
    bad = list(sref.baddata().values())
    cases = sref.corruption_cases(cpu.snappy_compress)
    streams = bad + [s for _, s, _, _ in cases]
    for z in bad:
        st, ln = cpu.snappy_length(z)
        assert st != 0 or ln < (1 << 20)
    # (output slots as every preamble announces: the largest lie here is ~2 MB)
    assert sum(cpu.snappy_length(s)[1] for s in streams) < (8 << 20)
    _, _, st = check_decompress(engine, streams, "reference bad streams")
    verdicts = [int(x) == 0 for x in st]
    assert verdicts[:3] == [False, False, False]
    assert verdicts[3:] == [v for _, _, v, _ in cases]


def _lit(b):
    """A literal tag with its bytes (snappy format: lengths <= 60 in the tag byte, else 1-2 more)."""
    n = len(b)
    if n <= 60:
        return bytes([(n - 1) << 2]) + b
    if n <= 256:
        return bytes([60 << 2, n - 1]) + b
    return bytes([61 << 2, (n - 1) & 0xFF, (n - 1) >> 8]) + b


def _copy1(length, off):   # 1-byte-offset copy: 4 <= length <= 11, off < 2048
    return bytes([1 | ((length - 4) << 2) | ((off >> 8) << 5), off & 0xFF])


def _varint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def test_consecutive_literals(engine):
    """Streams with literal after literal (valid snappy that snappy's own compressor never writes):
    a long literal's last dword may spill past its end in the LDS path, so the literal after it
    must land after the spill. Every length mod 4 and every destination alignment, against the
    oracle."""
    rng = np.random.default_rng(7)
    streams = []
    for a in range(4):   # destination alignment of the long literal
        for la in range(65, 73):   # long literal lengths: every value mod 4 (and mod 8)
            for lb in (1, 2, 3, 5, 17, 64, 65, 70):
                parts, out = [], b""
                if a:
                    x = rng.integers(0, 256, a, dtype=np.uint8).tobytes()
                    parts.append(_lit(x)); out += x
                for n_ in (la, lb, la + 3, 7):
                    x = rng.integers(0, 256, n_, dtype=np.uint8).tobytes()
                    parts.append(_lit(x)); out += x
                parts.append(_copy1(8, 5)); out += bytes(out[len(out) - 5 + (i % 5)] for i in range(8))
                x = rng.integers(0, 256, 90, dtype=np.uint8).tobytes()
                parts.append(_lit(x)); out += x
                s = _varint(len(out)) + b"".join(parts)
                assert cpu.snappy_uncompress(s) == (0, out)
                streams.append(s)
    check_decompress(engine, streams, "consecutive literals")

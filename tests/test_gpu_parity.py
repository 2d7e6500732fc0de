"""GPU parity tests: the HIP engine, called through the C-ABI, against the CPU oracle and the
golden vectors.  Bit-exact everywhere (integer/byte work).  One process, one engine context."""
import struct

import numpy as np
import pytest

import redrock_old_amd as rr
from oracle import cpu
from oracle import pyoracle as po

from helpers import assert_flat_equal, batch_from_blobs, expected_flat, golden, structured_mutations

pytestmark = pytest.mark.gpu
G = golden()


def reencoded(blob):
    return blob[:1] + struct.pack("<I", struct.unpack_from("<I", blob, 1)[0] & 0xFFFFFF) + blob[5:]


def test_golden_batch(engine):
    fx = G["kats"] + G["edges"]
    blobs = [bytes.fromhex(f["blob"]) for f in fx]
    data, offs = batch_from_blobs(blobs)
    v, e, a, t = engine.decode_host(data, offs)
    assert_flat_equal((v, e), expected_flat(fx), "golden")
    assert np.array_equal(a, data[:int(offs[-1])])
    nbad = sum(1 for f in fx if f["value"].get("status", 0))
    assert t["n_bad"] == nbad
    ok = np.nonzero(v["status"] == 0)[0]
    # encode the OK values only (bad values own no descriptors and are not encodable)
    out, ooffs, t2 = engine.encode_host(v[ok], e, a)
    assert t2["n_bad"] == 0
    exp = b"".join(reencoded(bytes.fromhex(fx[i].get("reencoded", fx[i]["blob"]))) for i in ok)
    assert bytes(out) == exp


def test_reference_shaped_values(engine):
    """ziplist.c:1255-1281's test lists and testredrock/test_redrock.py's value of every type
    (a 6,890-B string, a 100-int List, a 1000-member HT Set, a 1000 x 190-B HT Hash, a 100-member
    ziplist ZSet, a geo zset, an HLL string), each repeated so they share windows with each other
    and with the golden fixtures: the GPU decode equals the literal flat forms (the 1000-key
    tables go through the exact duplicate test of the fixup pass), and the encode rewrites them."""
    fx = (G["shapes"] + G["kats"]) * 7
    blobs = [bytes.fromhex(f["blob"]) for f in fx]
    data, offs = batch_from_blobs(blobs)
    v, e, a, t = engine.decode_host(data, offs)
    assert_flat_equal((v, e), expected_flat(fx), "reference shapes")
    assert t["n_bad"] == 0
    out, ooffs, t2 = engine.encode_host(v, e, a)
    assert t2["n_bad"] == 0 and bytes(out) == b"".join(blobs)


@pytest.mark.parametrize("cfg,n", [(1, 100000), (2, 100000), (3, 50000), (4, 100000), (10, 2400), (11, 400)])
def test_config_parity(engine, cfg, n):
    data, offs = rr.gen_batch(cfg, n)
    v, e, a, t = engine.decode_host(data, offs)
    ov, oe, oa, ot = cpu.decode(data, offs, nthreads=8)
    assert_flat_equal((v, e), (ov, oe), f"config {cfg}")
    assert np.array_equal(a, oa)
    assert t == ot
    out, ooffs, t2 = engine.encode_host(v, e, a)
    assert np.array_equal(ooffs, offs)
    assert np.array_equal(out, data[:int(offs[-1])])
    assert t2["n_bad"] == 0 and t2["bytes"] == int(offs[-1]) and t2["n_elems"] == t["n_elems"]
    assert t2["payload"] == t["payload"]


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 127, 128, 129, 4097])
def test_ragged_batch_sizes(engine, n):
    data, offs = rr.gen_batch(4, n, seed=1000 + n)
    v, e, a, t = engine.decode_host(data, offs)
    ov, oe, oa, ot = cpu.decode(data, offs)
    assert_flat_equal((v, e), (ov, oe), f"n={n}")
    out, ooffs, _ = engine.encode_host(v, e, a)
    assert np.array_equal(out, data[:int(offs[-1])])


def _int_like_strings(rng, n):
    """Strings near string2ll's accept/reject boundaries: every length 0..24, signs, leading
    zeros, int64 limits +-1, and stray non-digit bytes at random positions."""
    out = [s.encode() for s, _ in G["string2ll"]]
    for lim in (2**63 - 1, 2**63, 2**63 + 1, 10**18, 10**19 - 1, 10**19, 2**31, 2**24, 10**7, 10**14):
        for d in (-1, 0, 1):
            out += [str(lim + d).encode(), b"-" + str(lim + d).encode()]
    for _ in range(n):
        ln = int(rng.integers(0, 25))
        s = bytearray(rng.integers(ord("0"), ord("9") + 1, size=ln).astype(np.uint8).tobytes())
        r = rng.random()
        if ln and r < 0.3:
            s[0] = ord("-")
        if ln > 1 and rng.random() < 0.1:
            s[int(rng.integers(0, ln))] = int(rng.integers(0, 256))
        if ln > 1 and rng.random() < 0.1:
            s[1 if s[0] == ord("-") else 0] = ord("0")
        out.append(bytes(s))
    return out


def test_list_integer_parsing(engine):
    """List elements go through zipTryEncoding + string2ll (ziplist.c:480, util.c:360): the
    GPU's integer/string decision and value must equal the oracle's for every element."""
    rng = np.random.default_rng(11)
    items = _int_like_strings(rng, 6000)
    blobs = []
    for k in range(0, len(items), 16):
        b = bytes([14]) + struct.pack("<I", k & 0xFFFFFF)
        for it in items[k:k + 16]:
            b += struct.pack("<I", len(it)) + it
        blobs.append(b)
    data, offs = batch_from_blobs(blobs)
    v, e, a, t = engine.decode_host(data, offs)
    ov, oe, oa, ot = cpu.decode(data, offs)
    assert t == ot and t["n_bad"] == 0
    assert_flat_equal((v, e), (ov, oe), "list ints")
    out, ooffs, t2 = engine.encode_host(v, e, a)
    assert t2["n_bad"] == 0
    assert np.array_equal(out, data[:int(offs[-1])])


def test_list_counts_staged_and_far(engine):
    """count_kernel walks a List's length chain from an LDS stage of 4 KiB a wave (Lists packed
    in lane order, several packs a wave) and walks longer Lists from global memory: Lists from
    empty to ~40 KiB, truncated and overlong length fields, dense runs of Lists that take several
    packs, all interleaved with strings — records and descriptors equal the oracle's."""
    rng = np.random.default_rng(31)
    blobs = []
    for i in range(3000):
        r = rng.random()
        if r < 0.25:
            blobs.append(bytes([0, 1, 0, 0, 0, 0]) + rng.integers(0, 256, int(rng.integers(0, 80))).astype(np.uint8).tobytes())
            continue
        k = int(rng.integers(0, 40)) if r < 0.9 else int(rng.integers(200, 2000))
        b = bytes([14]) + struct.pack("<I", i & 0xFFFFFF)
        for _ in range(k):
            it = rng.integers(ord("a"), ord("z") + 1, int(rng.integers(0, 24))).astype(np.uint8).tobytes()
            b += struct.pack("<I", len(it)) + it
        m = rng.random()
        if m < 0.03 and len(b) > 9:
            b = b[:-int(rng.integers(1, 4))]                               # cut inside the last element
        elif m < 0.06 and k:
            b = b[:5] + struct.pack("<I", 0xFFFFFFF0) + b[9:]              # first length past the value
        blobs.append(b)
    data, offs = batch_from_blobs(blobs)
    v, e, a, t = engine.decode_host(data, offs)
    ov, oe, oa, ot = cpu.decode(data, offs)
    assert t == ot
    assert_flat_equal((v, e), (ov, oe), "lists staged / far")


def test_empty_batch(engine):
    v, e, a, t = engine.decode_host(np.zeros(16, np.uint8), np.zeros(1, np.uint64))
    assert len(v) == 0 and t["n_elems"] == 0 and t["n_bad"] == 0


def test_decode_capacity(engine):
    data, offs = rr.gen_batch(4, 3000)
    cap = 5000
    v, e, a, t = engine.decode_host(data, offs, elem_cap=cap)
    ov, oe, oa, ot = cpu.decode(data, offs, elem_cap=cap)
    assert t == ot and t["n_bad"] > 0
    # descriptors are written only below the first value that did not fit
    first = int(np.nonzero(ov["status"] == 11)[0][0])
    w = int(ov["elem_base"][first])
    assert_flat_equal((v, e[:w]), (ov, oe[:w]), "capacity")


def test_encode_capacity(engine):
    data, offs = rr.gen_batch(4, 3000)
    v, e, a, t = engine.decode_host(data, offs)
    cap = int(offs[1500])
    out, ooffs, t2 = engine.encode_host(v, e, a, data_cap=cap)
    assert np.array_equal(ooffs, offs)            # offsets are always complete
    assert t2["bytes"] == int(offs[-1]) and t2["n_bad"] > 0
    fits = int(np.searchsorted(offs[1:], cap, side="right"))
    assert np.array_equal(out[:int(offs[fits])], data[:int(offs[fits])])


def test_fuzzed_blobs_match_oracle(engine):
    """Random byte flips / truncations of valid blobs: statuses and descriptors must match the
    oracle value for value (no out-of-bounds reads: the kernel must survive every input)."""
    rng = np.random.default_rng(7)
    data, offs = rr.gen_batch(10, 480)
    blobs = []
    for i in range(len(offs) - 1):
        b = bytearray(data[offs[i]:offs[i + 1]].tobytes())
        for _ in range(4):
            m = bytearray(b)
            r = rng.integers(0, 4)
            if r == 0 and len(m):
                m[rng.integers(0, len(m))] ^= 1 << int(rng.integers(0, 8))
            elif r == 1 and len(m):
                m = m[:int(rng.integers(0, len(m)))]
            elif r == 2 and len(m) > 6:
                p = int(rng.integers(5, len(m)))
                m[p] = int(rng.integers(0, 256))
            blobs.append(bytes(m))
    fdata, foffs = batch_from_blobs(blobs)
    v, e, a, t = engine.decode_host(fdata, foffs)
    ov, oe, oa, ot = cpu.decode(fdata, foffs)
    assert_flat_equal((v, e), (ov, oe), "fuzz")
    assert t == ot


def test_device_api_matches_host_api(engine):
    import torch
    data, offs = rr.gen_batch(4, 20000)
    n = len(offs) - 1
    nb = int(offs[-1])
    dev = torch.device("cuda:0")
    d_data = torch.from_numpy(data).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    cap = rr.elem_bound(n, nb)
    d_vals = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    d_elems = torch.zeros(cap * 16, dtype=torch.uint8, device=dev)
    d_arena = torch.zeros((nb + 15) & ~15, dtype=torch.uint8, device=dev)
    d_tot = torch.zeros(4, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream()
    engine.decode_device(d_data, d_offs, d_vals, d_elems, d_arena, d_tot, stream=s)
    torch.cuda.synchronize()
    tot = d_tot.cpu().numpy().view(np.uint64)
    v = d_vals.cpu().numpy().view(rr.VALUE_DT)
    e = d_elems.cpu().numpy().view(rr.ELEM_DT)[:int(tot[0])]
    hv, he, ha, ht = engine.decode_host(data, offs)
    assert_flat_equal((v, e), (hv, he), "device api")
    assert int(tot[0]) == ht["n_elems"] and int(tot[3]) == ht["payload"]
    # device encode back into a second buffer
    d_out = torch.zeros((nb + 15) & ~15, dtype=torch.uint8, device=dev)
    d_ooffs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    engine.encode_device(d_vals, d_elems, d_arena, d_out, d_ooffs, d_tot, stream=s)
    torch.cuda.synchronize()
    assert np.array_equal(d_ooffs.cpu().numpy().view(np.uint64), offs)
    assert torch.equal(d_out[:nb], d_data[:nb])


def test_sums_zero_between_calls():
    """The window/group sums live in a context buffer that must be zero on entry: decode_kernel's
    last workgroup (encode: E3's last block) zeroes what its call used.  Calls of changing sizes
    on one fresh context — growing, shrinking, decode and encode interleaved, repeated on the
    device API — each equal the oracle (a sum left over from an earlier call would shift every
    later window's descriptor slots)."""
    eng = rr.Engine(0)
    try:
        for cfg, n in [(4, 30000), (1, 200000), (4, 5000), (3, 20000), (4, 30000), (2, 90000), (4, 5000)]:
            data, offs = rr.gen_batch(cfg, n, seed=77 + n)
            v, e, a, t = eng.decode_host(data, offs)
            ov, oe, oa, ot = cpu.decode(data, offs, nthreads=8)
            assert_flat_equal((v, e), (ov, oe), f"config {cfg} n={n}")
            assert t == ot
            out, ooffs, t2 = eng.encode_host(v, e, a)
            assert np.array_equal(ooffs, offs) and np.array_equal(out, data[:int(offs[-1])])
            assert t2["n_elems"] == t["n_elems"] and t2["payload"] == t["payload"]
    finally:
        eng.close()


def test_graph_replay_decode_encode():
    """Decode + encode captured in a HIP graph (torch.cuda.CUDAGraph) after rr_ctx_reserve, then
    replayed: no zeroing launch runs, so every replay relies on the previous one's kernels having
    left the sums zero.  Each replay's records, descriptors and re-encoded blobs equal the host
    path's; replays over a second batch copied into the same input buffers as well."""
    import torch
    dev = torch.device("cuda:0")
    eng = rr.Engine(0)
    try:
        data, offs = rr.gen_batch(4, 30000, seed=4242)
        n = len(offs) - 1
        data3, offs3 = rr.gen_batch(1, n, seed=4244)   # (replayed later through the same buffers)
        nb = (max(int(offs[-1]), int(offs3[-1])) + 15) & ~15
        cap = max(rr.elem_bound(n, int(offs[-1])), rr.elem_bound(n, int(offs3[-1])))
        d_data = torch.zeros(nb, dtype=torch.uint8, device=dev)
        d_offs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        d_vals = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
        d_elems = torch.zeros(cap * 16, dtype=torch.uint8, device=dev)
        d_arena = torch.zeros(nb, dtype=torch.uint8, device=dev)
        d_tot = torch.zeros(4, dtype=torch.int64, device=dev)
        d_out = torch.zeros(nb, dtype=torch.uint8, device=dev)
        d_ooffs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        d_tot2 = torch.zeros(4, dtype=torch.int64, device=dev)
        eng.reserve(n, nb)

        def load(dd, oo):
            d_data.zero_()
            d_data[:dd.size].copy_(torch.from_numpy(dd))
            d_offs.copy_(torch.from_numpy(oo.view(np.int64)))

        def check(dd, oo):
            hv, he, ha, ht = eng.decode_host(dd, oo)
            tot = d_tot.cpu().numpy().view(np.uint64)
            v = d_vals.cpu().numpy().view(rr.VALUE_DT)
            e = d_elems.cpu().numpy().view(rr.ELEM_DT)[:int(tot[0])]
            assert_flat_equal((v, e), (hv, he), "graph replay")
            assert int(tot[0]) == ht["n_elems"] and int(tot[3]) == ht["payload"]
            assert np.array_equal(d_ooffs.cpu().numpy().view(np.uint64), oo)
            m = int(oo[-1])
            assert torch.equal(d_out[:m], d_data[:m])

        load(data, offs)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):   # (one eager call first, as torch's capture recipe asks)
            eng.decode_device(d_data, d_offs, d_vals, d_elems, d_arena, d_tot, stream=s)
            eng.encode_device(d_vals, d_elems, d_arena, d_out, d_ooffs, d_tot2, stream=s)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            cs = torch.cuda.current_stream()
            eng.decode_device(d_data, d_offs, d_vals, d_elems, d_arena, d_tot, stream=cs)
            eng.encode_device(d_vals, d_elems, d_arena, d_out, d_ooffs, d_tot2, stream=cs)
        for _ in range(3):
            d_vals.zero_(); d_elems.zero_(); d_out.zero_()
            g.replay()
            torch.cuda.synchronize()
            check(data, offs)
        # the graph's launches are sized by the first batch's n: a second batch of the same count
        # through the same buffers (config 1 values, fewer bytes: other windows, other sums)
        load(data3, offs3)
        for _ in range(2):
            g.replay()
            torch.cuda.synchronize()
            check(data3, offs3)
    finally:
        eng.close()


@pytest.mark.parametrize("cfg", [4, 3, 2])
def test_full_size_mixed_roundtrip(engine, cfg):
    """1M-value batches at BASELINE.json's sizes (config 4 mixed = the headline, config 3 Hash
    ziplists, config 2 Zipf Strings): records and descriptors equal the oracle's, zero bad
    values, and encode(decode(b)) == b byte for byte on the GPU."""
    import torch
    data, offs = rr.gen_batch(cfg, 1_000_000)
    n = len(offs) - 1
    nb = int(offs[-1])
    dev = torch.device("cuda:0")
    d_data = torch.from_numpy(data).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    cap = rr.elem_bound(n, nb)
    d_vals = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    d_elems = torch.zeros(cap * 16, dtype=torch.uint8, device=dev)
    d_arena = torch.zeros((nb + 15) & ~15, dtype=torch.uint8, device=dev)
    d_tot = torch.zeros(4, dtype=torch.int64, device=dev)
    engine.decode_device(d_data, d_offs, d_vals, d_elems, d_arena, d_tot)
    torch.cuda.synchronize()
    tot = d_tot.cpu().numpy().view(np.uint64)
    assert int(tot[2]) == 0
    ov, oe, _, ot = cpu.decode(data, offs, nthreads=8)
    assert int(tot[0]) == ot["n_elems"] and int(tot[3]) == ot["payload"]
    v = d_vals.cpu().numpy().view(rr.VALUE_DT)
    assert np.array_equal(v, ov)
    e = d_elems.cpu().numpy().view(rr.ELEM_DT)[:int(tot[0])]
    assert np.array_equal(e, oe)
    d_out = torch.zeros((nb + 15) & ~15, dtype=torch.uint8, device=dev)
    d_ooffs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    engine.encode_device(d_vals, d_elems, d_arena, d_out, d_ooffs, d_tot)
    torch.cuda.synchronize()
    assert torch.equal(d_out[:nb], d_data[:nb])
    assert np.array_equal(d_ooffs.cpu().numpy().view(np.uint64), offs)


def _ht_blob(t, members, lru=7):
    n = len(members) if t == rr.T_SET_HT else len(members) // 2
    return bytes([t]) + struct.pack("<I", lru) + struct.pack("<Q", n) + b"".join(
        struct.pack("<Q", len(m)) + m for m in members)


def _sl_blob(pairs, lru=9):
    return bytes([rr.T_ZSET_SKIPLIST]) + struct.pack("<I", lru) + struct.pack("<Q", len(pairs)) + b"".join(
        struct.pack("<Q", len(m)) + m + (s if isinstance(s, bytes) else struct.pack("<d", s)) for m, s in pairs)


def _fixup_blobs(rng):
    """Blobs for the fixup pass (fixup_kernel): hash tables with repeated keys below and above the
    in-register fingerprint limit (16 keys) and past one LDS table pass (2048 keys), skiplists
    out of serZset's order, with tied scores, -0.0 / 0.0 ties, repeated members and NaN."""
    def word(lo, hi):
        return rng.integers(97, 123, int(rng.integers(lo, hi + 1)), dtype=np.uint8).tobytes()
    B = []
    for n, ndup in ((5, 2), (16, 1), (16, 0), (17, 3), (40, 10), (300, 0), (3000, 400), (9000, 50)):
        base = [word(0, 24) + str(i).encode() for i in range(n - ndup)]
        mem = list(base)
        for _ in range(ndup):
            mem.insert(int(rng.integers(0, len(mem) + 1)), base[int(rng.integers(0, len(base)))])
        B.append(_ht_blob(rr.T_SET_HT, mem))
    B.append(_ht_blob(rr.T_SET_HT, [b""] * 5 + [b"x"]))
    B.append(_ht_blob(rr.T_SET_HT, [b"same-prefix-0123456789-" + bytes([65 + i % 3]) for i in range(30)]))
    for n, dup_at in ((4, None), (8, 7), (16, 15), (16, None), (40, 39), (200, 3), (2600, 2599), (2600, None)):
        fields = [b"f%05d" % i for i in range(n)]
        if dup_at is not None:
            fields[dup_at] = fields[int(rng.integers(0, dup_at))]
        mem = []
        for f in fields:
            mem += [f, word(0, 40)]
        B.append(_ht_blob(rr.T_HASH_HT, mem))
    B.append(_ht_blob(rr.T_HASH_HT, [b"a", b"v", b"b", b"v", b"c", b"v"]))   # repeated values only
    for n in (2, 3, 16, 17, 100, 1000, 5000):
        pairs = [(word(1, 12), float(rng.integers(-50, 50))) for _ in range(n)]
        B.append(_sl_blob(pairs))                                                    # random order
        B.append(_sl_blob(sorted(pairs, key=lambda x: (x[1], x[0]), reverse=True)))  # serZset order
    B.append(_sl_blob([(b"a", 0.0), (b"m", -0.0), (b"m", 0.0), (b"m", -0.0), (b"b", 0.0)]))
    B.append(_sl_blob([(b"x", 1.0), (b"x", 1.0), (b"x", 2.0)]))
    B.append(_sl_blob([(b"x", 3.0), (b"y", float("nan")), (b"z", 1.0)]))
    B.append(_sl_blob([(b"x", struct.pack("<Q", 0xFFF8000000000001))]))
    B.append(_sl_blob([(b"q", float("inf")), (b"p", float("-inf")), (b"r", float("inf"))]))
    return B


def test_fixup_pass_matches_oracle(engine):
    """desSet de-duplication, desHash's duplicate-field assert, desZset's re-sort and NaN assert:
    GPU records, descriptors, totals and re-encoded bytes equal the C oracle's."""
    rng = np.random.default_rng(31)
    blobs = _fixup_blobs(rng)
    # interleave with ordinary values so fixed-up values share windows with fast-path ones
    data0, offs0 = rr.gen_batch(4, 400, seed=5)
    mixed = []
    for i, b in enumerate(blobs):
        mixed.append(b)
        mixed.append(bytes(data0[offs0[i]:offs0[i + 1]]))
    data, offs = batch_from_blobs(mixed)
    v, e, a, t = engine.decode_host(data, offs)
    ov, oe, oa, ot = cpu.decode(data, offs, nthreads=4)
    assert_flat_equal((v, e), (ov, oe), "fixup")
    assert t == ot
    st = ov["status"]
    assert (st == 13).sum() == 5 and (st == 14).sum() == 2       # the dup-field hashes, the NaN zsets
    ok = np.nonzero(st == 0)[0]
    out, ooffs, t2 = engine.encode_host(v, e, a)
    xo, xoffs, xt = cpu.encode(ov, oe, oa)
    assert t2 == xt and np.array_equal(ooffs, xoffs) and np.array_equal(out, xo)
    assert t2["n_bad"] == len(v) - len(ok)


def test_fixup_pass_device_entry_repeatable(engine):
    """The same batch decoded twice through the device entry point (the fixup queue and its
    ticket are reset per call) gives identical results."""
    import torch
    blobs = _fixup_blobs(np.random.default_rng(2))
    data, offs = batch_from_blobs(blobs)
    n, nb = len(offs) - 1, int(offs[-1])
    dev = torch.device("cuda:0")
    d_data = torch.from_numpy(data).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    cap = rr.elem_bound(n, nb)
    res = []
    for _ in range(2):
        d_vals = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
        d_elems = torch.zeros(cap * 16, dtype=torch.uint8, device=dev)
        d_arena = torch.zeros((nb + 15) & ~15, dtype=torch.uint8, device=dev)
        d_tot = torch.zeros(4, dtype=torch.int64, device=dev)
        engine.decode_device(d_data, d_offs, d_vals, d_elems, d_arena, d_tot)
        torch.cuda.synchronize()
        res.append((d_vals.cpu().numpy().copy(), d_elems.cpu().numpy().copy(), d_tot.cpu().numpy().copy()))
    assert all(np.array_equal(x, y) for x, y in zip(res[0], res[1]))
    ov, oe, _, ot = cpu.decode(data, offs)
    assert np.array_equal(res[0][0].view(rr.VALUE_DT), ov)
    assert np.array_equal(res[0][1].view(rr.ELEM_DT)[:len(oe)], oe)


def test_config4_at_baseline_size_10m(engine):
    """BASELINE.json config 4 at its own size: 10M mixed values (~5 GB of blobs, ~150M
    descriptors) decoded and encoded with the device entry points.  Exercises the 64-bit
    offsets, 32-bit elem_base / first-value tables and buffer-resource clamps at scale:
    records and descriptors equal the C oracle's (16 host threads), encode(decode(b)) == b."""
    import torch
    n = 10_000_000
    data, offs = rr.gen_batch(4, n)
    nb = int(offs[-1])
    assert nb > (1 << 32)                         # offsets and arena offsets past 32 bits
    ov, oe, _, ot = cpu.decode(data, offs, elem_cap=34 * n, nthreads=16)
    assert ot["n_bad"] == 0
    cap = ot["n_elems"] + 64
    dev = torch.device("cuda:0")
    d_data = torch.from_numpy(data).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    del data
    d_vals = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    d_elems = torch.zeros(cap * 16, dtype=torch.uint8, device=dev)
    d_arena = torch.zeros((nb + 15) & ~15, dtype=torch.uint8, device=dev)
    d_tot = torch.zeros(4, dtype=torch.int64, device=dev)
    engine.decode_device(d_data, d_offs, d_vals, d_elems, d_arena, d_tot)
    torch.cuda.synchronize()
    tot = d_tot.cpu().numpy().view(np.uint64)
    assert int(tot[2]) == 0 and int(tot[0]) == ot["n_elems"] and int(tot[3]) == ot["payload"]
    assert int(tot[1]) == nb
    assert np.array_equal(d_vals.cpu().numpy().view(rr.VALUE_DT), ov)
    assert np.array_equal(d_elems[:ot["n_elems"] * 16].cpu().numpy().view(rr.ELEM_DT), oe)
    del ov, oe
    assert torch.equal(d_arena[:nb], d_data[:nb])
    del d_arena
    d_out = torch.zeros((nb + 15) & ~15, dtype=torch.uint8, device=dev)
    d_ooffs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    d_arena2 = d_data                               # the arena mirrors the blob buffer
    engine.encode_device(d_vals, d_elems, d_arena2, d_out, d_ooffs, d_tot)
    torch.cuda.synchronize()
    tot = d_tot.cpu().numpy().view(np.uint64)
    assert int(tot[2]) == 0 and int(tot[1]) == nb
    assert torch.equal(d_out[:nb], d_data[:nb])
    assert np.array_equal(d_ooffs.cpu().numpy().view(np.uint64), offs)


@pytest.mark.parametrize("cfg,n", [(4, 3000), (3, 1500), (10, 600), (11, 40), (1, 2000)])
def test_fuzz_structured_decode_and_reencode(engine, cfg, n):
    """~60K mutated blobs over five configs: bit flips, truncations, random bytes, header and
    length fields overwritten with small / boundary / huge values (counts, lengths, zlbytes /
    zltail / zllen, intset width and count, encoding bytes), inserted and swapped bytes.  The
    GPU's records, descriptors and totals equal the oracle's value for value, and every value
    that decoded re-encodes to the oracle's bytes.  RR_FUZZ_ROUNDS=k repeats it with k seeds
    (an extended run; the suite runs one)."""
    import os
    for k in range(int(os.environ.get("RR_FUZZ_ROUNDS", "1"))):
        _fuzz_structured_round(engine, cfg, n, 1000 + cfg + 7919 * k)


def _fuzz_structured_round(engine, cfg, n, seed):
    data, offs = rr.gen_batch(cfg, n)
    blobs = structured_mutations(data, offs, seed)
    fdata, foffs = batch_from_blobs(blobs)
    v, e, a, t = engine.decode_host(fdata, foffs)
    ov, oe, oa, ot = cpu.decode(fdata, foffs, nthreads=8)
    assert_flat_equal((v, e), (ov, oe), f"structured fuzz cfg {cfg} seed {seed}")
    assert t == ot
    assert (v["status"] != 0).any() and (v["status"] == 0).any()
    # every value that decoded re-encodes like the oracle's encode of the same flat batch
    gd, go, gt = engine.encode_host(v, e, a)
    od, oo, otot = cpu.encode(ov, oe, oa)
    assert np.array_equal(go, oo) and np.array_equal(gd, od[:int(oo[-1])]) and gt == otot


def _device_decode(data, offs, cap=None):
    import torch
    n, nb = len(offs) - 1, int(offs[-1])
    dev = torch.device("cuda:0")
    d_data = torch.zeros((nb + 15) & ~15 or 16, dtype=torch.uint8, device=dev)
    d_data[:nb] = torch.from_numpy(data[:nb]).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    cap = rr.elem_bound(n, nb) if cap is None else cap
    d_vals = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    d_elems = torch.zeros(max(cap, 1) * 16, dtype=torch.uint8, device=dev)
    d_arena = torch.zeros(d_data.numel(), dtype=torch.uint8, device=dev)
    d_tot = torch.zeros(4, dtype=torch.int64, device=dev)
    eng = rr.Engine(0)
    eng.decode_device(d_data, d_offs, d_vals, d_elems, d_arena, d_tot)
    torch.cuda.synchronize()
    tot = d_tot.cpu().numpy().view(np.uint64).copy()
    eng.close()
    return (d_vals.cpu().numpy().view(rr.VALUE_DT), d_elems.cpu().numpy().view(rr.ELEM_DT)[:min(int(tot[0]), cap)],
            d_arena.cpu().numpy()[:nb], tot)


def _payload_equal(e, a, b):
    """the arena bytes every STR / ZLRAW descriptor points at"""
    k = (e["kind"] == 1) | (e["kind"] == 3)
    for d, ln in zip(e["data"][k].astype(np.int64), e["len"][k].astype(np.int64)):
        if not np.array_equal(a[d:d + ln], b[d:d + ln]):
            return False
    return True


@pytest.mark.parametrize("cfg,n", [(4, 1_000_000), (3, 200_000), (10, 8_000)])
def test_host_decode_pipelined_matches_device(engine, cfg, n):
    """rr_decode_batch_host on a batch of more than RR_HOST_CHUNK bytes runs chunked (uploads,
    per-chunk decodes with descriptor placement and elem_base rebase, downloads on a second
    stream): records, descriptors, totals and every payload equal one whole-batch device
    decode.  Config 10 carries malformed values (statuses and zero-filled slots)."""
    data, offs = rr.gen_batch(cfg, n)
    nb = int(offs[-1])
    assert nb > 16 << 20, "the batch must take the chunked path"
    v, e, a, tot = _device_decode(data, offs)
    hv, he, ha, ht = engine.decode_host(data, offs)
    assert_flat_equal((v, e), (hv, he), f"cfg {cfg} pipelined host decode")
    assert (int(tot[0]), int(tot[1]), int(tot[2]), int(tot[3])) == (ht["n_elems"], ht["bytes"], ht["n_bad"], ht["payload"])
    assert _payload_equal(e, a, ha)


def test_host_decode_pipelined_pinned_buffers(engine):
    """The same path with pinned host buffers (the overlap case) and a reused context: two
    calls of different batches through one engine give each batch's device decode."""
    import ctypes as C
    import torch
    L = rr.lib()
    for cfg, n in [(2, 150_000), (4, 300_000)]:
        data, offs = rr.gen_batch(cfg, n)
        nb = int(offs[-1])
        cap = rr.elem_bound(n, nb)
        h_data = torch.from_numpy(data).pin_memory()
        h_offs = torch.from_numpy(offs.view(np.int64)).pin_memory()
        h_vals = torch.zeros(n * 16, dtype=torch.uint8).pin_memory()
        h_elems = torch.zeros(cap * 16, dtype=torch.uint8).pin_memory()
        h_arena = torch.zeros(nb, dtype=torch.uint8).pin_memory()
        t = rr.Totals()
        rc = L.rr_decode_batch_host(engine._ctx, h_data.data_ptr(), h_offs.data_ptr(), n, h_vals.data_ptr(),
                                    h_elems.data_ptr(), cap, h_arena.data_ptr(), C.byref(t))
        assert rc == 0, rr.lib().rr_last_error()
        v, e, a, tot = _device_decode(data, offs)
        hv = h_vals.numpy().view(rr.VALUE_DT)
        he = h_elems.numpy().view(rr.ELEM_DT)[:int(t.n_elems)]
        assert_flat_equal((v, e), (hv, he), f"cfg {cfg} pinned")
        assert int(t.n_elems) == int(tot[0]) and int(t.payload) == int(tot[3])
        assert _payload_equal(e, a, h_arena.numpy())


def test_host_decode_pipelined_capacity(engine):
    """A chunked host decode whose descriptors overflow elem_cap is redone in one call: the
    capacity statuses, records and descriptors equal a whole-batch device decode with the same
    elem_cap."""
    data, offs = rr.gen_batch(4, 200_000)
    _, _, _, full = _device_decode(data, offs)
    cap = int(full[0]) * 3 // 5
    v, e, a, tot = _device_decode(data, offs, cap)
    hv, he, ha, ht = engine.decode_host(data, offs, elem_cap=cap)
    # descriptors of the values that fit (the slots below elem_cap of the value that crosses it
    # belong to no value and are not written)
    ok = v["status"] == 0
    end = int((v["elem_base"][ok].astype(np.int64) + v["n_elems"][ok]).max())
    assert_flat_equal((v, e[:end]), (hv, he[:end]), "pipelined capacity")
    assert ht["n_bad"] == int(tot[2]) > 0


def test_host_decode_without_arena(engine):
    """arena = NULL skips the arena's download (the caller's blob buffer is the mirror): the
    records and descriptors are those of the full call, and every STR / ZLRAW descriptor
    indexes the caller's own blob bytes."""
    import ctypes as C
    L = rr.lib()
    data, offs = rr.gen_batch(4, 120_000)   # > 16 MiB: the chunked path
    n, nb = len(offs) - 1, int(offs[-1])
    cap = rr.elem_bound(n, nb)
    hv, he, ha, ht = engine.decode_host(data, offs)
    vals = np.zeros(n, rr.VALUE_DT)
    els = np.zeros(cap, rr.ELEM_DT)
    t = rr.Totals()
    rc = L.rr_decode_batch_host(engine._ctx, data.ctypes.data, offs.ctypes.data, n, vals.ctypes.data,
                                els.ctypes.data, cap, None, C.byref(t))
    assert rc == 0
    assert_flat_equal((vals, els[:int(t.n_elems)]), (hv, he), "arena = NULL")
    assert _payload_equal(he, ha, data)


def _dense_class_batches(rng):
    """Homogeneous batches of small values: a 64 KiB window then holds hundreds of one class,
    so its batches carry 64 values (one or two lanes each: the grouped walks at G = 1, 2, 4)
    as well as the partly filled last batch; sizes vary so windows see every G."""
    def word(lo, hi):
        return rng.integers(97, 123, int(rng.integers(lo, hi + 1)), dtype=np.uint8).tobytes()

    def lst(k):
        items = [str(int(rng.integers(-10**6, 10**6))).encode() if rng.random() < 0.5 else word(0, 12) for _ in range(k)]
        return bytes([rr.T_LIST_QUICKLIST]) + struct.pack("<I", 5) + b"".join(struct.pack("<I", len(x)) + x for x in items)

    def iset(k):
        w = int(rng.choice([2, 4, 8]))
        vals = sorted(set(int(x) for x in rng.integers(-(1 << (8 * w - 1)), (1 << (8 * w - 1)) - 1, k)))
        return bytes([rr.T_SET_INTSET]) + struct.pack("<III", 3, w, len(vals)) + b"".join(
            v.to_bytes(w, "little", signed=True) for v in vals)

    def zl(t, k):
        items = []
        for i in range(k):
            items += [word(1, 10) + str(i).encode(),
                      (str(int(rng.integers(-10**9, 10**9))).encode() if rng.random() < 0.5 else word(0, 70))]
        z = po.build_ziplist(items)
        return bytes([t]) + struct.pack("<I", 11) + struct.pack("<Q", len(z)) + z

    def sl(k):
        pairs = sorted(((word(0, 9) + str(i).encode(), float(rng.integers(-10**6, 10**6)) + i / 7) for i in range(k)),
                       key=lambda x: (x[1], x[0]), reverse=True)
        return _sl_blob(pairs)

    makers = {
        "list": lambda k: lst(k),
        "intset": lambda k: iset(max(k, 1)),
        "set_ht": lambda k: _ht_blob(rr.T_SET_HT, [word(0, 8) + str(i).encode() for i in range(k)]),
        "hash_ht": lambda k: _ht_blob(rr.T_HASH_HT, sum(([b"f%d" % i, word(0, 12)] for i in range(k)), [])),
        "zset_sl": lambda k: sl(k),
        "hash_zl": lambda k: zl(rr.T_HASH_ZIPLIST, k),
        "zset_zl": lambda k: zl(rr.T_ZSET_ZIPLIST, k),
    }
    for name, mk in makers.items():
        for kmax in (1, 3, 9):
            yield f"{name} k<={kmax}", [mk(int(rng.integers(0, kmax + 1))) for _ in range(6000)]
        # and with every 37th value cut short, grown by a byte or with a body byte flipped (the
        # walks' failure paths; the oracle decides which values stay valid)
        blobs = [mk(int(rng.integers(0, 4))) for _ in range(6000)]
        for i in range(0, len(blobs), 37):
            b, how = blobs[i], (i // 37) % 3
            if how == 0:
                b = b[:-1]
            elif how == 1:
                b = b + b"\x00"
            elif len(b) > 14:
                j = int(rng.integers(13, len(b)))
                b = b[:j] + bytes([b[j] ^ (1 << int(rng.integers(0, 8)))]) + b[j + 1:]
            blobs[i] = b
        yield f"{name} damaged", blobs


def test_dense_single_class_windows(engine):
    """Windows holding hundreds of values of one class: every grouped walk at G = 1 / 2 / 4 and
    with partly filled batches, against the C oracle, plus the byte-exact round trip."""
    rng = np.random.default_rng(2024)
    for what, blobs in _dense_class_batches(rng):
        data, offs = batch_from_blobs(blobs)
        v, e, a, t = engine.decode_host(data, offs)
        ov, oe, oa, ot = cpu.decode(data, offs, nthreads=8)
        assert_flat_equal((v, e), (ov, oe), what)
        assert t == ot, what
        if "damaged" in what:
            assert t["n_bad"] > 0, what
            continue
        assert t["n_bad"] == 0, what
        out, ooffs, t2 = engine.encode_host(v, e, a)
        assert np.array_equal(out, data[:int(offs[-1])]), what


def test_config5_per_gpu_shard_at_full_size(engine):
    """BASELINE config 5 — 100M values in config-4 proportions over 8 GPUs — one GPU's share
    at its real size: the byte-balanced 8-way plan of the whole 100M batch (rr_shard_plan over
    the sizes of all 100M values), then the LAST shard (~12.5M values, ~6.2 GB) generated on
    its own, decoded on the device and checked bit-exact against the C oracle, encoded back on
    the device bit-exact, and placed at its whole-batch position with rr_flat_rebase
    (elem_base += the descriptors of the 87.5M values before it, arena offsets += its first
    byte, ~43 GB) — equal to the oracle's decode rebased the same way."""
    import torch
    N, G, nt = 100_000_000, 8, min(16, cpu.nprocs())
    nb, nd = rr.gen_sizes(5, 0, N, nthreads=nt)
    offs = np.zeros(N + 1, np.uint64)
    np.cumsum(nb, out=offs[1:])
    del nb
    plan = rr.shard_plan(offs, G)
    v0, v1, b0, b1 = (int(x) for x in plan[G - 1])
    elem_add = int(nd[:v0].sum(dtype=np.uint64))
    shard_descs = int(nd[v0:v1].sum(dtype=np.uint64))
    assert v1 == N and b1 == int(offs[N]) and 12_000_000 < v1 - v0 < 13_000_000
    assert 40e9 < b0 < 46e9 and 1.2e9 < elem_add < 2 ** 32 - shard_descs
    data, soffs = rr.gen_range(5, v0, v1, nthreads=nt)
    assert np.array_equal(soffs, offs[v0:v1 + 1] - np.uint64(b0))
    del offs
    n, nbytes = v1 - v0, b1 - b0
    ov, oe, _, ot = cpu.decode(data, soffs, elem_cap=shard_descs, nthreads=nt)
    assert ot["n_bad"] == 0 and ot["n_elems"] == shard_descs and np.array_equal(ov["n_elems"], nd[v0:v1])
    del nd
    dev = torch.device("cuda:0")
    d_data = torch.from_numpy(data).to(dev)
    d_offs = torch.from_numpy(soffs.view(np.int64)).to(dev)
    d_vals = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    d_elems = torch.zeros(shard_descs * 16, dtype=torch.uint8, device=dev)
    d_arena = torch.zeros(d_data.numel(), dtype=torch.uint8, device=dev)
    d_tot = torch.zeros(4, dtype=torch.int64, device=dev)
    engine.reserve(n, nbytes)
    engine.decode_device(d_data, d_offs, d_vals, d_elems, d_arena, d_tot)
    torch.cuda.synchronize()
    tot = d_tot.cpu().numpy().view(np.uint64)
    assert int(tot[0]) == shard_descs and int(tot[1]) == nbytes and int(tot[2]) == 0
    assert torch.equal(d_arena[:nbytes], d_data[:nbytes])
    assert_flat_equal((d_vals.cpu().numpy().view(rr.VALUE_DT), d_elems.cpu().numpy().view(rr.ELEM_DT)), (ov, oe),
                      "config 5 last shard")
    # encode back on the device
    d_out = torch.zeros(d_data.numel(), dtype=torch.uint8, device=dev)
    d_ooffs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    d_tot2 = torch.zeros(4, dtype=torch.int64, device=dev)
    engine.encode_device(d_vals, d_elems, d_arena, d_out, d_ooffs, d_tot2)
    torch.cuda.synchronize()
    assert int(d_tot2[2].item()) == 0 and torch.equal(d_out[:nbytes], d_data[:nbytes])
    assert torch.equal(d_ooffs, d_offs)
    del d_out, d_ooffs
    # the shard at its place in the whole 100M batch
    engine.flat_rebase(d_vals, d_elems, elem_add, b0)
    torch.cuda.synchronize()
    ov["elem_base"] += np.uint32(elem_add)
    ref = ((oe["kind"] == rr.K_STR) | (oe["kind"] == rr.K_ZLRAW)) & ((oe["data"] | oe["len"]) != 0)
    oe["data"][ref] += np.uint64(b0)
    gv, ge = d_vals.cpu().numpy().view(rr.VALUE_DT), d_elems.cpu().numpy().view(rr.ELEM_DT)
    assert int(gv["elem_base"].max()) + int(gv["n_elems"][gv["elem_base"].argmax()]) == elem_add + shard_descs
    assert int(ge["data"][ref].max()) > 40_000_000_000
    assert_flat_equal((gv, ge), (ov, oe), "config 5 last shard rebased to its whole-batch position")


@pytest.mark.parametrize("cfg,n", [(1, 500_000), (2, 60_000), (4, 65_000), (3, 45_000)])
def test_one_launch_full_generation(engine, cfg, n):
    """Device-resident batches of one full window generation (up to 512 windows of ~68 KiB) take
    the one-launch decode (decode_kernel's ONE form): config 1 at 500K values puts ~980 values in
    a window (two sort chunks: the later chunk's classes kept in the scratch), config 2's Zipf
    strings leave windows unstaged, configs 3 / 4 the grouped walks.  Records, descriptors,
    totals and payloads equal the oracle's; the round trip re-encodes the batch."""
    data, offs = rr.gen_batch(cfg, n)
    nb = int(offs[-1])
    v, e, a, tot = _device_decode(data, offs)
    ov, oe, oa, ot = cpu.decode(data, offs, nthreads=8)
    assert_flat_equal((v, e), (ov, oe), f"cfg {cfg} one launch")
    assert (int(tot[0]), int(tot[1]), int(tot[2]), int(tot[3])) == (ot["n_elems"], ot["bytes"], ot["n_bad"], ot["payload"])
    assert _payload_equal(e, a, oa)
    out, ooffs, _ = engine.encode_host(v, e, a)
    assert np.array_equal(ooffs, offs) and out.tobytes() == data[:nb].tobytes()


@pytest.mark.parametrize("cfg,n,slack", [(1, 100_000, 3), (4, 20_000, 8)])
def test_one_launch_data_cap_past_the_batch(engine, cfg, n, slack):
    """A device batch whose buffer (data_cap) runs far past its last value, the tail filled with
    random bytes: the one-launch form guesses its values from data_cap, so its windows past the
    data own no values and the search's guess is off; records, descriptors, totals and the
    arena's [offsets[0], offsets[n]) equal the oracle's, and no byte past the batch is copied."""
    import torch
    data, offs = rr.gen_batch(cfg, n)
    nb = int(offs[-1])
    cap_b = ((nb + 15) & ~15) * slack
    dev = torch.device("cuda:0")
    host = np.random.default_rng(5).integers(0, 256, cap_b, dtype=np.uint8)
    host[:nb] = data[:nb]
    d_data = torch.from_numpy(host).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    cap = rr.elem_bound(n, nb)
    d_vals = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    d_elems = torch.zeros(cap * 16, dtype=torch.uint8, device=dev)
    d_arena = torch.zeros(cap_b, dtype=torch.uint8, device=dev)
    d_tot = torch.zeros(4, dtype=torch.int64, device=dev)
    engine.decode_device(d_data, d_offs, d_vals, d_elems, d_arena, d_tot)
    torch.cuda.synchronize()
    tot = d_tot.cpu().numpy().view(np.uint64)
    v = d_vals.cpu().numpy().view(rr.VALUE_DT)
    e = d_elems.cpu().numpy().view(rr.ELEM_DT)[:int(tot[0])]
    a = d_arena.cpu().numpy()
    ov, oe, oa, ot = cpu.decode(data, offs, nthreads=8)
    assert_flat_equal((v, e), (ov, oe), f"cfg {cfg} data_cap x{slack}")
    assert (int(tot[0]), int(tot[1]), int(tot[2]), int(tot[3])) == (ot["n_elems"], ot["bytes"], ot["n_bad"], ot["payload"])
    assert _payload_equal(e, a, oa)
    assert not a[(nb + 15) & ~15:].any(), "bytes past the batch copied into the arena"

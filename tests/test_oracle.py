"""CPU tests: the oracles are pinned against the golden vectors and against each other.

Pins: KATs K1-K9 hand-derived from rock_serdes.c; util.c:754-897 string2ll and
ll2string vectors; the ziplist.c:114-149 byte example; intset.c:361-375 encoding boundaries;
edge/malformed fixtures (tests/golden/make_golden.py).  The C oracle, the Python restatement and
the synthetic generator are three independent writers/readers of the format; every pair is
cross-checked here.
"""
import struct

import numpy as np
import pytest

import redrock_old_amd as rr
from oracle import cpu
from oracle import pyoracle as po

from helpers import assert_flat_equal, batch_from_blobs, expected_flat, golden


G = golden()
M64 = (1 << 64) - 1


def reencoded(blob):
    """What serObject(desObject(blob)) writes: robj.lru keeps only 24 bits (server.h:592-599)."""
    if len(blob) < 5:
        return blob
    return blob[:1] + struct.pack("<I", struct.unpack_from("<I", blob, 1)[0] & 0xFFFFFF) + blob[5:]


@pytest.mark.parametrize("kat", G["kats"], ids=[k["name"] for k in G["kats"]])
def test_kat_decode_encode(kat):
    blob = bytes.fromhex(kat["blob"])
    data, offs = batch_from_blobs([blob])
    exp = expected_flat([kat])
    v, e, a, t = cpu.decode(data, offs)
    assert_flat_equal((v, e), exp, kat["name"])
    assert t["n_bad"] == 0
    out, ooffs, _ = cpu.encode(exp[0], exp[1], data)
    assert bytes(out) == blob
    # Python restatement agrees as well
    pv, pe = po.decode_one(blob, 0)
    assert pv["status"] == 0 and [[k, d & M64, ln, z] for k, d, ln, z in pe] == kat["elems"]
    assert po.encode_one(dict(type=blob[0], enc=kat["value"]["enc"], lru=0), pe, blob) == blob


def test_kat_batch_all_together():
    blobs = [bytes.fromhex(k["blob"]) for k in G["kats"]]
    data, offs = batch_from_blobs(blobs)
    v, e, a, t = cpu.decode(data, offs, nthreads=3)
    assert_flat_equal((v, e), expected_flat(G["kats"]), "kat batch")
    out, ooffs, _ = cpu.encode(v, e, a)
    assert bytes(out) == b"".join(blobs)


@pytest.mark.parametrize("fx", G["edges"], ids=[f["name"] for f in G["edges"]])
def test_edge_fixture(fx):
    blob = bytes.fromhex(fx["blob"])
    data, offs = batch_from_blobs([blob])
    v, e, a, t = cpu.decode(data, offs)
    assert_flat_equal((v, e), expected_flat([fx]), fx["name"])
    if fx["value"]["status"] == 0:
        out, _, _ = cpu.encode(v, e, a)
        assert bytes(out) == reencoded(bytes.fromhex(fx.get("reencoded", fx["blob"])))
    else:
        assert t["n_bad"] == 1


def test_string2ll_vectors():
    for s, want in G["string2ll"]:
        assert cpu.string2ll(s.encode()) == want, s
        assert po.string2ll(s.encode()) == want, s


def test_ll2string_vectors():
    for v, s in G["ll2string"]:
        assert cpu.ll2str(v) == s.encode()
        assert po.ll2str(v) == s.encode()


def test_ziplist_reference_example():
    zl = bytes.fromhex(G["ziplist_example"]["two_five"].replace(" ", ""))
    st, ents = cpu.parse_ziplist(zl)
    assert st == 0 and list(ents["kind"]) == [rr.K_INT, rr.K_INT] and list(ents["data"]) == [2, 5]
    # append the "Hello World" entry exactly as ziplist.c:143 shows it
    entry = bytes.fromhex(G["ziplist_example"]["hello_world_entry"].replace(" ", ""))
    body = zl[10:-1] + entry
    zl2 = struct.pack("<IIH", 10 + len(body) + 1, 14, 3) + body + b"\xff"
    st, ents = cpu.parse_ziplist(zl2)
    assert st == 0 and ents[2]["kind"] == rr.K_STR and ents[2]["len"] == 11
    assert zl2[ents[2]["data"]:ents[2]["data"] + 11] == b"Hello World"
    assert po.parse_ziplist(zl2)[2] == (po.K_STR, 16, 11, 0)
    assert po.build_ziplist([b"2", b"5", b"Hello World"]) == zl2


def _width_rule():
    """_intsetValueEncoding (intset.c:45-52) as pinned by intset.c:361-375: the INT16 / INT32
    ranges are the extreme values the golden table assigns width 2 / 4."""
    t = G["intset_encoding"]
    r2 = (min(v for v, w in t if w == 2), max(v for v, w in t if w == 2))
    r4 = (min(v for v, w in t if w == 4), max(v for v, w in t if w == 4))
    assert r2 == (-32768, 32767) and r4 == (-(1 << 31), (1 << 31) - 1)
    return lambda v: 2 if r2[0] <= v <= r2[1] else 4 if r4[0] <= v <= r4[1] else 8


def test_intset_encoding_boundaries():
    rule = _width_rule()
    for v, w in G["intset_encoding"]:
        assert rule(v) == w


@pytest.mark.parametrize("cfg,n", [(4, 3000), (10, 480), (11, 300)])
def test_generator_intset_width_choice(cfg, n):
    """Every intset the generator writes is sorted, duplicate-free and has the smallest width
    holding all its members — the intset a Redis server would hold (intset.c:45-52, :104-120)."""
    rule = _width_rule()
    data, offs = rr.gen_batch(cfg, n)
    seen = 0
    for i in range(n):
        b = bytes(data[offs[i]:offs[i + 1]])
        if b[0] != rr.T_SET_INTSET or len(b) < 13:
            continue
        w, c = struct.unpack_from("<II", b, 5)
        vals = [int.from_bytes(b[13 + k * w:13 + (k + 1) * w], "little", signed=True) for k in range(c)]
        assert vals == sorted(set(vals))
        assert w == max([rule(v) for v in vals] + [2]), (i, w, vals[:4])
        seen += 1
    assert seen > 0


STRICTER = {"bad_intset_width", "intset_u32_wrap", "bad_ziplist_encoding", "bad_ziplist_odd_entries",
            "bad_ziplist_zllen"}


def _members(blob):
    """(count field, sorted member / field-value tuples) of an HT blob."""
    _, el = po.decode_one(blob)
    per = 1 if blob[0] == rr.T_SET_HT else 2
    items = sorted(tuple(blob[x[1]:x[1] + x[2]] for x in el[j:j + per]) for j in range(0, len(el), per))
    return struct.unpack_from("<Q", blob, 5)[0], items


@pytest.mark.parametrize("fx", G["edges"], ids=[f["name"] for f in G["edges"]])
def test_faithful_vs_flat_roundtrip(fx):
    """The reference-faithful restatement (robj / dict / skiplist / quicklist rebuilt, then
    serObject) against the flat round trip on every edge fixture: the same values are rejected,
    and an accepted value re-serializes to the same bytes (HT types: the same count and the same
    members, since dict order is a permutation — SURVEY.md §8c).  The [stricter] fixtures are
    the documented deviations: the reference loads them, the engine rejects them."""
    blob = bytes.fromhex(fx["blob"])
    data, offs = batch_from_blobs([blob])
    fout, foffs, fbad, _, _ = cpu.faithful_roundtrip(data, offs)
    status = fx["value"]["status"]
    if fx["name"] in STRICTER:
        assert status != 0 and fbad == 0
        assert bytes(fout) == reencoded(blob)     # the reference copies these bytes through
        return
    assert (fbad == 1) == (status != 0)
    if status:
        return
    v, e, a, _ = cpu.decode(data, offs)
    out, _, t = cpu.encode(v, e, a)
    assert t["n_bad"] == 0
    if blob[0] in (rr.T_SET_HT, rr.T_HASH_HT):
        assert _members(bytes(fout)) == _members(bytes(out))
    else:
        assert bytes(fout) == bytes(out)


@pytest.mark.parametrize("cfg,n", [(1, 3000), (2, 3000), (3, 800), (4, 4000), (10, 240), (11, 150)])
def test_generator_oracle_roundtrip(cfg, n):
    data, offs = rr.gen_batch(cfg, n)
    v, e, a, t = cpu.decode(data, offs, nthreads=4)
    assert t["n_bad"] == 0
    assert np.array_equal(a, data[:int(offs[-1])])
    out, ooffs, t2 = cpu.encode(v, e, a, nthreads=2)
    assert np.array_equal(ooffs, offs)
    assert np.array_equal(out, data[:int(offs[-1])])
    # single-thread == multi-thread
    v1, e1, _, _ = cpu.decode(data, offs, nthreads=1)
    assert_flat_equal((v1, e1), (v, e), f"cfg{cfg} mt")


@pytest.mark.parametrize("cfg,n", [(4, 600), (10, 96)])
def test_python_restatement_matches_c(cfg, n):
    data, offs = rr.gen_batch(cfg, n)
    v, e, a, t = cpu.decode(data, offs)
    blobs = [bytes(data[offs[i]:offs[i + 1]]) for i in range(n)]
    _, _, pv, pe, _ = po.decode_batch(blobs)
    for i in range(n):
        for k in ("type", "enc", "status", "lru", "n_elems", "elem_base"):
            assert pv[i][k] == v[i][k], (i, k)
    assert len(pe) == len(e)
    for x, y in zip(pe, e):
        assert (x[0], x[1] & 0xFFFFFFFFFFFFFFFF, x[2], x[3]) == (y["kind"], y["data"], y["len"], y["zenc"])


def test_faithful_roundtrip():
    """Reference-faithful mode (robj/sds/dict/skiplist/quicklist): exact for every non-HT
    type; HT values come back as a permutation of the same members."""
    data, offs = rr.gen_batch(4, 3000)
    out, ooffs, bad, _, _ = cpu.faithful_roundtrip(data, offs)
    assert bad == 0
    assert np.array_equal(ooffs, offs)
    for i in range(len(offs) - 1):
        a = bytes(data[offs[i]:offs[i + 1]])
        b = bytes(out[ooffs[i]:ooffs[i + 1]])
        if a[0] in (rr.T_SET_HT, rr.T_HASH_HT):
            _, ea = po.decode_one(a)
            _, eb = po.decode_one(b)
            per = 1 if a[0] == rr.T_SET_HT else 2
            ma = sorted(tuple(a[x[1]:x[1] + x[2]] for x in ea[j:j + per]) for j in range(0, len(ea), per))
            mb = sorted(tuple(b[x[1]:x[1] + x[2]] for x in eb[j:j + per]) for j in range(0, len(eb), per))
            assert ma == mb
        else:
            assert a == b, i


def test_decode_capacity_and_empty():
    data, offs = rr.gen_batch(4, 100)
    v, e, a, t = cpu.decode(data, offs, elem_cap=10)
    assert t["n_bad"] > 0 and (v["status"] == 11).any()
    v, e, a, t = cpu.decode(np.zeros(16, np.uint8), np.zeros(1, np.uint64))
    assert len(v) == 0 and t["n_elems"] == 0


@pytest.mark.parametrize("fx", G["shapes"], ids=[f["name"] for f in G["shapes"]])
def test_reference_shaped_values(fx):
    """ziplist.c:1255-1281's createList / createIntList and the value of every type
    testredrock/test_redrock.py:76-117 warms up: the C oracle's decode equals the literal flat
    form, its encode rewrites the blob, and the reference-faithful restatement (robj rebuilt,
    serObject) accepts it and writes the same bytes (HT types: the same members)."""
    blob = bytes.fromhex(fx["blob"])
    data, offs = batch_from_blobs([blob])
    v, e, a, t = cpu.decode(data, offs)
    assert_flat_equal((v, e), expected_flat([fx]), fx["name"])
    assert t["n_bad"] == 0
    out, _, _ = cpu.encode(v, e, a)
    assert bytes(out) == blob
    fout, _, fbad, _, _ = cpu.faithful_roundtrip(data, offs)
    assert fbad == 0
    if blob[0] in (rr.T_SET_HT, rr.T_HASH_HT):
        assert _members(bytes(fout)) == _members(blob)
    else:
        assert bytes(fout) == blob


def test_reference_shaped_batch():
    """All of them in one multi-threaded batch (arena offsets across values)."""
    blobs = [bytes.fromhex(f["blob"]) for f in G["shapes"]]
    data, offs = batch_from_blobs(blobs)
    v, e, a, t = cpu.decode(data, offs, nthreads=4)
    assert_flat_equal((v, e), expected_flat(G["shapes"]), "shapes batch")
    out, _, _ = cpu.encode(v, e, a)
    assert bytes(out) == b"".join(blobs)


def test_config5_generator_is_seekable():
    """Config 5 (the 100M batch of BASELINE config 5): any value range generated alone equals
    the same range of the whole batch, sizes and descriptor counts come without the bytes and
    agree with the C oracle's decode."""
    d, o = rr.gen_batch(5, 12000)
    d2, o2 = rr.gen_range(5, 0, 12000, nthreads=4)
    assert np.array_equal(d, d2) and np.array_equal(o, o2)
    d3, o3 = rr.gen_range(5, 5000, 9001, nthreads=3)
    assert np.array_equal(o3, o[5000:9002] - o[5000])
    assert np.array_equal(d3[:int(o3[-1])], d[int(o[5000]):int(o[9001])])
    nb, nd = rr.gen_sizes(5, 0, 12000, nthreads=5)
    assert np.array_equal(np.cumsum(nb.astype(np.int64)), o[1:].astype(np.int64))
    v, e, a, t = cpu.decode(d, o, nthreads=4)
    assert t["n_bad"] == 0 and np.array_equal(v["n_elems"], nd) and t["n_elems"] == int(nd.sum())
    # config-4 proportions: 40 % strings, 15 % each collection type
    types, counts = np.unique(d[o[:-1].astype(np.int64)], return_counts=True)
    frac = dict(zip(types.tolist(), (counts / 12000).tolist()))
    assert abs(frac[0] - 0.40) < 0.03 and abs(frac[14] - 0.15) < 0.02

"""The host codec (include/rr_host.h, redrock_old_amd/csrc/rr_host.c): the CPU routing target of
the compat shim for RedRock's per-key call sites (desObject at rock.c:468 / :538, serObject at
rock.c:691; SURVEY.md §8b "runs the CPU path for a single value").  It is product code, not the
oracle, and must give the GPU path's exact flat form: records, descriptors, statuses, totals,
offsets and bytes equal the oracle's (which the GPU suite holds the GPU to) on the golden
fixtures, every synthetic config, the structured fuzz corpus and capacity cuts.  CPU only."""
import numpy as np
import pytest

import redrock_old_amd as rr
from helpers import assert_flat_equal, batch_from_blobs, expected_flat, golden, structured_mutations
from oracle import cpu

G = golden()
FIXTURES = G["kats"] + G["edges"] + G["shapes"]


def _same_decode(data, offs, what, elem_cap=None):
    if elem_cap is None:
        elem_cap = rr.elem_bound(len(offs) - 1, int(offs[-1]))
    v, e, a, t = rr.host_decode(data, offs, elem_cap)
    ov, oe, oa, ot = cpu.decode(data, offs, elem_cap)
    assert_flat_equal((v, e), (ov, oe), what)
    # rr_host_check_value (the shim's verdict-only walk of ziplists): the same records, CAPACITY
    # aside (it has no elem_cap), elem_base 0
    c = rr.host_check(data, offs)
    want = ov.copy()
    want["elem_base"] = 0
    cut = want["status"] == 11
    assert np.array_equal(c[~cut], want[~cut]), what
    assert t == ot, (what, t, ot)
    assert np.array_equal(a, oa)
    return v, e, a, t


def _same_encode(v, e, a, what, data_cap=None):
    d, o, t = rr.host_encode(v, e, a, data_cap)
    od, oo, ot = cpu.encode(v, e, a, data_cap)
    assert np.array_equal(o, oo), what
    assert np.array_equal(d, od[:int(oo[-1])][:len(d)]), what
    assert t == ot, (what, t, ot)
    return d, o, t


def test_golden_batch_matches_literals_and_oracle():
    """K1-K9, the edge fixtures and the reference's test shapes in one batch: the flat form equals
    the hand-written literals of tests/golden/kat.json and the oracle; every valid value
    re-encodes to the bytes serObject writes."""
    blobs = [bytes.fromhex(f["blob"]) for f in FIXTURES]
    data, offs = batch_from_blobs(blobs)
    v, e, a, t = _same_decode(data, offs, "golden batch")
    assert_flat_equal((v, e), expected_flat(FIXTURES), "golden literals")
    d, o, t2 = _same_encode(v, e, a, "golden re-encode")
    for i, f in enumerate(FIXTURES):
        if f["value"].get("status", 0) == 0:
            want = bytes.fromhex(f.get("reencoded", f["blob"]))
            want = want[:1] + (int.from_bytes(want[1:5], "little") & 0xFFFFFF).to_bytes(4, "little") + want[5:]
            assert bytes(d[int(o[i]):int(o[i + 1])]) == want, f["name"]


@pytest.mark.parametrize("fx", FIXTURES, ids=[f["name"] for f in FIXTURES])
def test_each_fixture_one_value(fx):
    """rr_host_decode_value, the shim's one-value entry: the fixture's status, record and
    descriptors (base 0: offsets into the blob itself); a too-small buffer says how many slots."""
    blob = bytes.fromhex(fx["blob"])
    st, v, e, need = rr.host_decode_value(blob, cap=1 << 16)
    want_v, want_e = expected_flat([fx])
    assert st == int(want_v[0]["status"])
    for k in ("type", "enc", "status", "lru", "n_elems"):
        assert int(v[k]) == int(want_v[0][k]), (fx["name"], k)
    if st == 0:
        n = int(v["n_elems"])
        assert np.array_equal(e, want_e[:n]), fx["name"]
        if n > 1:   # one slot short: RR_E_CAPACITY and the slots it needs, then it fits
            st2, v2, _, need2 = rr.host_decode_value(blob, cap=need - 1)
            assert st2 == 11 and need2 == need
            st3, v3, e3, _ = rr.host_decode_value(blob, cap=need)
            assert st3 == 0 and np.array_equal(e3, e)


@pytest.mark.parametrize("cfg,n", [(1, 3000), (2, 2000), (3, 1500), (4, 6000), (10, 3000), (11, 60)])
def test_configs_match_oracle(cfg, n):
    """Every synthetic config (SURVEY.md §8d shapes; 10 = edge cases with malformed values, 11 =
    large values): decode equal to the oracle, encode(decode(b)) == b."""
    data, offs = rr.gen_batch(cfg, n)
    v, e, a, t = _same_decode(data, offs, f"cfg {cfg}")
    d, o, t2 = _same_encode(v, e, a, f"cfg {cfg} encode")
    if t["n_bad"] == 0:
        assert np.array_equal(o, offs) and np.array_equal(d, data[:int(offs[-1])])


@pytest.mark.parametrize("cfg,n,seed", [(4, 2000, 1), (3, 800, 2), (10, 600, 3), (11, 30, 4), (1, 1000, 5),
                                        (4, 2000, 11), (10, 600, 13)])
def test_structured_fuzz_matches_oracle(cfg, n, seed):
    """The GPU suite's structured fuzz corpus (tests/helpers.py structured_mutations): every
    mutated blob's status, record and descriptors equal the oracle's; the decoded ones re-encode
    to the oracle's bytes."""
    data, offs = rr.gen_batch(cfg, n)
    fdata, foffs = batch_from_blobs(structured_mutations(data, offs, 1000 + cfg + 7919 * seed))
    v, e, a, t = _same_decode(fdata, foffs, f"fuzz cfg {cfg} seed {seed}")
    assert (v["status"] != 0).any() and (v["status"] == 0).any()
    _same_encode(v, e, a, f"fuzz cfg {cfg} seed {seed} encode")


def test_random_bytes_match_oracle():
    """Blobs of random bytes under every type tag: no value reads past its blob (the host codec
    walks every length field), and the verdicts equal the oracle's."""
    rng = np.random.default_rng(5)
    tags = [0, 2, 4, 5, 11, 12, 13, 14, 1, 255]
    blobs = []
    for _ in range(4000):
        n = int(rng.integers(0, 64))
        b = bytearray(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        if b:
            b[0] = tags[int(rng.integers(len(tags)))]
        blobs.append(bytes(b))
    data, offs = batch_from_blobs(blobs)
    _same_decode(data, offs, "random bytes")


@pytest.mark.parametrize("frac", [0.0, 0.3, 0.77, 1.0])
def test_capacity_cuts_match_oracle(frac):
    """elem_cap below the batch's need: values past it get RR_E_CAPACITY with their counts, the
    ones before it decode; encode with data_cap cut: offsets complete, later values unwritten."""
    data, offs = rr.gen_batch(10, 1500)
    full = int(cpu.decode(data, offs)[3]["n_elems"])
    v, e, a, t = _same_decode(data, offs, f"cap {frac}", elem_cap=int(full * frac))
    d0, o0, t0 = rr.host_encode(*_same_decode(data, offs, "full")[:3])
    _same_encode(*_same_decode(data, offs, "full")[:3], f"data cap {frac}", data_cap=int(int(o0[-1]) * frac))


def test_empty_and_tiny_batches():
    for blobs in ([], [b""], [b"\x00"], [b"\x00\x01\x02\x03\x04"], [b"\x0e\x00\x00\x00\x00"]):
        data, offs = batch_from_blobs(blobs)
        _same_decode(data, offs, repr(blobs))


def test_skiplist_order_and_duplicates_match_oracle():
    """Hand-built skiplists out of serZset's order (shuffled pairs, tied scores, -0.0 / +0.0, ±inf,
    equal members) and HT sets / hashes with repeated members and fields, up to 300 keys (the
    table-based duplicate test): the order the oracle sorts into, the copies it drops, DUP."""
    rng = np.random.default_rng(9)
    blobs = []
    scores = [0.0, -0.0, 1.0, -1.0, float("inf"), float("-inf"), 2.5, 2.5]
    for k in (2, 5, 16, 17, 40, 300):
        for _ in range(6):
            pairs = []
            for _ in range(k):
                m = bytes(rng.integers(97, 100, int(rng.integers(0, 3)), dtype=np.uint8))
                s = float(scores[int(rng.integers(len(scores)))]) if rng.random() < 0.5 else float(rng.integers(-3, 3))
                pairs.append((m, s))
            body = k.to_bytes(8, "little") + b"".join(len(m).to_bytes(8, "little") + m + np.float64(s).tobytes()
                                                    for m, s in pairs)
            blobs.append(bytes([5]) + b"\x00" * 4 + body)
            mem = [bytes(rng.integers(97, 100, int(rng.integers(0, 4)), dtype=np.uint8)) for _ in range(k)]
            blobs.append(bytes([2]) + b"\x00" * 4 + k.to_bytes(8, "little") +
                         b"".join(len(m).to_bytes(8, "little") + m for m in mem))
            fields = [bytes(rng.integers(97, 123, int(rng.integers(1, 3)), dtype=np.uint8)) for _ in range(k)]
            blobs.append(bytes([4]) + b"\x00" * 4 + k.to_bytes(8, "little") +
                         b"".join(len(f).to_bytes(8, "little") + f + (1).to_bytes(8, "little") + b"v" for f in fields))
    data, offs = batch_from_blobs(blobs)
    v, e, a, t = _same_decode(data, offs, "orders and duplicates")
    st = v["status"]
    assert (st == 13).any() and (st == 0).any()
    _same_encode(v, e, a, "orders and duplicates encode")

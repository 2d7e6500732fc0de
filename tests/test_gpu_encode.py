"""GPU encode tests: the window/emit encode pipeline (rr_kernels.hip E1-E5) against the CPU
oracle's encode (oracle/rr_oracle.c rro_encode, rock_serdes.c:512-535 restated) on flat batches
the decoder never produces: relocated arenas and permuted descriptor ranges, values far larger
than one output window, zero-length members, unencodable descriptors and a data_cap that cuts a
value.  Bit-exact: bytes, offsets and totals."""
import struct

import numpy as np
import pytest

import redrock_old_amd as rr
from oracle import cpu

from helpers import batch_from_blobs

pytestmark = pytest.mark.gpu


def _lru(i):
    return (i * 2654435761) & 0xFFFFFF


def s_raw(i, payload):
    return bytes([rr.T_STRING]) + struct.pack("<I", _lru(i)) + b"\x00" + payload


def l_list(i, items):
    return bytes([rr.T_LIST_QUICKLIST]) + struct.pack("<I", _lru(i)) + b"".join(
        struct.pack("<I", len(x)) + x for x in items)


def s_ht(i, members, t=rr.T_SET_HT):
    n = len(members) if t == rr.T_SET_HT else len(members) // 2
    return bytes([t]) + struct.pack("<I", _lru(i)) + struct.pack("<Q", n) + b"".join(
        struct.pack("<Q", len(x)) + x for x in members)


def z_sl(i, pairs):
    return bytes([rr.T_ZSET_SKIPLIST]) + struct.pack("<I", _lru(i)) + struct.pack("<Q", len(pairs)) + b"".join(
        struct.pack("<Q", len(m)) + m + struct.pack("<d", s) for m, s in pairs)


def _check_against_oracle(engine, v, e, a, data_cap=None):
    out, ooffs, t = engine.encode_host(v, e, a, data_cap=data_cap)
    xo, xoffs, xt = cpu.encode(v, e, a, data_cap=data_cap)
    assert np.array_equal(ooffs, xoffs)
    assert t == xt
    n = min(len(out), len(xo))
    if data_cap is not None:
        n = min(n, data_cap)
    assert np.array_equal(out[:n], xo[:n])
    return out, ooffs, t


def test_values_larger_than_a_window(engine):
    """Values of 40-300 KB span many 16 KiB output windows; each window writes only its slice."""
    rng = np.random.default_rng(11)
    blobs = []
    for i in range(12):
        k = i % 4
        if k == 0:
            blobs.append(s_raw(i, rng.integers(0, 256, 40000 + 9973 * i, dtype=np.uint8).tobytes()))
        elif k == 1:
            items = [str(int(x)).encode() if j % 3 == 0 else rng.integers(0, 256, int(rng.integers(0, 90)),
                                                                          dtype=np.uint8).tobytes()
                     for j, x in enumerate(rng.integers(-10**18, 10**18, 5000))]
            blobs.append(l_list(i, items))
        elif k == 2:
            # distinct members (a repeated member would be dropped: desSet de-duplicates)
            blobs.append(s_ht(i, [b""] + [b"%d:" % j + rng.integers(0, 256, int(rng.integers(0, 70)),
                                                                      dtype=np.uint8).tobytes()
                                          for j in range(3001)]))
        else:
            # in serZset's order (descending score, member), as a serialized skiplist is
            pairs = [(rng.integers(65, 91, int(rng.integers(1, 40)), dtype=np.uint8).tobytes(),
                      float(rng.standard_normal())) for _ in range(2000)]
            blobs.append(z_sl(i, sorted(pairs, key=lambda x: (x[1], x[0]), reverse=True)))
        blobs.append(s_raw(i + 100, b"x" * int(rng.integers(0, 50))))   # small neighbours
    data, offs = batch_from_blobs(blobs)
    v, e, a, t = engine.decode_host(data, offs)
    assert t["n_bad"] == 0
    out, ooffs, t2 = _check_against_oracle(engine, v, e, a)
    assert np.array_equal(ooffs, offs)
    assert np.array_equal(out, data[:int(offs[-1])])


def test_relocated_arena_and_permuted_ranges(engine):
    """Descriptor ranges in shuffled order and payloads moved to odd offsets in a new arena:
    the encoder must follow elem_base / data, not assume the decoder's layout."""
    rng = np.random.default_rng(5)
    data, offs = rr.gen_batch(4, 6000, seed=77)
    v, e, a, t = engine.decode_host(data, offs)
    n = len(v)
    order = rng.permutation(n)
    e2 = np.zeros_like(e)
    v2 = v.copy()
    arena2 = bytearray()
    pos = 0
    for i in order:
        b, c = int(v["elem_base"][i]), int(v["n_elems"][i])
        seg = e[b:b + c].copy()
        for k in range(c):
            if seg["kind"][k] in (rr.K_STR, rr.K_ZLRAW):
                ln = int(seg["len"][k])
                arena2 += bytes(int(rng.integers(0, 7)))          # misalign the next payload
                seg["data"][k] = len(arena2)
                src = int(e["data"][b + k])
                arena2 += a[src:src + ln].tobytes()
        e2[pos:pos + c] = seg
        v2["elem_base"][i] = pos
        pos += c
    a2 = np.frombuffer(bytes(arena2) + bytes(16), np.uint8)
    out, ooffs, t2 = _check_against_oracle(engine, v2, e2, a2)
    assert np.array_equal(out, data[:int(offs[-1])])


def test_unencodable_descriptors_and_capacity_cut(engine):
    """Wrong descriptor kinds / intset widths are RR_E_ENCODE (size 0); a data_cap that cuts a
    value leaves it and every later value unwritten, with the same totals as the oracle."""
    data, offs = rr.gen_batch(4, 4000, seed=3)
    v, e, a, t = engine.decode_host(data, offs)
    rng = np.random.default_rng(9)
    e = e.copy()
    for i in rng.choice(len(v), 60, replace=False):
        c = int(v["n_elems"][i])
        if c:
            e["kind"][int(v["elem_base"][i]) + int(rng.integers(0, c))] = rr.K_SCORE
    for cap in (None, int(offs[2000]) + 7, int(offs[len(v) // 3]), 100):
        _check_against_oracle(engine, v, e, a, data_cap=cap)


@pytest.mark.parametrize("cfg,n", [(1, 300000), (2, 20000), (3, 20000), (11, 400)])
def test_encode_configs_match_oracle(engine, cfg, n):
    data, offs = rr.gen_batch(cfg, n)
    v, e, a, t = engine.decode_host(data, offs)
    out, ooffs, t2 = _check_against_oracle(engine, v, e, a)
    assert np.array_equal(out, data[:int(offs[-1])])


def test_encode_rejects_bad_status_and_out_of_range(engine):
    """decode with a short elem_cap, then encode that flat batch: the values that
    got RR_E_CAPACITY (and malformed ones) are unencodable — size 0, counted bad — and no
    descriptor past elem_cap nor payload past arena_cap is read.  Matches the oracle."""
    data, offs = rr.gen_batch(4, 3000, seed=12)
    blobs = [bytes(data[offs[i]:offs[i + 1]]) for i in range(len(offs) - 1)]
    blobs[7] = blobs[7][:3]                      # one malformed value (RR_E_SHORT)
    data, offs = batch_from_blobs(blobs)
    cap = 9000
    v, e, a, t = engine.decode_host(data, offs, elem_cap=cap)
    ov, oe, oa, ot = cpu.decode(data, offs, elem_cap=cap)
    assert t == ot and (v["status"] == 11).any() and v["status"][7] == 1
    _check_against_oracle(engine, v, e, a)
    # descriptors pointing past the arena, and a value whose range passes elem_cap
    v2, e2 = v.copy(), e.copy()
    ok = np.nonzero((v2["status"] == 0) & (v2["n_elems"] > 0))[0]
    for i in ok[:40]:
        k = int(v2["elem_base"][i])
        if e2["kind"][k] in (rr.K_STR, rr.K_ZLRAW):
            e2["data"][k] = len(a) - 2
            e2["len"][k] = 5
    v2["elem_base"][ok[50]] = len(e2) - 1
    out, ooffs, t2 = _check_against_oracle(engine, v2, e2, a)
    assert t2["n_bad"] > t["n_bad"]


def test_windows_with_more_runs_than_the_run_queue(engine):
    """E4 queues one copy run per payload, RR_ENC_RCAP (416) per 16 KiB output window; a window
    of tiny payloads (1-3 byte strings, Lists of 1-byte elements: 2-3K runs per window) takes
    the queue-overflow path for the rest.  Bytes, offsets and totals must equal the oracle's,
    with the decoder's mirror arena (aligned granule copies) and with a relocated one (byte plan),
    and encode(decode(b)) == b."""
    rng = np.random.default_rng(23)
    blobs = []
    for i in range(9000):
        k = i % 3
        if k == 0:
            blobs.append(s_raw(i, bytes(rng.integers(97, 123, int(rng.integers(1, 4)), dtype=np.uint8))))
        elif k == 1:
            items = [bytes([int(rng.integers(97, 123))]) for _ in range(int(rng.integers(1, 40)))]
            blobs.append(l_list(i, items))
        else:
            blobs.append(s_ht(i, [bytes([97 + j]) * int(rng.integers(1, 3))   # (distinct members)
                                  for j in range(int(rng.integers(1, 12)))]))
    data, offs = batch_from_blobs(blobs)
    v, e, a, t = engine.decode_host(data, offs)
    assert t["n_bad"] == 0
    out, ooffs, t2 = _check_against_oracle(engine, v, e, a)
    assert np.array_equal(out, data[:int(offs[-1])])
    # the same payloads one byte further on in a new arena: no run is aligned with its image
    # offset mod 16, so every window takes the byte plan
    e2 = e.copy()
    strs = np.isin(e2["kind"], [rr.K_STR, rr.K_ZLRAW])
    e2["data"][strs] += 1
    a2 = np.concatenate([np.zeros(1, np.uint8), a, np.zeros(16, np.uint8)])
    out2, ooffs2, t3 = _check_against_oracle(engine, v, e2, a2)
    assert np.array_equal(out2, data[:int(offs[-1])])


def _reversed_layout(v, e, a):
    """The same flat batch with the descriptor ranges and the payloads laid out in reverse value
    order: the first values' payloads sit at the arena's end."""
    n = len(v)
    e2 = np.zeros_like(e)
    v2 = v.copy()
    arena2 = bytearray()
    pos = 0
    for i in range(n - 1, -1, -1):
        b, c = int(v["elem_base"][i]), int(v["n_elems"][i])
        seg = e[b:b + c].copy()
        for k in range(c):
            if seg["kind"][k] in (rr.K_STR, rr.K_ZLRAW):
                src, ln = int(e["data"][b + k]), int(seg["len"][k])
                seg["data"][k] = len(arena2)
                arena2 += a[src:src + ln].tobytes()
        e2[pos:pos + c] = seg
        v2["elem_base"][i] = pos
        pos += c
    return v2, e2, np.frombuffer(bytes(arena2) + bytes(16), np.uint8)


@pytest.mark.parametrize("layout", ["mirror", "reversed"])
def test_host_encode_pipelined_matches_one_call(engine, layout):
    """rr_encode_batch_host on inputs past 16 MiB runs in chunks (uploads, encodes and downloads
    overlapped; each chunk waits for the arena prefix its payloads reach): bytes, offsets and
    totals equal the oracle's one-call encode — with the decoder's mirror arena, with a layout
    whose first values' payloads are uploaded last, and with data_caps that cut a value."""
    data, offs = rr.gen_batch(4, 60000, seed=61)
    v, e, a, t = engine.decode_host(data, offs)
    if layout == "reversed":
        v, e, a = _reversed_layout(v, e, a)
    assert len(v) * 16 + len(e) * 16 + len(a) > 16 << 20   # the chunked path
    nb = int(offs[-1])
    out, ooffs, t2 = _check_against_oracle(engine, v, e, a)
    assert np.array_equal(out, data[:nb]) and t2["bytes"] == nb
    for cap in (int(offs[30000]) + 5, int(offs[59000]), nb // 7):
        _check_against_oracle(engine, v, e, a, data_cap=cap)


def test_list_decimals_both_wave_paths(engine):
    """Integer List elements (sdsll2str, sds.c:450-479) through the emit kernel's two decimal
    paths: a wave holding at most 21 integers spreads each one's three 8-digit chunks over three
    lanes, a wave with more writes each on its own lane.  All-integer Lists (every task of a wave an
    integer), Lists mixing integers and strings (a few a wave), a List of 3,000 integers whose
    decimals straddle the 16 KiB output windows, and the boundary values of every chunk: decode
    equal to the oracle, encode(decode(b)) == b byte for byte."""
    rng = np.random.default_rng(2026)
    edges = [0, 1, -1, 9, 10, -10, 99, 100, 10**8 - 1, 10**8, -(10**8), 10**8 + 1, 10**16 - 1, 10**16,
             -(10**16), 10**16 + 7, 2**63 - 1, -(2**63), 1234567890123456789, -999999999999999999]
    def ints(k):
        out = []
        for _ in range(k):
            b = int(rng.integers(0, 64))
            m = int(rng.integers(0, 2**63, dtype=np.uint64)) >> (63 - b) if b else 0
            out.append(-m if rng.integers(0, 2) else m)
        return out
    blobs = []
    for i in range(40):   # all integers: more than 21 a wave
        blobs.append(l_list(i, [str(x).encode() for x in edges + ints(60)]))
    for i in range(40, 80):   # mixed: a few integers a wave
        items = []
        for x in edges[(i % 5):(i % 5) + 6]:
            items += [str(x).encode(), b"s" * int(rng.integers(1, 40)), b"abc-" + str(i).encode()]
        blobs.append(l_list(i, items))
    blobs.append(l_list(80, [str(x).encode() for x in ints(3000) + edges]))   # crosses windows
    data, offs = batch_from_blobs(blobs)
    ov, oe, oa, ot = cpu.decode(data, offs)
    assert (ov["status"] == 0).all()
    v, e, a, t = engine.decode_host(data, offs)
    out, ooffs, t2 = _check_against_oracle(engine, v, e, a)
    assert np.array_equal(ooffs, offs) and np.array_equal(out[:int(offs[-1])], data[:int(offs[-1])])

"""The one-launch small-batch kernels (decode_small_kernel / encode_small_kernel in
rr_kernels.hip): the route of the unchanged per-value callers — desObject per restored key
(rock.c:468), serObject per evicted key (rock.c:691, rock_hotkey.c:347).  Every case runs
through the C-ABI on `engine_small` (default options) and is checked bit for bit against the
CPU oracle, the golden vectors, and the batch pipeline (`engine`, RR_CTX_NO_SMALL) on the same
inputs: records, descriptors, arena, totals, encoded bytes and offsets."""
import struct

import numpy as np
import pytest

import redrock_old_amd as rr
from oracle import cpu

from helpers import assert_flat_equal, batch_from_blobs, expected_flat, golden

pytestmark = pytest.mark.gpu


def _blobs(cfg, n, seed=None):
    data, offs = rr.gen_batch(cfg, n, seed)
    return [bytes(data[offs[i]:offs[i + 1]]) for i in range(n)]


def _fits(blobs):
    return len(blobs) <= rr.SMALL_N and ((sum(len(b) for b in blobs) + 15) & ~15) <= rr.SMALL_BYTES


def _check(engine_small, engine, blobs, what, reencode=True):
    """decode (host path) on the one-launch kernel == oracle == pipeline; encode back."""
    assert _fits(blobs), what
    data, offs = batch_from_blobs(blobs)
    v, e, a, t = engine_small.decode_host(data, offs)
    ov, oe, oa, ot = cpu.decode(data, offs)
    assert_flat_equal((v, e), (ov, oe), what)
    assert t == ot, (what, t, ot)
    assert np.array_equal(a, oa[:len(a)]), what
    pv, pe, pa, pt = engine.decode_host(data, offs)
    assert_flat_equal((v, e), (pv, pe), what + " vs pipeline")
    assert t == pt
    if reencode:   # (an output capacity within the one-launch limit)
        out, ooffs, t2 = engine_small.encode_host(v, e, a, data_cap=int(offs[-1]) + 16)
        xo, xoffs, xt = cpu.encode(ov, oe, oa)
        assert t2 == xt and np.array_equal(ooffs, xoffs) and np.array_equal(out, xo), what
    return v, e, a, t


@pytest.mark.parametrize("cfg", [1, 2, 3, 4, 10])
def test_single_values(engine_small, engine, cfg):
    """n = 1: every value of a batch decoded and encoded on its own (the per-key calls)."""
    for i, b in enumerate(_blobs(cfg, 40 if cfg != 10 else 48, seed=70 + cfg)):
        if not _fits([b]):
            continue
        v, e, a, t = _check(engine_small, engine, [b], f"cfg {cfg} value {i}")
        if cfg != 10:   # (serObject output: it re-encodes to itself)
            out, ooffs, _ = engine_small.encode_host(v, e, a, data_cap=len(b) + 16)
            assert out.tobytes() == b


@pytest.mark.parametrize("cfg", [2, 3, 4, 10])
def test_63_values(engine_small, engine, cfg):
    blobs = [b for b in _blobs(cfg, 2000, seed=63 + cfg)]
    batch, total = [], 0
    for b in blobs:   # the first 63 of at most 2 KiB (they fit the one-launch limits together)
        if len(batch) == 63:
            break
        if len(b) <= 2048 and total + len(b) + 16 <= rr.SMALL_BYTES:
            batch.append(b)
            total += len(b)
    assert len(batch) == 63
    _check(engine_small, engine, batch, f"cfg {cfg} n 63")


@pytest.mark.parametrize("n", [200, 256, 300])
def test_wave_route_limits(engine_small, engine, n):
    """n = 200 and 256 config-4 values of at most 450 bytes: the one-launch kernels' wave-per-value
    route at its limit (SMALL_GW); n = 300 of them averages above SMALL_LANE_BYTES, so the host
    takes the pipeline instead of the lane route — the same results either way."""
    blobs = [b for b in _blobs(4, 3000, seed=256 + n) if len(b) <= 450][:n]
    assert len(blobs) == n
    while not _fits(blobs):
        blobs = blobs[:-1]
    _check(engine_small, engine, blobs, f"n {len(blobs)}")


def test_4096_small_values(engine_small, engine):
    """n = 4096 (the one-launch limit): the config-4 values of at most 30 bytes (INT and
    EMBSTR strings, small intsets / lists / ziplists)."""
    data, offs = rr.gen_batch(4, 40000, seed=4096)
    blobs = [bytes(data[offs[i]:offs[i + 1]]) for i in range(40000) if offs[i + 1] - offs[i] <= 30][:4096]
    assert len(blobs) == 4096
    _check(engine_small, engine, blobs, "n 4096")


def test_golden_vectors(engine_small, engine):
    """The K1-K9 known answers and the edge fixtures (malformed ones included), in batches that
    fit: records against the hand-derived golden flat forms."""
    G = golden()
    fx = [f for f in G["kats"] + G["edges"] if len(bytes.fromhex(f["blob"])) < rr.SMALL_BYTES // 2]
    i = 0
    while i < len(fx):
        part, total = [], 0
        while i < len(fx) and total + len(bytes.fromhex(fx[i]["blob"])) + 16 <= rr.SMALL_BYTES:
            part.append(fx[i])
            total += len(bytes.fromhex(fx[i]["blob"]))
            i += 1
        blobs = [bytes.fromhex(f["blob"]) for f in part]
        data, offs = batch_from_blobs(blobs)
        v, e, a, t = engine_small.decode_host(data, offs)
        assert_flat_equal((v, e), expected_flat(part), "golden")
        _check(engine_small, engine, blobs, "golden vs oracle", reencode=False)


def test_fuzzed_blobs(engine_small, engine):
    """Byte flips and truncations of edge-case values: statuses and descriptors match."""
    rng = np.random.default_rng(11)
    src = [b for b in _blobs(10, 240) if len(b) < 2000]
    blobs = []
    for b in src:
        m = bytearray(b)
        r = rng.integers(0, 3)
        if r == 0 and len(m):
            m[rng.integers(0, len(m))] ^= 1 << int(rng.integers(0, 8))
        elif r == 1 and len(m):
            m = m[:int(rng.integers(0, len(m)))]
        blobs.append(bytes(m))
        if sum(len(x) for x in blobs) > rr.SMALL_BYTES - 4096:
            break
    _check(engine_small, engine, blobs, "fuzz", reencode=False)


def _sl(pairs):
    body = b"".join(struct.pack("<Q", len(m)) + m + struct.pack("<d", s) for m, s in pairs)
    return bytes([5]) + struct.pack("<I", 7) + struct.pack("<Q", len(pairs)) + body


def _ht(members, hash_=False):
    body = b"".join(struct.pack("<Q", len(m)) + m for m in members)
    return bytes([4 if hash_ else 2]) + struct.pack("<I", 3) + struct.pack("<Q", len(members) // (2 if hash_ else 1)) + body


def test_fixups_in_one_launch(engine_small, engine):
    """The marked values — a set with repeated members (first copy kept), a hash with a repeated
    field (RR_E_DUP), an unsorted skiplist (re-sorted), a NaN score (RR_E_NAN), a set of more
    than 16 keys — fixed inside the one-launch kernel."""
    blobs = [_ht([b"a", b"b", b"a", b"c", b"b"]), _ht([b"f", b"1", b"g", b"2", b"f", b"3"], hash_=True),
             _sl([(b"x", 1.0), (b"y", 3.0), (b"z", 2.0)]), _sl([(b"x", 3.0), (b"y", float("nan"))]),
             _ht([b"m%d" % k for k in range(40)] + [b"m7"])]
    blobs += _blobs(4, 30, seed=9)
    v, e, a, t = _check(engine_small, engine, blobs, "fixups", reencode=False)
    assert list(v["status"][:4]) == [0, 13, 0, 14]


def test_device_entry_points(engine_small, engine):
    """rr_decode_batch / rr_encode_batch with device buffers within the limits (data_cap <=
    128 KiB): the one-launch kernels, equal to the pipeline's device calls."""
    import torch
    dev = torch.device("cuda:0")
    blobs = _blobs(4, 200, seed=3)[:100]
    data, offs = batch_from_blobs(blobs)
    n, nb = len(offs) - 1, int(offs[-1])
    cap = rr.elem_bound(n, nb)
    res = []
    for eng in (engine_small, engine):
        d_data = torch.from_numpy(data).to(dev)
        d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
        d_vals = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
        d_elems = torch.zeros(cap * 16, dtype=torch.uint8, device=dev)
        d_arena = torch.zeros(len(data), dtype=torch.uint8, device=dev)
        d_tot = torch.full((4,), -1, dtype=torch.int64, device=dev)
        eng.decode_device(d_data, d_offs, d_vals, d_elems, d_arena, d_tot)
        d_out = torch.zeros(len(data), dtype=torch.uint8, device=dev)
        d_oo = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        d_t2 = torch.full((4,), -1, dtype=torch.int64, device=dev)
        eng.encode_device(d_vals, d_elems, d_arena, d_out, d_oo, d_t2)
        torch.cuda.synchronize()
        res.append([x.cpu().numpy() for x in (d_vals, d_elems, d_arena, d_tot, d_out, d_oo, d_t2)])
    for x, y in zip(res[0], res[1]):
        assert np.array_equal(x, y)
    assert res[0][4][:nb].tobytes() == data[:nb].tobytes()


def test_capacity_cuts(engine_small, engine):
    """elem_cap below the descriptors (RR_E_CAPACITY from the cut on) and data_cap below the
    encoded bytes (values past it not written, their bytes zero): as the pipeline."""
    blobs = _blobs(4, 120, seed=12)
    data, offs = batch_from_blobs(blobs)
    _, oe, _, _ = cpu.decode(data, offs)
    cap = len(oe) // 2
    a1 = engine_small.decode_host(data, offs, elem_cap=cap)
    a2 = engine.decode_host(data, offs, elem_cap=cap)
    assert_flat_equal(a1[:2], a2[:2], "elem_cap cut")
    assert a1[3] == a2[3] and a1[3]["n_bad"] > 0
    v, e, a, _ = engine.decode_host(data, offs)
    dcap = int(offs[60]) + 7
    o1 = engine_small.encode_host(v, e, a, data_cap=dcap)
    o2 = engine.encode_host(v, e, a, data_cap=dcap)
    assert np.array_equal(o1[1], o2[1]) and o1[2] == o2[2] and o1[2]["n_bad"] > 0
    assert o1[0].tobytes()[:dcap] == o2[0].tobytes()[:dcap]


def test_golden_fixtures_one_per_call(engine_small):
    """Every golden fixture (K1-K9 and the edge cases, malformed ones included) as its own n = 1
    call — the route every desObject through the shim takes — against the hand-derived flat form."""
    G = golden()
    for f in G["kats"] + G["edges"]:
        b = bytes.fromhex(f["blob"])
        if not _fits([b]):
            continue
        data, offs = batch_from_blobs([b])
        if data.size == 0:   # (an empty blob: the host entry point wants a data buffer)
            data = np.zeros(16, np.uint8)
        v, e, a, t = engine_small.decode_host(data, offs)
        assert_flat_equal((v, e), expected_flat([f]), f.get("name", "fixture"))


def test_handoff_under_uneven_load(engine_small):
    """The one-launch kernels' completion hand-off (signal_done: every wave's stores
    acknowledged, one system release, the flag) checked while a second context keeps the GPU
    busy with 1M-value pipeline decodes on another stream: host-path decode and encode calls of
    n = 1, 7, 63 and 4096 on one context, every record, descriptor, totals word, encoded byte and
    offset against the oracle (MI355X_MICROARCH.md: test every hand-off under uneven load)."""
    import torch
    dev = torch.device("cuda:0")
    load = rr.Engine(0)
    load.set_options(rr.CTX_NO_SMALL)
    ld, lo = rr.gen_batch(4, 1_000_000, seed=555)
    d_data = torch.from_numpy(ld).to(dev)
    d_offs = torch.from_numpy(lo.view(np.int64)).to(dev)
    ln, lnb = len(lo) - 1, int(lo[-1])
    d_vals = torch.empty(ln * 16, dtype=torch.uint8, device=dev)
    d_elems = torch.empty(rr.elem_bound(ln, lnb) * 16, dtype=torch.uint8, device=dev)
    d_arena = torch.empty(len(ld), dtype=torch.uint8, device=dev)
    d_tot = torch.zeros(4, dtype=torch.int64, device=dev)
    s = torch.cuda.Stream(dev)

    def keep_busy():
        if s.query():   # queue ~50 ms more whenever the loader's stream has drained
            for _ in range(150):
                load.decode_device(d_data, d_offs, d_vals, d_elems, d_arena, d_tot, stream=s)

    # the cases: small batches of config-4 and edge values, with their oracle results
    src = _blobs(4, 20000, seed=71) + _blobs(10, 400, seed=72)
    tiny = [b for b in _blobs(4, 120000, seed=73) if len(b) <= 30]
    cases = []
    for n, pool in ((1, src), (7, src), (63, [b for b in src if len(b) <= 1500]), (4096, tiny)):
        for k in range(3):
            part = pool[k * n:(k + 1) * n]
            while part and not _fits(part):
                part = part[:-1]
            if len(part) < n:
                continue
            data, offs = batch_from_blobs(part)
            ov, oe, oa, ot = cpu.decode(data, offs)
            xo, xoffs, xt = cpu.encode(ov, oe, oa)
            cases.append((f"n {n} #{k}", data, offs, (ov, oe, oa, ot), (xo, xoffs, xt)))
    assert len(cases) == 12
    import time
    checked = busy = 0
    lat = []
    try:
        for rep in range(6):
            for what, data, offs, (ov, oe, oa, ot), (xo, xoffs, xt) in cases:
                keep_busy()
                t0 = time.perf_counter()
                v, e, a, t = engine_small.decode_host(data, offs)
                lat.append(time.perf_counter() - t0)
                assert_flat_equal((v, e), (ov, oe), what)
                assert t == ot, (what, rep, t, ot)
                if int(offs[-1]) + 16 <= rr.SMALL_BYTES:
                    out, ooffs, t2 = engine_small.encode_host(ov, oe, oa, data_cap=int(offs[-1]) + 16)
                    assert t2 == xt and np.array_equal(ooffs, xoffs) and np.array_equal(out, xo), (what, rep)
                busy += not s.query()   # (the loader still had work queued when the call returned)
                checked += 1
    finally:
        s.synchronize()
        load.close()
    assert checked == 6 * len(cases)
    # (how many calls returned while the load was still queued depends on host launch speed
    # against the GPU's drain rate, not on correctness: reported, not asserted — ADVICE r5)
    print(f"decode calls beside the load: median {1e6 * sorted(lat)[len(lat) // 2]:.1f} us, max {1e6 * max(lat):.1f} us; "
          f"{busy} of {checked} returned while the load was still queued")


def test_failed_second_launch_resets_sums(engine):
    """A pipeline call that stops after its first kernel (a failed second launch, an aborted
    stream) leaves the zero-between-calls window/group sums non-zero; the context re-zeroes
    them before its next call, so later decodes and encodes are still exact."""
    data, offs = rr.gen_batch(4, 20000, seed=31)
    ov, oe, oa, ot = cpu.decode(data, offs)
    engine.decode_host(data, offs)   # (the sums sized for this batch)
    engine.debug_fail_second()
    with pytest.raises(rr.RRError):
        engine.decode_host(data, offs)
    v, e, a, t = engine.decode_host(data, offs)
    assert_flat_equal((v, e), (ov, oe), "decode after a withheld second launch")
    assert t == ot
    xo, xoffs, xt = cpu.encode(ov, oe, oa)
    engine.debug_fail_second()
    with pytest.raises(rr.RRError):
        engine.encode_host(v, e, a)
    out, ooffs, t2 = engine.encode_host(v, e, a)
    assert t2 == xt and np.array_equal(ooffs, xoffs) and np.array_equal(out, xo)
    v, e, a, t = engine.decode_host(data, offs)   # (and the decode after the encode's failure)
    assert_flat_equal((v, e), (ov, oe), "decode after a withheld encode launch")


@pytest.mark.parametrize("cfg,n", [(1, 100000), (4, 30000), (3, 20000), (2, 6000)])
def test_one_launch_help_path(engine, cfg, n):
    """The one-launch decode (decode_kernel's ONE form, a batch of one window generation): with
    the test hook every window sums all earlier windows itself (one_window_sum, the look-back's
    help for windows whose workgroups have not started) instead of reading their words; the
    records, descriptors, arena and totals equal the oracle's, and the next call (no hook) is
    exact too, so the call left its words zero."""
    data, offs = rr.gen_batch(cfg, n, seed=97 + cfg)
    ov, oe, oa, ot = cpu.decode(data, offs)
    for hook in (True, False):
        if hook:
            engine.debug_one_help()
        v, e, a, t = engine.decode_host(data, offs)
        assert_flat_equal((v, e), (ov, oe), f"cfg {cfg} help {hook}")
        assert t == ot and np.array_equal(a, oa[:len(a)]), (cfg, hook)

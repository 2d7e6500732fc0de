"""Sharding across ranks through the C library's own plan, placement and
rebase: rr_shard_plan (the rule shard_plan_kernel runs for rr_split_plan), rr_gather_layout
(where rr_gather puts each shard's descriptors) and rr_flat_rebase_host / rr_flat_rebase (the
placement flat_rebase_kernel applies on the root).  CPU tests: gloo with world sizes 2 and 3
running the C library's own transfer schedules (rr_split_schedule / rr_gather_schedule: the
exact lists rr_split and rr_gather post inside their ncclGroup), the C oracle as the per-shard
decoder (the checker stands in for the device on CPU).
GPU tests: every shard decoded through the HIP C-ABI, placed by the device rebase, and the RCCL
entry points with one rank."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import redrock_old_amd as rr
from oracle import cpu

from helpers import assert_flat_equal


def _whole(cfg, n, seed=None):
    data, offs = rr.gen_batch(cfg, n, seed)
    v, e, _, _ = cpu.decode(data, offs)
    return data, offs, v, e


def shard_of(data, offsets, lo, hi):
    """What rr_split hands rank k: values [lo, hi)'s bytes in a zero-padded 16-aligned buffer
    and their offsets rebased to 0 (offsets_rebase_kernel)."""
    offsets = np.asarray(offsets, np.uint64)
    b0, b1 = int(offsets[lo]), int(offsets[hi])
    buf = np.zeros((b1 - b0 + 15) & ~15, np.uint8)
    buf[: b1 - b0] = data[b0:b1]
    return buf, (offsets[lo: hi + 1] - offsets[lo]).astype(np.uint64)


def place(plan, parts, n):
    """The root's placement of decoded shards (values, elems) — rr_gather's layout and rebase,
    through the C library's host forms."""
    at, tot = rr.gather_layout([len(e) for _, e in parts])
    vals = np.zeros(n, rr.VALUE_DT)
    els = np.zeros(tot, rr.ELEM_DT)
    for k, (sv, se) in enumerate(parts):
        v0, v1, b0 = int(plan[k][0]), int(plan[k][1]), int(plan[k][2])
        dv = np.array(sv, rr.VALUE_DT, copy=True)
        de = np.array(se, rr.ELEM_DT, copy=True)
        rr.flat_rebase_host(dv, de, int(at[k]), b0)
        vals[v0:v1] = dv
        els[int(at[k]):int(at[k]) + len(de)] = de
    return vals, els


@pytest.mark.parametrize("g", [1, 2, 3, 8])
def test_plan_balanced(g):
    data, offs = rr.gen_batch(4, 5000)
    plan = rr.shard_plan(offs, g)
    assert plan[0, 0] == 0 and plan[-1, 1] == 5000 and (plan[1:, 0] == plan[:-1, 1]).all()
    total = int(offs[-1])
    sizes = (plan[:, 3] - plan[:, 2]).astype(np.int64)
    assert int(sizes.sum()) == total
    big = int(np.max(np.diff(offs.astype(np.int64))))
    for s in sizes:   # each shard within one value of the even split
        assert abs(int(s) - total / g) <= big + 1
    for k in range(g):   # shard k starts at the first value at or after k * total / g
        t = (total * k) // g
        v0 = int(plan[k, 0])
        assert k == 0 or (int(offs[v0]) >= t and (v0 == 0 or int(offs[v0 - 1]) < t))


def test_plan_edges():
    plan = rr.shard_plan(np.zeros(1, np.uint64), 4)
    assert (plan == 0).all()
    offs = np.array([0, 100], np.uint64)   # one value: it lands in one shard
    plan = rr.shard_plan(offs, 3)
    assert plan[0, 0] == 0 and plan[-1, 1] == 1 and int((plan[:, 1] - plan[:, 0]).sum()) == 1


def test_gather_layout_and_32bit_guard():
    at, tot = rr.gather_layout([5, 0, 7, 1])
    assert list(at) == [0, 5, 5, 12] and tot == 13
    with pytest.raises(rr.RRError):
        rr.gather_layout([2 ** 31, 2 ** 31])   # past 2^32 - 1: elem_base is 32-bit
    v = np.zeros(1, rr.VALUE_DT)
    e = np.zeros(1, rr.ELEM_DT)
    with pytest.raises(rr.RRError):
        rr.flat_rebase_host(v, e, 2 ** 32 - 1, 0)
    rr.flat_rebase_host(v, e, 2 ** 32 - 2, 16)
    assert int(v[0]["elem_base"]) == 2 ** 32 - 2 and int(e[0]["data"]) == 0   # zero slots stay zero


@pytest.mark.parametrize("cfg,g", [(4, 2), (4, 5), (10, 3), (3, 4)])
def test_rebase_equals_whole_decode(cfg, g):
    data, offs, v, e = _whole(cfg, 3000 if cfg != 10 else 600)
    n = len(offs) - 1
    plan = rr.shard_plan(offs, g)
    parts = []
    for k in range(g):
        d, o = shard_of(data, offs, int(plan[k, 0]), int(plan[k, 1]))
        assert len(d) % 16 == 0
        sv, se, _, _ = cpu.decode(d, o)
        parts.append((sv, se))
    assert_flat_equal(place(plan, parts, n), (v, e), f"cfg {cfg} g {g}")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy())


def _run_schedule(xfers, bufs):
    """Post a C transfer schedule over gloo (isend / irecv, all in flight, as inside rr_split's
    ncclGroup), then land the received bytes in their buffers."""
    ops, landing = [], []
    for peer, direction, buf, off, nbytes in xfers:
        view = bufs[buf][off:off + nbytes]
        assert len(view) == nbytes, (buf, off, nbytes, len(bufs[buf]))
        if direction == rr.XFER_SEND:
            ops.append(dist.isend(torch.from_numpy(view.copy()), peer))
        else:
            t = torch.empty(nbytes, dtype=torch.uint8)
            ops.append(dist.irecv(t, peer))
            landing.append((view, t))
    for op in ops:
        op.wait()
    for view, t in landing:
        view[:] = t.numpy()


def _worker(rank, world, port, cfg, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        root = 0
        data = offs = None
        # rr_split_plan: the root plans (rr_shard_plan), every rank gets the plan
        plan_t = torch.zeros(world * 4, dtype=torch.int64)
        if rank == root:
            data, offs = rr.gen_batch(cfg, n)
            plan_t.copy_(torch.from_numpy(rr.shard_plan(offs, world).view(np.int64).reshape(-1)))
        dist.broadcast(plan_t, root)
        plan = plan_t.numpy().view(np.uint64).reshape(world, 4)
        v0, v1, b0, b1 = (int(x) for x in plan[rank])
        # rr_split: the C schedule, then the root's own shard by a local copy and the rebase of
        # the offsets to 0 (offsets_rebase_kernel)
        bufs = {rr.BUF_MINE_DATA: np.zeros((b1 - b0 + 15) & ~15, np.uint8),
                rr.BUF_MINE_OFFSETS: np.zeros((v1 - v0 + 1) * 8, np.uint8)}
        if rank == root:
            bufs[rr.BUF_WHOLE_DATA] = data
            bufs[rr.BUF_WHOLE_OFFSETS] = offs.view(np.uint8)
            bufs[rr.BUF_MINE_DATA][: b1 - b0] = data[b0:b1]
            bufs[rr.BUF_MINE_OFFSETS][:] = offs[v0:v1 + 1].view(np.uint8)
        _run_schedule(rr.split_schedule(plan, rank, root), bufs)
        d = bufs[rr.BUF_MINE_DATA]
        o = bufs[rr.BUF_MINE_OFFSETS].view(np.uint64) - np.uint64(b0)
        sv, se, _, _ = cpu.decode(d, o)
        # rr_gather: all-gather of the descriptor counts, the C schedule (peers send records +
        # descriptors, the root receives them at their places), the root's own shard copied in,
        # then every shard rebased at its place (rr_gather_layout, rr_flat_rebase_host)
        ne = torch.zeros(world, dtype=torch.int64)
        dist.all_gather_into_tensor(ne, torch.tensor([len(se)], dtype=torch.int64))
        ne = [int(x) for x in ne]
        bufs = {rr.BUF_MINE_VALUES: np.ascontiguousarray(sv).view(np.uint8).reshape(-1),
                rr.BUF_MINE_ELEMS: np.ascontiguousarray(se).view(np.uint8).reshape(-1)}
        if rank == root:
            at, tot = rr.gather_layout(ne)
            wv = np.zeros(n, rr.VALUE_DT)
            we = np.zeros(tot, rr.ELEM_DT)
            wv[v0:v1] = sv
            we[int(at[root]):int(at[root]) + len(se)] = se
            bufs[rr.BUF_WHOLE_VALUES] = wv.view(np.uint8).reshape(-1)
            bufs[rr.BUF_WHOLE_ELEMS] = we.view(np.uint8).reshape(-1)
        _run_schedule(rr.gather_schedule(plan, ne, rank, root), bufs)
        if rank == root:
            for k in range(world):
                kv0, kv1, kb0 = int(plan[k, 0]), int(plan[k, 1]), int(plan[k, 2])
                ea = int(at[k])
                rr.flat_rebase_host(wv[kv0:kv1], we[ea:ea + ne[k]], ea, kb0)
            xv, xe, _, _ = cpu.decode(data, offs)
            assert_flat_equal((wv, we), (xv, xe), f"split/gather cfg {cfg} world {world}")
        q.put((rank, "ok", v0, v1 - v0))
    except Exception as ex:   # report to the parent
        q.put((rank, repr(ex), -1, -1))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cfg,n,world", [(4, 4000, 2), (10, 300, 2), (10, 0, 2), (2, 700, 2), (4, 3000, 3),
                                         (10, 2, 3)])
def test_split_gather_gloo(cfg, n, world):
    """The C schedules run over gloo; (10, 2, 3): two values over three ranks, so a shard is empty."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cfg, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert [r[1] for r in res] == ["ok"] * world, res
    assert res[0][2] == 0 and sum(r[3] for r in res) == n
    assert all(res[k + 1][2] == res[k][2] + res[k][3] for k in range(world - 1))
    if (cfg, n, world) == (10, 2, 3):
        assert any(r[3] == 0 for r in res)


def test_schedules_pair_up():
    """Every send one rank's schedule posts is a receive of the same size in its peer's, in the
    same order per pair (what lets ncclGroup and gloo match them)."""
    for g, n in [(1, 100), (3, 1000), (8, 5000), (4, 2)]:
        _, offs = rr.gen_batch(4, n)
        plan = rr.shard_plan(offs, g)
        ne = [int(x) for x in np.random.default_rng(g).integers(0, 500, g)]
        for root in range(g):
            for sched in (lambda r: rr.split_schedule(plan, r, root), lambda r: rr.gather_schedule(plan, ne, r, root)):
                lists = {r: sched(r) for r in range(g)}
                for r in range(g):
                    for peer in range(g):
                        sends = [x[4] for x in lists[r] if x[0] == peer and x[1] == rr.XFER_SEND]
                        recvs = [x[4] for x in lists[peer] if x[0] == r and x[1] == rr.XFER_RECV]
                        assert sends == recvs, (g, root, r, peer)
                assert all(x[4] > 0 for xs in lists.values() for x in xs)   # no zero-byte transfer
    with pytest.raises(rr.RRError):   # a gather placed past 2^32 - 1 descriptors
        rr.gather_schedule(rr.shard_plan(np.array([0, 1, 2], np.uint64), 2), [2 ** 31, 2 ** 31], 0, 0)


@pytest.mark.gpu
def test_sharded_device_decode_equals_whole(engine):
    """Every shard decoded by the HIP engine, rebased, equals the engine's whole-batch decode
    and the oracle's."""
    data, offs, v, e = _whole(4, 20000)
    plan = rr.shard_plan(offs, 4)
    parts = []
    for k in range(4):
        d, o = shard_of(data, offs, int(plan[k, 0]), int(plan[k, 1]))
        sv, se, _, _ = engine.decode_host(d, o)
        parts.append((sv, se))
    assert_flat_equal(place(plan, parts, len(offs) - 1), (v, e), "sharded HIP decode")


@pytest.mark.parametrize("g", [2, 7])
def test_rebase_with_malformed_values(g):
    """Golden fixtures (valid + malformed, whose reserved slots are zero-filled) repeated over
    shards: the rebased shard decodes equal the expected whole-batch flat form."""
    from helpers import batch_from_blobs, expected_flat, golden
    fx = (golden()["kats"] + golden()["edges"]) * 3
    data, offs = batch_from_blobs([bytes.fromhex(f["blob"]) for f in fx])
    assert any(f["value"].get("status", 0) for f in fx)
    plan = rr.shard_plan(offs, g)
    parts = []
    for k in range(g):
        d, o = shard_of(data, offs, int(plan[k, 0]), int(plan[k, 1]))
        sv, se, _, _ = cpu.decode(d, o)
        parts.append((sv, se))
    assert_flat_equal(place(plan, parts, len(offs) - 1), expected_flat(fx), f"golden g {g}")


@pytest.mark.parametrize("n,g", [(5000, 1), (5000, 3), (5000, 8), (3, 8), (0, 4), (1, 3)])
def test_c_shard_plan_rule(n, g):
    """rr_shard_plan (the rule shard_plan_kernel runs on the device for rr_split_plan): shard k
    starts at the first value whose first byte is at or after floor(total * k / g)."""
    _, offs = rr.gen_batch(4, n) if n else (None, np.zeros(1, np.uint64))
    plan = rr.shard_plan(offs, g)
    total = int(offs[-1])
    targets = np.array([(total * k) // g for k in range(g + 1)], np.uint64)
    cuts = np.searchsorted(offs[:n], targets, side="left").astype(np.int64)
    cuts[0], cuts[-1] = 0, n
    cuts = np.maximum.accumulate(cuts)
    assert (plan[:, 0] == cuts[:-1]).all() and (plan[:, 1] == cuts[1:]).all()
    assert (plan[:, 2] == offs[cuts[:-1]]).all() and (plan[:, 3] == offs[cuts[1:]]).all()


def _device_shards(engine, data, offs, g, torch_dev):
    """Decode each shard on the device; returns whole-sized (values, elems) tensors with every
    shard copied to its place and rebased by rr_flat_rebase, and the total descriptor count."""
    n = len(offs) - 1
    plan = rr.shard_plan(offs, g)
    parts, ne_tot = [], 0
    for k in range(g):
        v0, v1, b0, b1 = (int(x) for x in plan[k])
        d, o = shard_of(data, offs, v0, v1)
        nv, nb = v1 - v0, b1 - b0
        cap = rr.elem_bound(nv, nb)
        t_vals = torch.zeros(max(nv, 1) * 16, dtype=torch.uint8, device=torch_dev)[:nv * 16]
        t_elems = torch.zeros(max(cap, 1) * 16, dtype=torch.uint8, device=torch_dev)
        t_arena = torch.zeros(max(len(d), 16), dtype=torch.uint8, device=torch_dev)
        t_tot = torch.zeros(4, dtype=torch.int64, device=torch_dev)
        engine.decode_device(torch.from_numpy(d).to(torch_dev), torch.from_numpy(o.view(np.int64)).to(torch_dev),
                             t_vals, t_elems, t_arena, t_tot)
        ne = int(t_tot[0].item())
        parts.append((t_vals, t_elems[:ne * 16], ne, b0))
        ne_tot += ne
    w_vals = torch.zeros(max(n, 1) * 16, dtype=torch.uint8, device=torch_dev)
    w_elems = torch.zeros(max(ne_tot, 1) * 16, dtype=torch.uint8, device=torch_dev)
    at, tot = rr.gather_layout([p[2] for p in parts])   # rr_gather's placement
    assert tot == ne_tot
    for k, (t_vals, t_elems, ne, b0) in enumerate(parts):
        v0, v1, eb = int(plan[k][0]), int(plan[k][1]), int(at[k])
        dv, de = w_vals[v0 * 16:v1 * 16], w_elems[eb * 16:(eb + ne) * 16]
        dv.copy_(t_vals)
        de.copy_(t_elems)
        engine.flat_rebase(dv, de, eb, b0)
    torch.cuda.synchronize()
    return w_vals[:n * 16], w_elems[:ne_tot * 16]


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,n,g", [(4, 20000, 4), (10, 500, 3), (4, 2000, 7)])
def test_device_rebase_equals_whole(engine, cfg, n, g):
    """Shards decoded on the device and placed by the device rebase (rr_flat_rebase, the step
    rr_gather runs on the root) equal the whole batch's oracle decode."""
    data, offs, v, e = _whole(cfg, n)
    w_vals, w_elems = _device_shards(engine, data, offs, g, torch.device("cuda:0"))
    got = (w_vals.cpu().numpy().view(rr.VALUE_DT), w_elems.cpu().numpy().view(rr.ELEM_DT))
    assert_flat_equal(got, (v, e), f"device rebase cfg {cfg} g {g}")


@pytest.mark.gpu
def test_device_rebase_golden_malformed(engine):
    from helpers import batch_from_blobs, expected_flat, golden
    fx = (golden()["kats"] + golden()["edges"]) * 3
    data, offs = batch_from_blobs([bytes.fromhex(f["blob"]) for f in fx])
    w_vals, w_elems = _device_shards(engine, data, offs, 5, torch.device("cuda:0"))
    got = (w_vals.cpu().numpy().view(rr.VALUE_DT), w_elems.cpu().numpy().view(rr.ELEM_DT))
    assert_flat_equal(got, expected_flat(fx), "device rebase golden")


@pytest.mark.gpu
def test_rccl_split_gather_single_rank(engine):
    """rr_comm over RCCL with one rank (the box has one GPU; the N>1 data movement is the same
    ncclSend/Recv calls, rehearsed over gloo above): split_plan -> split -> decode -> gather
    equals the whole decode."""
    dev = torch.device("cuda:0")
    data, offs, v, e = _whole(4, 30000)
    n, nb = len(offs) - 1, int(offs[-1])
    comm = rr.Comm(engine, 1, 0, rr.Comm.new_id())
    try:
        d_data = torch.from_numpy(data).to(dev)
        d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
        plan = comm.split_plan(d_data, d_offs, root=0)
        assert (plan[0].v0, plan[0].v1, plan[0].b0, plan[0].b1) == (0, n, 0, nb)
        m_data = torch.full(((nb + 15) & ~15,), 0xAB, dtype=torch.uint8, device=dev)
        m_offs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        assert comm.split(plan, d_data, d_offs, m_data, m_offs, root=0) == n
        torch.cuda.synchronize()
        assert torch.equal(m_data[:nb].cpu(), d_data[:nb].cpu()) and torch.equal(m_offs.cpu(), d_offs.cpu())
        assert int(m_data[nb:].sum().item()) == 0   # the tail padding is zeroed
        cap = rr.elem_bound(n, nb)
        t_vals = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
        t_elems = torch.zeros(cap * 16, dtype=torch.uint8, device=dev)
        t_arena = torch.zeros(len(data), dtype=torch.uint8, device=dev)
        t_tot = torch.zeros(4, dtype=torch.int64, device=dev)
        engine.decode_device(m_data, m_offs, t_vals, t_elems, t_arena, t_tot)
        ne = int(t_tot[0].item())
        w_vals = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
        w_elems = torch.zeros(ne * 16, dtype=torch.uint8, device=dev)
        comm.gather(plan, t_vals, t_elems, ne, w_vals, w_elems, root=0)
        torch.cuda.synchronize()
        got = (w_vals.cpu().numpy().view(rr.VALUE_DT), w_elems.cpu().numpy().view(rr.ELEM_DT))
        assert_flat_equal(got, (v, e), "rccl single-rank split/gather")
    finally:
        comm.close()

"""Sharding across ranks: byte-balanced partition, offset/elem_base rebase,
root split/gather over torch.distributed.  CPU tests use gloo with world_size 2 and the C
oracle as the per-shard decoder (the checker stands in for the device here; the GPU test at
the bottom decodes every shard through the HIP C-ABI)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import redrock_old_amd as rr
from redrock_old_amd import shard
from oracle import cpu

from helpers import assert_flat_equal


def _whole(cfg, n, seed=None):
    data, offs = rr.gen_batch(cfg, n, seed)
    v, e, _, _ = cpu.decode(data, offs)
    return data, offs, v, e


@pytest.mark.parametrize("g", [1, 2, 3, 8])
def test_partition_balanced(g):
    data, offs = rr.gen_batch(4, 5000)
    cuts = shard.partition(offs, g)
    assert cuts[0] == 0 and cuts[-1] == 5000 and np.all(np.diff(cuts) >= 0)
    total = int(offs[-1])
    sizes = [int(offs[cuts[k + 1]] - offs[cuts[k]]) for k in range(g)]
    assert sum(sizes) == total
    big = int(np.max(np.diff(offs.astype(np.int64))))
    for s in sizes:   # each shard within one value of the even split
        assert abs(s - total / g) <= big + 1


def test_partition_edges():
    assert list(shard.partition(np.zeros(1, np.uint64), 4)) == [0, 0, 0, 0, 0]
    offs = np.array([0, 100], np.uint64)   # one value: it lands in one shard
    cuts = shard.partition(offs, 3)
    assert cuts[0] == 0 and cuts[-1] == 1


@pytest.mark.parametrize("cfg,g", [(4, 2), (4, 5), (10, 3), (3, 4)])
def test_rebase_equals_whole_decode(cfg, g):
    data, offs, v, e = _whole(cfg, 3000 if cfg != 10 else 600)
    n = len(offs) - 1
    cuts = shard.partition(offs, g)
    parts = []
    for k in range(g):
        d, o = shard.shard_of(data, offs, int(cuts[k]), int(cuts[k + 1]))
        assert len(d) % 16 == 0
        sv, se, _, _ = cpu.decode(d, o)
        parts.append((sv, se, int(offs[cuts[k]])))
    got = shard.rebase_flat(parts)
    assert len(got[0]) == n
    assert_flat_equal(got, (v, e), f"cfg {cfg} g {g}")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, cfg, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cpu")
        data = offs = None
        if rank == 0:
            data, offs = rr.gen_batch(cfg, n)
        d, o, lo, b0 = shard.split(dist, torch, dev, data, offs)
        sv, se, _, _ = cpu.decode(d, o)
        out = shard.gather(dist, torch, dev, sv, se, b0)
        if rank == 0:
            wv, we, _, _ = cpu.decode(data, offs)
            assert_flat_equal(out, (wv, we), f"split/gather cfg {cfg}")
        q.put((rank, "ok", lo, len(o) - 1))
    except Exception as ex:   # report to the parent
        q.put((rank, repr(ex), -1, -1))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cfg,n", [(4, 4000), (10, 300), (10, 0), (2, 700)])
def test_split_gather_gloo_world2(cfg, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, cfg, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert [r[1] for r in res] == ["ok", "ok"], res
    assert res[0][2] == 0 and res[0][3] + res[1][3] == n and res[1][2] == res[0][3]


@pytest.mark.gpu
def test_sharded_device_decode_equals_whole(engine):
    """Every shard decoded by the HIP engine, rebased, equals the engine's whole-batch decode
    and the oracle's."""
    data, offs, v, e = _whole(4, 20000)
    cuts = shard.partition(offs, 4)
    parts = []
    for k in range(4):
        d, o = shard.shard_of(data, offs, int(cuts[k]), int(cuts[k + 1]))
        sv, se, _, _ = engine.decode_host(d, o)
        parts.append((sv, se, int(offs[cuts[k]])))
    assert_flat_equal(shard.rebase_flat(parts), (v, e), "sharded HIP decode")


@pytest.mark.parametrize("g", [2, 7])
def test_rebase_with_malformed_values(g):
    """Golden fixtures (valid + malformed, whose reserved slots are zero-filled) repeated over
    shards: the rebased shard decodes equal the expected whole-batch flat form."""
    from helpers import batch_from_blobs, expected_flat, golden
    fx = (golden()["kats"] + golden()["edges"]) * 3
    data, offs = batch_from_blobs([bytes.fromhex(f["blob"]) for f in fx])
    assert any(f["value"].get("status", 0) for f in fx)
    cuts = shard.partition(offs, g)
    parts = []
    for k in range(g):
        d, o = shard.shard_of(data, offs, int(cuts[k]), int(cuts[k + 1]))
        sv, se, _, _ = cpu.decode(d, o)
        parts.append((sv, se, int(offs[cuts[k]])))
    assert_flat_equal(shard.rebase_flat(parts), expected_flat(fx), f"golden g {g}")

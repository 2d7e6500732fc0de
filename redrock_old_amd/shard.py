"""Multi-GPU sharding of blob batches.

Values are independent, so a batch shards into contiguous value ranges with no exchange in the
compute: each rank decodes / encodes its own shard with the single-GPU entry points.  What
remains is bookkeeping, done here on the host side:

  partition      cut a batch into G contiguous value ranges balanced by blob bytes (exclusive
                 prefix of |blob_i| cut at k*Σ/G);
  shard_of       the shard's blob bytes (copied to a 16-byte aligned buffer, the decode
                 alignment rule of rr_serdes.h) and its offsets rebased to 0;
  rebase_flat    turn per-shard flat outputs into the whole batch's flat form: elem_base +=
                 descriptors of earlier shards, STR/ZLRAW arena offsets += blob bytes of earlier
                 shards (the arena mirrors the blob buffer, so the shard's arena is exactly the
                 slice of the whole arena);
  split / gather the optional root scatter / gather over torch.distributed (RCCL over xGMI on
                 GPUs, gloo in the CPU tests) for batches that start or must end on one rank.
                 The per-shard sizes travel in one all_gather of 3 words per rank.

The bench runs pre-sharded (each rank's batch is generated in place), so its timed region
holds no collective at all.
"""
from __future__ import annotations

import numpy as np

from . import ELEM_DT, K_STR, K_ZLRAW, VALUE_DT


def partition(offsets: np.ndarray, g: int) -> np.ndarray:
    """Value-index cut points c[0..g] (c[0] = 0, c[g] = n): shard k = values [c[k], c[k+1]).
    Shard k starts at the first value whose first byte is at or after k*Σ/G."""
    offsets = np.asarray(offsets, np.uint64)
    n = len(offsets) - 1
    total = int(offsets[-1])
    targets = np.array([(total * k) // g for k in range(g + 1)], np.uint64)
    cuts = np.searchsorted(offsets[:n], targets, side="left").astype(np.int64)
    cuts[0], cuts[-1] = 0, n
    return np.maximum.accumulate(cuts)


def shard_of(data: np.ndarray, offsets: np.ndarray, lo: int, hi: int):
    """(data, offsets) of values [lo, hi): bytes copied to a zero-padded 16-aligned buffer."""
    offsets = np.asarray(offsets, np.uint64)
    b0, b1 = int(offsets[lo]), int(offsets[hi])
    buf = np.zeros((b1 - b0 + 15) & ~15, np.uint8)
    buf[: b1 - b0] = data[b0:b1]
    return buf, (offsets[lo: hi + 1] - offsets[lo]).astype(np.uint64)


def rebase_flat(shards):
    """shards: list of (values, elems, byte_base) per shard in order, elems holding exactly the
    shard's descriptor slots.  Returns the whole batch's (values, elems)."""
    vals, els = [], []
    ebase = 0
    for values, elems, byte_base in shards:
        v = np.array(values, dtype=VALUE_DT, copy=True)
        e = np.array(elems, dtype=ELEM_DT, copy=True)
        v["elem_base"] += np.uint32(ebase)
        arena_ref = (e["kind"] == K_STR) | (e["kind"] == K_ZLRAW)
        # zero-filled slots of malformed values carry data 0 and kind STR: keep them zero
        arena_ref &= (e["data"] != 0) | (e["len"] != 0)
        e["data"][arena_ref] += np.uint64(byte_base)
        vals.append(v)
        els.append(e)
        ebase += len(e)
    return (np.concatenate(vals) if vals else np.zeros(0, VALUE_DT),
            np.concatenate(els) if els else np.zeros(0, ELEM_DT))


# ---- torch.distributed split / gather -----------------------------------------------------
def _sizes(dist, torch, device, words):
    t = torch.tensor(words, dtype=torch.int64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [[int(x) for x in o.cpu().tolist()] for o in out]


def split(dist, torch, device, data=None, offsets=None, root: int = 0):
    """Root holds the whole batch (numpy); every rank returns its shard (numpy data, offsets)
    and the shard's first value index and byte base in the whole batch."""
    rank, g = dist.get_rank(), dist.get_world_size()
    if rank == root:
        cuts = partition(offsets, g)
        plan = [[int(cuts[k]), int(cuts[k + 1]), int(offsets[cuts[k]]), int(offsets[cuts[k + 1]])]
                for k in range(g)]
        flat = torch.tensor(sum(plan, []), dtype=torch.int64, device=device)
    else:
        flat = torch.zeros(4 * g, dtype=torch.int64, device=device)
    dist.broadcast(flat, root)
    plan = np.array(flat.cpu().tolist(), np.int64).reshape(g, 4)
    lo, hi, b0, b1 = (int(x) for x in plan[rank])
    nbytes = (b1 - b0 + 15) & ~15
    if rank == root:
        for k in range(g):
            if k == root:
                continue
            klo, khi = int(plan[k][0]), int(plan[k][1])
            d, o = shard_of(data, offsets, klo, khi)
            if d.size:
                dist.send(torch.from_numpy(d).to(device), k)
            dist.send(torch.from_numpy(o.view(np.int64)).to(device), k)
        d, o = shard_of(data, offsets, lo, hi)
    else:
        td = torch.empty(nbytes, dtype=torch.uint8, device=device)
        if nbytes:
            dist.recv(td, root)
        to = torch.empty(hi - lo + 1, dtype=torch.int64, device=device)
        dist.recv(to, root)
        d, o = td.cpu().numpy(), to.cpu().numpy().view(np.uint64)
    return d, o, lo, b0


def gather(dist, torch, device, values, elems, byte_base: int, root: int = 0):
    """Every rank passes its decoded shard (numpy values, elems with exactly its slots);
    root returns the whole batch's rebased (values, elems), other ranks None."""
    rank, g = dist.get_rank(), dist.get_world_size()
    sizes = _sizes(dist, torch, device, [len(values), len(elems), byte_base])
    if rank != root:
        if len(values):
            dist.send(torch.from_numpy(np.ascontiguousarray(values).view(np.uint8)).to(device), root)
        if len(elems):
            dist.send(torch.from_numpy(np.ascontiguousarray(elems).view(np.uint8)).to(device), root)
        return None
    parts = []
    for k in range(g):
        nv, ne, bb = sizes[k]
        if k == root:
            parts.append((values, elems, bb))
            continue
        tv = torch.empty(nv * 16, dtype=torch.uint8, device=device)
        if nv:
            dist.recv(tv, k)
        te = torch.empty(ne * 16, dtype=torch.uint8, device=device)
        if ne:
            dist.recv(te, k)
        parts.append((tv.cpu().numpy().view(VALUE_DT), te.cpu().numpy().view(ELEM_DT), bb))
    return rebase_flat(parts)

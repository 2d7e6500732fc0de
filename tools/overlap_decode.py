"""Diagnostics: do two decode calls on two streams overlap?  Times K calls of A then B serially
on one stream against A on stream 1 beside B on stream 2 (two engine contexts, separate outputs).
Usage (GPU box): python tools/overlap_decode.py [config] [n] [K]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import redrock_old_amd as rr  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
K = int(sys.argv[3]) if len(sys.argv) > 3 else 20
data, offs = rr.gen_batch(cfg, n)
nb = int(offs[-1])
dev = torch.device("cuda:0")
d_data = torch.from_numpy(data).to(dev)
d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
cap = rr.elem_bound(n, nb)


def outputs():
    return (torch.empty(n * 16, dtype=torch.uint8, device=dev), torch.empty(cap * 16, dtype=torch.uint8, device=dev),
            torch.empty((nb + 15) & ~15, dtype=torch.uint8, device=dev), torch.zeros(4, dtype=torch.int64, device=dev))


engA, engB = rr.Engine(0), rr.Engine(0)
engA.reserve(n, nb)
engB.reserve(n, nb)
oA, oB = outputs(), outputs()
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def run(serial):
    for _ in range(K):
        engA.decode_device(d_data, d_offs, *oA, stream=s1)
        engB.decode_device(d_data, d_offs, *oB, stream=s1 if serial else s2)


for serial in (True, False, True, False):
    run(serial)
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e2 = torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(s1)
    s2.wait_event(e0)
    run(serial)
    e1.record(s1)
    e2.record(s2)
    torch.cuda.synchronize()
    ms = max(e0.elapsed_time(e1), e0.elapsed_time(e2)) / K
    print(f"cfg={cfg} {'serial  ' if serial else 'parallel'} ms per A+B pair {ms:.4f}  per call {ms / 2:.4f}")
ok = torch.equal(oA[0], oB[0]) and torch.equal(oA[1], oB[1])
print("outputs equal:", ok)

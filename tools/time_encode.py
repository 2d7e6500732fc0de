"""Diagnostics: time rr_encode_batch (device-resident, HIP events) on a config batch and check
the round trip.  Usage: [RR_LIB=...] python tools/time_encode.py [config] [n] [steps]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import redrock_old_amd as rr  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
data, offs = rr.gen_batch(cfg, n)
nb = int(offs[-1])
dev = torch.device("cuda:0")
eng = rr.Engine(0)
eng.reserve(n, nb)
d_data = torch.from_numpy(data).to(dev)
d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
cap = rr.elem_bound(n, nb)
d_vals = torch.empty(n * 16, dtype=torch.uint8, device=dev)
d_elems = torch.empty(cap * 16, dtype=torch.uint8, device=dev)
d_arena = torch.empty((nb + 15) & ~15, dtype=torch.uint8, device=dev)
d_tot = torch.zeros(4, dtype=torch.int64, device=dev)
d_out = torch.empty((nb + 15) & ~15, dtype=torch.uint8, device=dev)
d_ooffs = torch.empty(n + 1, dtype=torch.int64, device=dev)
s = torch.cuda.current_stream()
eng.decode_device(d_data, d_offs, d_vals, d_elems, d_arena, d_tot, stream=s)
for _ in range(3):
    eng.encode_device(d_vals, d_elems, d_arena, d_out, d_ooffs, d_tot, stream=s)
torch.cuda.synchronize()
ok = bool(torch.equal(d_out[:nb], d_data[:nb]))
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(s)
for _ in range(steps):
    eng.encode_device(d_vals, d_elems, d_arena, d_out, d_ooffs, d_tot, stream=s)
e1.record(s)
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / steps
print(f"encode cfg={cfg} n={n} bytes={nb} lib={os.environ.get('RR_LIB', 'librr_serdes.so')}"
      f" ms={ms:.4f} GiB/s={nb / ms / 1e-3 / 2**30:.1f} roundtrip={ok}")

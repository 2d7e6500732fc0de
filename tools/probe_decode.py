"""Diagnostics: run the probe build of the decode kernel on the 1M mixed batch and print the
per-phase cycle counters (s_memtime deltas summed over waves) and path counters.
Usage (GPU box): RR_LIB=librr_serdes_probe.so python tools/probe_decode.py [config] [n]"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import redrock_old_amd as rr  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
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
for _ in range(3):
    eng.decode_device(d_data, d_offs, d_vals, d_elems, d_arena, d_tot)
torch.cuda.synchronize()
L = rr.lib()
L.rr_probe_counters.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
out = np.zeros(16, np.uint64)
L.rr_probe_counters(eng._ctx, out.ctypes.data_as(C.c_void_p), 16)
names = ["windows", "staged", "chunks", "fast", "exact", "cyc_copy", "cyc_walk", "cyc_emit", "cyc_exact",
         "nrec", "fail_walk", "fail_count", "fail_ecap"]
for i, k in enumerate(names):
    print(f"{k:12s} {int(out[i]):>16d}")
w = max(int(out[0]), 1)
print("per window cycles: copy %.0f walk %.0f emit %.0f exact %.0f" % (
    out[5] / w, out[6] / w, out[7] / w, out[8] / w))

"""Diagnostics: per-window phase cycles and per-class batch cycles of the decode kernel.
Build:  make -C redrock_old_amd/csrc VARIANT=probe EXTRA=-DRR_PROBE
Run (GPU box):  RR_LIB=librr_serdes_probe.so python tools/probe_decode.py [config] [n]"""
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
# (the call's windows are sized at run time, at least 1 KiB: room for that many)
nmax = len(data) // 1024 + 2
probe = torch.zeros(nmax * 37, dtype=torch.int64, device=dev)   # (PROBE_WORDS)
L = rr.lib()
L.rr_probe_set.argtypes = [C.c_void_p]
assert L.rr_probe_set(C.c_void_p(probe.data_ptr())) == 0
for _ in range(3):
    eng.decode_device(d_data, d_offs, d_vals, d_elems, d_arena, d_tot)
torch.cuda.synchronize()
p = probe.cpu().numpy().reshape(nmax, 37).astype(np.float64)
p = p[(p[:, 0] + p[:, 1] + p[:, 2]) > 0]   # the windows the call ran
nwin = len(p)
names = ["STR", "IS", "LIST", "HTSET", "SL", "ZL", "EXACT", "HTHASH"]   # rr_decode_class.h classes
NC = len(names)
print(f"cfg {cfg}: {nwin} windows, staged {int(p[:, 29].sum())}, values/window {p[:, 28].mean():.1f}")
print("phase cycles per window (mean / p90):  copy %.0f / %.0f   sort %.0f / %.0f   batches %.0f / %.0f" % (
    p[:, 0].mean(), np.percentile(p[:, 0], 90), p[:, 1].mean(), np.percentile(p[:, 1], 90),
    p[:, 2].mean(), np.percentile(p[:, 2], 90)))
if p[:, 35].any():   # the one-launch form ([35] its look-back rounds): copy = locate, sort = stage .. first slot
    print("one-launch: locate %.0f   locate .. stage landed %.0f   stage .. first slot %.0f   (cycles, mean)" % (
        p[:, 0].mean(), p[:, 32].mean(), (p[:, 1] - p[:, 32]).mean()))
    print("  of which: classify + publish %.0f   first chunk's sort %.0f   look-back %.0f (rounds %.2f, max %d)" % (
        p[:, 33].mean(), p[:, 34].mean(), (p[:, 1] - p[:, 32] - p[:, 33] - p[:, 34]).mean(), p[:, 35].mean(), p[:, 35].max()))
nbt = p[:, 3 + NC:3 + 2 * NC].sum()
if p[:, 36].any() and nbt:
    print("batch start -> its values' offsets in registers: %.0f cycles a batch, %.0f a window (of %.0f batch cycles)" % (
        p[:, 36].sum() / nbt, p[:, 36].mean(), p[:, 2].mean()))
for c, nm in enumerate(names):
    nbat = p[:, 3 + NC + c].sum()
    if nbat:
        print(f"{nm:6s} batches {int(nbat):8d}  cycles/batch {p[:, 3 + c].sum() / nbat:9.0f}  "
              f"lanes/batch {p[:, 3 + 2 * NC + c].sum() / nbat:5.1f}")
# the raw per-window words (timeline: [27] start / [30] end on the 100 MHz clock, [31] HW_ID |
# XCC_ID << 32) for tools/timeline.py
out = os.environ.get("PROBE_OUT")
if out:
    np.save(out, probe.cpu().numpy().reshape(nmax, 37)[:nwin])

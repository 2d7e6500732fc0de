"""Diagnostics: where the snappy decompressor's time goes, per LDS-path block (s_memtime cycles
of each phase, summed over the call by the probe build's counters).
Build:  bash tools/build_variants.sh probe "-DRR_PROBE"
Run (GPU box):  RR_LIB=librr_serdes_probe.so python tools/probe_snappy.py [config] [n]"""
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
cuts = np.append(np.arange(0, nb, 16384, dtype=np.uint64), np.uint64(nb))
nblk = len(cuts) - 1
eng = rr.Engine(0)
L = rr.lib()
d_data = torch.from_numpy(data).cuda()
d_offs = torch.from_numpy(cuts.view(np.int64)).cuda()
cap = int(L.rr_snappy_compress_bound(nblk, d_data.numel()))
d_comp = torch.zeros(cap, dtype=torch.uint8, device="cuda")
d_coffs = torch.zeros(nblk + 1, dtype=torch.int64, device="cuda")
d_back = torch.zeros(d_data.numel(), dtype=torch.uint8, device="cuda")
d_boffs = torch.zeros(nblk + 1, dtype=torch.int64, device="cuda")
d_st = torch.zeros(nblk, dtype=torch.uint8, device="cuda")
s = torch.cuda.current_stream()
eng.snappy_compress_device(d_data, d_offs, d_comp, d_coffs, stream=s)
zb = int(d_coffs[-1].item())
dec = lambda: eng.snappy_decompress_device(d_comp[:((zb + 15) & ~15) or 16], d_coffs, d_back, d_boffs, d_st, stream=s)
dec()
torch.cuda.synchronize()
assert L.rr_snz_probe_reset() == 0
dec()
torch.cuda.synchronize()
v = (C.c_ulonglong * 9)()
assert L.rr_snz_probe_read(v) == 0
ok = int(d_st.max().item()) == 0 and torch.equal(d_back[:nb], d_data[:nb])
blocks, batches, tags = v[6], v[7], v[8]
print(f"cfg {cfg}: {nblk} blocks ({blocks} on the LDS path), {batches / max(blocks, 1):.1f} batches and "
      f"{tags / max(blocks, 1):.1f} tags a block, roundtrip={ok}")
names = ["stage", "A chain", "B decode", "literals", "backrefs", "output"]
tot = sum(v[:6])
for k, nm in enumerate(names):
    print(f"  {nm:9s} {v[k] / max(blocks, 1):10.0f} cycles/block  {v[k] / max(tot, 1):6.3f}")
print(f"  {'total':9s} {tot / max(blocks, 1):10.0f} cycles/block")

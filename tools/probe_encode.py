"""Diagnostics: per-window phase times of the encode emit kernel (probe build).
Build:  bash tools/build_variants.sh probe "-DRR_PROBE"
Run (GPU box):  RR_LIB=librr_serdes_probe.so python tools/probe_encode.py [config] [n]"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import redrock_old_amd as rr  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
W = int(os.environ.get("RR_ENC_W", 16384))   # must match the build (rr_kernels.hip RR_ENC_W)
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
eng.decode_device(d_data, d_offs, d_vals, d_elems, d_arena, d_tot)
torch.cuda.synchronize()
PW = 13
nwin = d_out.numel() // W + 1
# (allocated for 4 KiB windows: a build with smaller windows than W still stays inside it)
probe = torch.zeros((d_out.numel() // 4096 + 1) * PW, dtype=torch.int64, device=dev)
L = rr.lib()
L.rr_eprobe_set.argtypes = [C.c_void_p]
assert L.rr_eprobe_set(C.c_void_p(probe.data_ptr())) == 0
for _ in range(3):
    eng.encode_device(d_vals, d_elems, d_arena, d_out, d_ooffs, d_tot)
torch.cuda.synchronize()
assert torch.equal(d_out[:nb], d_data[:nb])
p = probe.cpu().numpy()[:nwin * PW].reshape(nwin, PW).astype(np.float64)
p = p[p[:, 5] > 0]
print(f"cfg {cfg}: {len(p)} windows of {W} B, values/window {p[:, 6].mean():.1f}, "
      f"tasks/window {p[:, 7].mean():.0f}, pieces/window {p[:, 8].mean():.0f} (max {p[:, 8].max():.0f})")
for i, name in [(0, "init"), (1, "headers"), (2, "tasks"), (10, " es+scan"), (11, " writes"), (9, "  field"), (12, "  decimal"),
                (3, "copy"), (4, "store"), (5, "total")]:
    print(f"  {name:8s} mean {p[:, i].mean() * 10 / 1000:8.2f} us  p90 {np.percentile(p[:, i], 90) * 10 / 1000:8.2f} us")
# E1 (enc_size_kernel): phases summed over one call's blocks (s_memtime cycles)
assert L.rr_e1probe_reset() == 0
eng.encode_device(d_vals, d_elems, d_arena, d_out, d_ooffs, d_tot)
torch.cuda.synchronize()
e1 = (C.c_ulonglong * 6)()
assert L.rr_e1probe_read(e1) == 0
blk = max(e1[3], 1)
print(f"E1: {e1[3]} blocks, {e1[4] / blk:.0f} round tasks and {e1[5] / blk:.1f} rounds a block")
tot = e1[0] + e1[1] + e1[2]
for k, name in enumerate(["head", "rounds", "tail"]):
    print(f"  {name:8s} {e1[k] / blk:10.0f} cycles/block  {e1[k] / max(tot, 1):6.3f}")

"""Diagnostics: device decode of a config batch against the CPU oracle, with a summary of the
first differing records (which window, which field).  usage: [RR_LIB=...] python tools/check_decode.py cfg n"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import redrock_old_amd as rr  # noqa: E402
from oracle import cpu  # noqa: E402

cfg, n = int(sys.argv[1]), int(sys.argv[2])
data, offs = rr.gen_batch(cfg, n)
nb = int(offs[-1])
ov, oe, _, ot = cpu.decode(data, offs, nthreads=16)
dev = torch.device("cuda:0")
eng = rr.Engine(0)
eng.set_options(rr.CTX_NO_SMALL)
d_data = torch.from_numpy(data).to(dev)
d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
cap = rr.elem_bound(n, nb)
d_vals = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
d_elems = torch.zeros(cap * 16, dtype=torch.uint8, device=dev)
d_arena = torch.zeros((nb + 15) & ~15, dtype=torch.uint8, device=dev)
d_tot = torch.zeros(4, dtype=torch.int64, device=dev)
eng.decode_device(d_data, d_offs, d_vals, d_elems, d_arena, d_tot)
torch.cuda.synchronize()
v = d_vals.cpu().numpy().view(rr.VALUE_DT)
e = d_elems.cpu().numpy().view(rr.ELEM_DT)[:len(oe)]
a = d_arena.cpu().numpy()[:nb]
bad = np.nonzero(v != ov)[0]
ebad = np.nonzero(e != oe)[0]
print(f"lib={os.environ.get('RR_LIB', 'librr_serdes.so')} cfg={cfg} n={n} bytes={nb} values_bad={len(bad)} elems_bad={len(ebad)} "
      f"arena_ok={np.array_equal(a, data[:nb])} totals={d_tot.cpu().numpy().view(np.uint64).tolist()} oracle={ot}")
for i in bad[:5]:
    print("  value", int(i), "offset", int(offs[i]), "got", v[i], "want", ov[i])

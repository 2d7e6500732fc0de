"""Diagnostics: time the GPU snappy block compression (include/rr_snappy.h) on a config batch
cut into 16 KiB RocksDB data blocks, device-resident, HIP events; and the CPU oracle on
`threads` host threads for comparison.
Usage: python tools/time_snappy.py [config] [n] [steps] [block] [threads]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import redrock_old_amd as rr  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
bs = int(sys.argv[4]) if len(sys.argv) > 4 else 16384
threads = int(sys.argv[5]) if len(sys.argv) > 5 else 0
data, offs = rr.gen_batch(cfg, n)
nb = int(offs[-1])
cuts = np.append(np.arange(0, nb, bs, dtype=np.uint64), np.uint64(nb))
nblk = len(cuts) - 1
eng = rr.Engine(0)
d_data = torch.from_numpy(data).cuda()
d_offs = torch.from_numpy(cuts.view(np.int64)).cuda()
cap = int(rr.lib().rr_snappy_compress_bound(nblk, d_data.numel()))
d_comp = torch.zeros(cap, dtype=torch.uint8, device="cuda")
d_coffs = torch.zeros(nblk + 1, dtype=torch.int64, device="cuda")
d_back = torch.zeros(d_data.numel(), dtype=torch.uint8, device="cuda")
d_boffs = torch.zeros(nblk + 1, dtype=torch.int64, device="cuda")
d_st = torch.zeros(nblk, dtype=torch.uint8, device="cuda")
s = torch.cuda.current_stream()


def timed(fn):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(steps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


tc = timed(lambda: eng.snappy_compress_device(d_data, d_offs, d_comp, d_coffs, stream=s))
zb = int(d_coffs[-1].item())
td = timed(lambda: eng.snappy_decompress_device(d_comp[:((zb + 15) & ~15) or 16], d_coffs, d_back, d_boffs, d_st, stream=s))
ok = int(d_st.max().item()) == 0 and torch.equal(d_back[:nb], d_data[:nb])
print(f"cfg={cfg} n={n} blocks={nblk}x{bs} bytes={nb} compressed={zb} ratio={zb / nb:.3f} roundtrip={ok}")
print(f"compress   {tc:.3f} ms  {nb / tc / 1e6:.1f} GB/s of input")
print(f"decompress {td:.3f} ms  {nb / td / 1e6:.1f} GB/s of output")
if threads:
    from oracle import cpu
    sub = cuts[: min(nblk, 4000) + 1]
    _, _, t1 = cpu.snappy_compress_blocks(data, sub, nthreads=threads)
    z, zo, _ = cpu.snappy_compress_blocks(data, sub, nthreads=threads)
    _, _, t2 = cpu.snappy_uncompress_blocks(z, zo, sub, nthreads=threads)
    sb = int(sub[-1])
    print(f"cpu oracle {threads} thr: compress {sb / t1 / 1e9:.2f} GB/s, decompress {sb / t2 / 1e9:.2f} GB/s (first {len(sub) - 1} blocks)")

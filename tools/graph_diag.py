import ctypes, sys, os
sys.path.insert(0, '/root/repo' if os.path.exists('/root/repo') else '.')
import numpy as np, torch
import redrock_old_amd as rr
dev = torch.device("cuda:0")
hip = ctypes.CDLL("libamdhip64.so")
eng = rr.Engine(0)
data, offs = rr.gen_batch(4, 30000, seed=4242)
n = len(offs) - 1; nb = (int(offs[-1]) + 15) & ~15; cap = rr.elem_bound(n, int(offs[-1]))
d_data = torch.zeros(nb, dtype=torch.uint8, device=dev); d_data[:data.size].copy_(torch.from_numpy(data))
d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
d_vals = torch.zeros(n * 16, dtype=torch.uint8, device=dev); d_elems = torch.zeros(cap * 16, dtype=torch.uint8, device=dev)
d_arena = torch.zeros(nb, dtype=torch.uint8, device=dev); d_tot = torch.zeros(4, dtype=torch.int64, device=dev)
eng.reserve(n, nb)
hv, he, ha, ht = eng.decode_host(data, offs)
s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    eng.decode_device(d_data, d_offs, d_vals, d_elems, d_arena, d_tot, stream=s)
torch.cuda.current_stream().wait_stream(s); torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    cs = torch.cuda.current_stream()
    st = ctypes.c_int(-1)
    rc = hip.hipStreamIsCapturing(ctypes.c_void_p(cs.cuda_stream), ctypes.byref(st))
    print("hipStreamIsCapturing rc", rc, "status", st.value, flush=True)
    eng.decode_device(d_data, d_offs, d_vals, d_elems, d_arena, d_tot, stream=cs)
for k in range(3):
    d_vals.zero_(); g.replay(); torch.cuda.synchronize()
    v = d_vals.cpu().numpy().view(rr.VALUE_DT)
    print("replay", k, "ok", bool(np.array_equal(v, hv)), "bad", int((v != hv).sum()), flush=True)

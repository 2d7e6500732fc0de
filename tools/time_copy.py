"""Diagnostics: device copy bandwidth of the copy kernel's shapes (rr_copy_shape, rr_kernels.hip)
over the bench's blob size; prints TB/s (read + write bytes) per shape."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import redrock_old_amd as rr  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 497_270_352
steps = 20
L = rr.lib()
L.rr_copy_shape.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_int, C.c_void_p]
eng = rr.Engine(0)
dev = torch.device("cuda:0")
src = torch.randint(0, 255, (nb,), dtype=torch.uint8, device=dev)
dst = torch.empty_like(src)
s = torch.cuda.current_stream()
for shape in range(9):
    def run():
        assert L.rr_copy_shape(eng._ctx, dst.data_ptr(), src.data_ptr(), nb, shape, C.c_void_p(s.cuda_stream)) == 0
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(steps):
        run()
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    assert torch.equal(dst[:4096], src[:4096]) and torch.equal(dst[-4096:], src[-4096:])
    print(f"shape={shape} ms={ms:.4f} TB/s={2 * nb / ms / 1e9:.3f}")

"""Extended structured fuzz of the host codec (rr_host.c, the compat shim's CPU route) against the
oracle, beyond the CPU suite's seven seeds (diagnostics, CPU only): for every seed and config,
the GPU suite's mutation corpus (tests/helpers.py structured_mutations) decoded by
rr_host_decode_batch and by the oracle (records, descriptors, statuses, totals, arena equal),
the verdict-only walk rr_host_check_value on the same blobs, and the decoded values re-encoded by
rr_host_encode_batch against the oracle's encoder.
usage: python tools/fuzz_host_codec.py [seeds] [first_seed]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import redrock_old_amd as rr  # noqa: E402
from helpers import assert_flat_equal, batch_from_blobs, structured_mutations  # noqa: E402
from oracle import cpu  # noqa: E402

SEEDS = int(sys.argv[1]) if len(sys.argv) > 1 else 200
S0 = int(sys.argv[2]) if len(sys.argv) > 2 else 100
CFGS = [(4, 1500), (3, 600), (10, 500), (11, 20), (1, 800), (2, 400)]

t0 = time.time()
blobs = bad = checked = 0
for seed in range(S0, S0 + SEEDS):
    for cfg, n in CFGS:
        data, offs = rr.gen_batch(cfg, n, seed=seed)
        fdata, foffs = batch_from_blobs(structured_mutations(data, offs, 1000 + cfg + 7919 * seed))
        cap = rr.elem_bound(len(foffs) - 1, int(foffs[-1]))
        v, e, a, t = rr.host_decode(fdata, foffs, cap)
        ov, oe, oa, ot = cpu.decode(fdata, foffs, cap)
        what = f"seed {seed} cfg {cfg}"
        assert_flat_equal((v, e), (ov, oe), what)
        assert t == ot and np.array_equal(a, oa), what
        c = rr.host_check(fdata, foffs)
        want = ov.copy()
        want["elem_base"] = 0
        keep = want["status"] != 11
        assert np.array_equal(c[keep], want[keep]), what
        d, o, t2 = rr.host_encode(v, e, a)
        od, oo, ot2 = cpu.encode(v, e, a)
        assert np.array_equal(o, oo) and np.array_equal(d, od[:int(oo[-1])][:len(d)]) and t2 == ot2, what + " encode"
        blobs += len(foffs) - 1
        bad += int((v["status"] != 0).sum())
        checked += 1
    if (seed - S0) % 20 == 19:
        print(f"  seeds {S0}..{seed}: {checked} batches, {blobs} blobs, {bad} rejected, {time.time() - t0:.0f} s", flush=True)
print(f"host codec fuzz: seeds {S0}..{S0 + SEEDS - 1}, configs {[c for c, _ in CFGS]}: {checked} batches, {blobs} blobs "
      f"({bad} rejected by both), every record, descriptor, status, total, arena byte and re-encoded byte equal to the "
      f"oracle; {time.time() - t0:.0f} s")

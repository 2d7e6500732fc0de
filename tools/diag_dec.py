"""Decode diagnostics (GPU box): decode_host against the oracle on generated batches; prints the
first differing value record / descriptor with its neighbourhood, per configuration."""
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import redrock_old_amd as rr  # noqa: E402
from oracle import cpu  # noqa: E402

eng = rr.Engine()
eng.set_options(rr.CTX_NO_SMALL)
cases = [(4, 60000, 61), (1, 100000, None), (2, 100000, None), (3, 50000, None), (4, 100000, None), (4, 4097, 5097)]
for cfg, n, seed in cases:
    data, offs = rr.gen_batch(cfg, n, seed=seed) if seed is not None else rr.gen_batch(cfg, n)
    v, e, a, t = eng.decode_host(data, offs)
    ov, oe, oa, ot = cpu.decode(data, offs, nthreads=8)
    line = f"cfg{cfg} n={n}: totals {'ok' if t == ot else (t, ot)}"
    if not np.array_equal(v, ov):
        bad = np.nonzero(v != ov)[0]
        i = int(bad[0])
        line += f"; {len(bad)} values differ, first #{i}: {v[i]} vs {ov[i]}; bad idx sample {bad[:20].tolist()}"
        cls = {}
        for j in bad:
            k = (int(ov[j]["type"]), int(ov[j]["enc"]))
            cls[k] = cls.get(k, 0) + 1
        line += f"; by (type,enc) {cls}"
    elif len(e) != len(oe) or not np.array_equal(e, oe):
        m = min(len(e), len(oe))
        bad = np.nonzero(e[:m] != oe[:m])[0]
        j = int(bad[0]) if len(bad) else m
        vi = int(np.searchsorted(ov["elem_base"], j, side="right") - 1)
        line += (f"; {len(bad)} descs differ, first #{j} (value {vi} {ov[vi]}): "
                 f"{e[j] if j < len(e) else None} vs {oe[j] if j < len(oe) else None}")
        vals = np.unique(np.searchsorted(ov["elem_base"], bad, side="right") - 1)
        line += f"; values {vals[:20].tolist()} ({len(vals)})"
    elif not np.array_equal(a, oa):
        line += "; arena differs"
    else:
        line += "; OK"
    print(line, flush=True)

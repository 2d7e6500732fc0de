"""Per-CU timeline of decode_kernel windows from a probe dump (tools/probe_decode.py with
PROBE_OUT=file.npy, probe build): how long windows live, how many run per CU at once, the idle
gaps between a slot's windows, and the phase split.  usage: python tools/timeline.py file.npy"""
import sys

import numpy as np

p = np.load(sys.argv[1]).astype(np.int64)
t0, t1, hw = p[:, 27], p[:, 30], p[:, 31]
ok = (t0 > 0) & (t1 > 0)
p, t0, t1, hw = p[ok], t0[ok], t1[ok], hw[ok]
base = t0.min()
s, e = (t0 - base) * 10, (t1 - base) * 10   # ns (100 MHz)
xcc = (hw >> 32) & 0xF
cu = (hw >> 8) & 0xF
sh = (hw >> 12) & 0x1
se = (hw >> 13) & 0x7
cuid = ((xcc * 8 + se) * 2 + sh) * 16 + cu
print(f"windows {len(p)}, span {e.max() / 1e3:.1f} us, CUs seen {len(np.unique(cuid))}, XCCs {sorted(set(xcc.tolist()))}")
life = (e - s)
print(f"window lifetime us: mean {life.mean() / 1e3:.2f} p10 {np.percentile(life, 10) / 1e3:.2f} "
      f"p90 {np.percentile(life, 90) / 1e3:.2f}")
cyc = p[:, 0] + p[:, 1] + p[:, 2]
print(f"memtime cycles per window {cyc.mean():.0f} -> clock {cyc.sum() / life.sum() * 1e3 / 1e3:.2f} GHz")
# per CU: concurrency over time and gaps
conc, gaps, firsts, lasts = [], [], [], []
for c in np.unique(cuid):
    m = cuid == c
    ss, ee = np.sort(s[m]), np.sort(e[m])
    firsts.append(ss.min())
    lasts.append(ee.max())
    ev = sorted([(x, 1) for x in s[m]] + [(x, -1) for x in e[m]])
    cur, last, acc = 0, ev[0][0], np.zeros(4)
    for t, d in ev:
        acc[min(cur, 3)] += t - last
        cur += d
        last = t
    conc.append(acc / max(acc.sum(), 1))
conc = np.array(conc).mean(0)
print("share of each CU's busy span with 0/1/2/3+ windows resident: " + " ".join(f"{x:.3f}" for x in conc))
firsts, lasts = np.array(firsts), np.array(lasts)
print(f"CU first start us: max {firsts.max() / 1e3:.2f}; CU last end us: min {lasts.min() / 1e3:.2f} "
      f"median {np.median(lasts) / 1e3:.2f} max {lasts.max() / 1e3:.2f}")
# phase split in time (memtime fractions applied to each lifetime)
fr = p[:, :3] / np.maximum(cyc, 1)[:, None]
print("phase share of lifetime: copy %.3f sort %.3f batches %.3f" % tuple(fr.mean(0)))
# generations: windows starting per us
h, _ = np.histogram(s / 1e3, bins=np.arange(0, e.max() / 1e3 + 1, 1.0))
print("window starts per us (first 40 us):", h[:40].tolist())

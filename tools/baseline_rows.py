"""BASELINE.md's single-GPU table rows, generated from committed bench lines (one bench.py JSON
line per configuration, tools/baseline_table.sh), so the table cannot drift from the lines.
usage: python tools/baseline_rows.py ROUNDTAG   (reads profiles/<ROUNDTAG>_bench_<name>.json)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
R = sys.argv[1] if len(sys.argv) > 1 else "r4"
ROWS = [("cfg1", "1 (100K × 64 B String, {mb} MB)"), ("cfg2", "2 (1M Zipf String, {mb} MB)"),
        ("cfg3", "3 (1M Hash ziplist ×16, {mb} MB)"), ("cfg4_10m", "4 (10M mixed, {gb} GB)"),
        ("", "1M mixed (headline, {mb} MB)"),
        ("cfg5_shard7", "5 (100M mixed, 49.6 GB; one GPU's shard: the last of the 8-way plan, {gb} GB)")]


def row(name, label):
    p = os.path.join(ROOT, "profiles", f"{R}_bench{'_' + name if name else ''}.json")
    if not os.path.exists(p) and name == "cfg4_10m":   # the evidence call's 10M line
        p = os.path.join(ROOT, "profiles", f"{R}_bench_10m.json")
    if not os.path.exists(p):
        return None
    d = json.load(open(p))
    c, cpu, dec, enc, rf = d["config"], d.get("cpu_baseline") or {}, d["decode"], d["encode"], d["roofline"]
    nb = c["blob_bytes_per_gpu"]
    lab = label.format(mb=round(nb / 1e6, 1), gb=round(nb / 1e9, 2))
    us = lambda ms: f"{ms * 1e3:.1f} µs" if ms < 0.1 else f"{ms:.3f} ms"
    cpu_f = f"{cpu.get('value', float('nan')):.2f} / {cpu.get('encode_gib_s', float('nan')):.2f} GiB/s"
    return (f"| {lab} | dec / enc | {cpu_f} | {cpu.get('flat_1t_gib_s', float('nan')):.2f} GiB/s | "
            f"{cpu.get('flat_16t_gib_s', float('nan')):.2f} GiB/s | **{dec['gib_s']:,.0f}** / {enc['gib_s']:,.0f} GiB/s "
            f"({us(dec['event_ms_per_launch'])} / {us(enc['event_ms_per_launch'])}) | driver | driver | driver | "
            f"{rf['frac']:.3f} ({rf['frac_of_copy']:.2f}) |")


print("| Config | Direction | CPU faithful 1T | CPU flat 1T | CPU flat 16T | GPU×1 | GPU×2 | GPU×4 | GPU×8 | "
      "HBM fraction (of copy) |")
print("|---|---|---|---|---|---|---|---|---|---|")
for name, label in ROWS:
    r = row(name, label)
    if r:
        print(r)

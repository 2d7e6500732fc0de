"""Summarise a tools/pmc_decode.sh output directory: per-kernel counters (mean per dispatch)
and kernel-trace durations.  Usage: python tools/pmc_summary.py gpurun_out/pmcN"""
import collections
import csv
import glob
import os
import re
import sys


def short(name):
    m = re.search(r"(\w+_kernel)\b", name)
    return m.group(1) if m else name.split("(")[0].split("::")[-1][:24]


d = sys.argv[1]
for f in sorted(os.listdir(d)):
    p = glob.glob(os.path.join(d, f, "*counter_collection.csv"))
    if not p:
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(p[0])):
        k = short(r["Kernel_Name"])
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    for k in agg:
        if k.startswith(("vectorized", "__amd")):
            continue
        print(f"{f:6s} {k:24s}", " ".join(f"{c}={v / len(disp[k]):.4g}" for c, v in sorted(agg[k].items())))
for p in glob.glob(os.path.join(d, "trace", "*kernel_stats.csv")):
    for r in csv.DictReader(open(p)):
        print(f"trace  {short(r['Name']):24s} calls={r['Calls']} avg_us={float(r['AverageNs']) / 1e3:.1f}")

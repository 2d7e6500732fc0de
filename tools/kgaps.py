"""Print the last kernels of a rocprofv3 kernel_trace.csv with their durations and the idle gap
before each (diagnostics: is a small call bound by the GPU or by the host's submissions?).
usage: python tools/kgaps.py run_kernel_trace.csv [last]"""
import csv
import re
import sys

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).replace("void ", "")
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name.split("<")[0]))
rows.sort()
last = int(sys.argv[2]) if len(sys.argv) > 2 else 12
prev = None
for s, e, name in rows[-last:]:
    gap = (s - prev) / 1000 if prev is not None else 0.0
    print(f"  {name[:28]:28s} dur {(e - s) / 1000:6.1f} us  gap before {gap:5.1f} us")
    prev = e

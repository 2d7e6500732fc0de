"""Sum rocprofv3 PMC counter_collection.csv values per kernel (diagnostics).
usage: python3 tools/pmc_by_kernel.py [-a] DIR [DIR ...]   (-a: every counter, per call)"""
import collections
import csv
import glob
import re
import sys

allc = "-a" in sys.argv
for d in [a for a in sys.argv[1:] if a != "-a"]:
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    calls = collections.defaultdict(set)
    for p in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
            name = re.sub(r"[<(].*", "", name)
            tot[name][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[(name, r["Counter_Name"])].add(r.get("Dispatch_Id", ""))
    for k, c in tot.items():
        if not any(x in k for x in ("decode", "count", "scan", "enc_", "post", "snz")):
            continue
        bc, ia = c.get("SQ_LDS_BANK_CONFLICT", 0), c.get("SQ_LDS_IDX_ACTIVE", 0)
        line = f"{d.rstrip('/').split('/')[-1]:26s} {k:20s}"
        if ia:
            line += f" conflict/active {bc / ia:.3f} (conflict {bc:.3e}, active {ia:.3e})"
        if "SQ_INSTS_LDS" in c:
            line += f"  LDS insts {c['SQ_INSTS_LDS']:.3e}"
        if "SQ_WAIT_INST_LDS" in c and c.get("SQ_WAVE_CYCLES"):
            line += f"  wait_inst_lds/wave_cycles {c['SQ_WAIT_INST_LDS'] / c['SQ_WAVE_CYCLES']:.3f}"
        print(line)
        if allc:
            for cn in sorted(c):
                ncall = max(1, len(calls[(k, cn)]))
                print(f"    {cn:24s} {c[cn] / ncall:.4e} per call ({ncall} calls)")

"""Turn a tools/profile_bench.sh directory into the committed profile summary:
per-kernel average durations (kernel trace) and per-launch HBM traffic of one
rr_decode_batch call (FETCH_SIZE x2, the MI355X_MICROARCH.md gfx950 correction for 16 B/lane
streaming reads, + WRITE_SIZE; both in KB per dispatch), summed over the pipeline's kernels.
Usage: python tools/traffic_summary.py PROFDIR OUT.json"""
import collections
import csv
import glob
import json
import os
import re
import sys

d, out = sys.argv[1], sys.argv[2]


def short(name):
    m = re.search(r"(\w+_kernel)\b", name)
    return m.group(1) if m else name.split("(")[0].strip()


res = {"kernels": {}, "traffic_bytes_per_call": None}
for p in glob.glob(os.path.join(d, "trace", "*kernel_stats.csv")):
    for r in csv.DictReader(open(p)):
        res["kernels"][short(r["Name"])] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3}
per = collections.defaultdict(dict)
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for p in glob.glob(os.path.join(d, c, "*counter_collection.csv")):
        acc = collections.defaultdict(float)
        disp = collections.defaultdict(set)
        for r in csv.DictReader(open(p)):
            k = short(r["Kernel_Name"])
            acc[k] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
        for k in acc:
            per[k][c] = acc[k] / len(disp[k]) * 1024   # KB -> bytes, per dispatch
# (no zeroing launch: the sums are zero between calls, restored by the pipelines themselves)
if "enc_emit_kernel" in per:   # RR_PROFILE=encode run (one decode call precedes the encode steps)
    pipeline = ("enc_size_kernel", "enc_index_kernel", "enc_emit_kernel")
else:
    pipeline = ("count_kernel", "decode_kernel")
res["pipeline"] = list(pipeline)
tot = 0.0
for k in pipeline:
    if k in per:
        f, w = per[k].get("FETCH_SIZE", 0.0), per[k].get("WRITE_SIZE", 0.0)
        res["kernels"].setdefault(k, {}).update({"fetch_bytes": f, "write_bytes": w, "hbm_bytes": 2 * f + w})
        tot += 2 * f + w
res["traffic_bytes_per_call"] = tot if per else None
# the workload tag bench.py matches the summary by (profile_bench.sh's default workload: the
# bench line's 1M-value config-4 batch); an existing tag in OUT is kept
wl = {"config": 4, "n": 1000000, "blob_bytes": 497270349,
      "command": ("bench.py --profile-encode" if "enc_emit_kernel" in per else "bench.py --profile-only") +
                 " (rocprofv3 --kernel-trace --stats; --pmc FETCH_SIZE; --pmc WRITE_SIZE)"}
if os.path.exists(out):
    try:
        wl = json.load(open(out)).get("workload") or wl
    except ValueError:
        pass
res["workload"] = wl
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))

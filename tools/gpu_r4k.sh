#!/bin/bash
# Round-4 GPU step: per-kernel durations of the 100K-value config-1 decode call and its timeline.
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ks1s -o run -- python3 $R/tools/time_decode.py 1 100000 50 > $R/gpurun_out/ks1s.log 2>&1
cd $R
python3 tools/kstats.py $(find gpurun_out/ks1s -name "*kernel_stats.csv")
python3 - <<'PY'
import csv, glob
rows = []
for p in glob.glob("gpurun_out/ks1s/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(p)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
tail = rows[-12:]
t0 = int(tail[0]["Start_Timestamp"])
for r in tail:
    print(f'{(int(r["Start_Timestamp"]) - t0) / 1e3:9.2f} {(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3:8.2f}  {r["Kernel_Name"][:60]}')
PY

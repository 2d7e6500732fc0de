#!/bin/bash
# per-kernel durations of the encode call (rocprofv3 kernel trace + stats) for a library build
# usage (GPU box, repo root): tools/kstats_encode.sh OUTDIR [lib] [config]
OUT=$(realpath -m "$1"); LIB=${2:-librr_serdes.so}; CFG=${3:-4}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
RR_LIB=$LIB timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
    python3 "$ROOT/tools/time_encode.py" "$CFG" ${RR_N:-1000000} 20 > "$OUT/run.log" 2>&1
rc=$?
python3 "$ROOT/tools/kstats.py" $(find "$OUT" -name "*kernel_stats.csv")
exit $rc

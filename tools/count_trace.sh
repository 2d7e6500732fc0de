#!/bin/bash
# Kernel-trace stats of the decode pipeline for every in-tree variant library (diagnostics).
# Usage (GPU box, repo root): bash tools/count_trace.sh OUTDIR [config]
set -e
OUT=$(realpath -m "$1"); CFG=${2:-4}; ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for lib in $(cd "$ROOT/redrock_old_amd" && ls librr_serdes*.so | grep -v probe); do
  RR_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$lib" -o run -- \
      python3 "$ROOT/tools/time_decode.py" "$CFG" 1000000 10 > "$OUT/$lib.log" 2>&1
done

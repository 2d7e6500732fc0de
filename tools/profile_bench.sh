#!/bin/bash
# rocprofv3 evidence for bench.py's decode (device-resident 1M mixed batch):
#   trace/   kernel-trace + stats (per-kernel average durations)
#   fetch/   FETCH_SIZE pass, write/ WRITE_SIZE pass (HBM traffic, separate passes)
# Usage (GPU box, repo root): [RR_PROFILE=encode] bash tools/profile_bench.sh OUTDIR [extra bench args]
set -e
OUT=$(realpath -m "$1"); shift
ROOT=$(pwd)
MODE=--profile-only
[ "${RR_PROFILE:-decode}" = encode ] && MODE=--profile-encode
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$ROOT/bench.py" $MODE --steps 20 --warmup 3 "$@" > "$OUT/trace.log" 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/$c" -o run -- \
      python3 "$ROOT/bench.py" $MODE --steps 5 --warmup 1 "$@" > "$OUT/$c.log" 2>&1
done

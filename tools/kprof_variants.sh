#!/bin/bash
# Per-kernel rocprofv3 stats of tools/time_decode.py for several in-tree builds (diagnostics).
# usage (GPU box, repo root): tools/kprof_variants.sh "default var1 var2" [cfg] [n]
set -e
ROOT=$(pwd)
mkdir -p gpurun_out/kprof
cfg=${2:-4}; n=${3:-1000000}
cd /tmp && export TMPDIR=/tmp
for v in $1; do
  lib=librr_serdes_$v.so; [ "$v" = default ] && lib=librr_serdes.so
  RR_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/kprof/$v" -o run -- \
      python3 "$ROOT/tools/time_decode.py" $cfg $n 20 > "$ROOT/gpurun_out/kprof/$v.log" 2>&1
  echo "== $v: $(grep cfg "$ROOT/gpurun_out/kprof/$v.log")"
  python3 "$ROOT/tools/kstats.py" $(find "$ROOT/gpurun_out/kprof/$v" -name '*kernel_stats.csv')
done

#!/bin/bash
# per-kernel times of tools/time_snappy.py for two libraries (diagnostics; GPU box, repo root)
OUT=$(realpath -m gpurun_out/kss); ROOT=$(pwd); mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for L in librr_serdes.so librr_serdes_head.so; do
  RR_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$L -o run -- python3 $ROOT/tools/time_snappy.py 2 1000000 5 > $OUT/$L.log 2>&1 || exit 1
  echo "== $L"; python3 $ROOT/tools/kstats.py $(find $OUT/$L -name "*kernel_stats.csv")
done

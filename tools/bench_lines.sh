#!/bin/bash
# The round's bench lines on the GPU box (repo root): the default bench.py line (1M config 4,
# CPU baseline, split/gather, snappy legs) and the 10M config-4 line -> gpurun_out/ev/
# usage: tools/bench_lines.sh ROUNDTAG
set -e
R=${1:-r3}
E=gpurun_out/ev
mkdir -p $E
timeout -k 10 600 python3 -u bench.py > $E/bench.log 2>&1 && echo "bench done"
grep '^{' $E/bench.log | tail -1 > $E/${R}_bench.json
timeout -k 10 600 python3 -u bench.py --n 10000000 --steps 10 --warmup 2 --no-cpu --no-split --no-snappy > $E/bench10m.log 2>&1 && echo "bench 10m done"
grep '^{' $E/bench10m.log | tail -1 > $E/${R}_bench_10m.json
cat $E/${R}_bench.json

#!/bin/bash
# BASELINE.md's single-GPU rows (GPU box, repo root): one bench.py line per BASELINE config,
# each with its CPU baseline legs, into gpurun_out/bl/.  usage: tools/baseline_table.sh
mkdir -p gpurun_out/bl
run() {   # name args...
    local name=$1; shift
    timeout -k 10 400 python3 -u bench.py --no-split --no-snappy "$@" > gpurun_out/bl/$name.log 2>&1
    local rc=$?
    grep '^{' gpurun_out/bl/$name.log | tail -1 > gpurun_out/bl/$name.json
    echo "$name rc=$rc"
    return $rc
}
run cfg1 --config 1 --n 100000 --no-host && \
run cfg2 --config 2 --no-host && \
run cfg3 --config 3 --no-host && \
run cfg4_10m --config 4 --n 10000000 --steps 10 --warmup 2 --no-host && \
run cfg5_shard7 --config 5 --steps 10 --warmup 2 --no-host

#!/bin/bash
# Round-4 GPU step: no zeroing launch (sums zero between calls) — the GPU suite, then decode and
# encode timing against the pre-round build.
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/q_tests.log 2>&1; tail -3 gpurun_out/q_tests.log
bash tools/ab_decode.sh "head prev" "4 3 1"
: > gpurun_out/ab100k.log
for rep in 1 2; do for v in librr_serdes.so librr_serdes_head.so librr_serdes_prev.so; do
  RR_LIB=$v timeout -k 10 120 python tools/time_decode.py 1 100000 50 | grep cfg >> gpurun_out/ab100k.log
done; done
cat gpurun_out/ab100k.log
bash tools/ab_encode.sh "head" "4"

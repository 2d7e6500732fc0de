#!/bin/bash
# Round-4 GPU step: stage / arena writes predicated per lane instead of a shared dummy LDS slot —
# parity, then decode timing against the committed build (head).
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/aa_tests.log 2>&1; tail -2 gpurun_out/aa_tests.log
: > gpurun_out/ab100k.log
for rep in 1 2 3; do for v in librr_serdes.so librr_serdes_head.so; do
  RR_LIB=$v timeout -k 10 120 python tools/time_decode.py 1 100000 50 | grep cfg >> gpurun_out/ab100k.log
done; done
cat gpurun_out/ab100k.log
bash tools/ab_decode.sh "head" "4 3 2 1"

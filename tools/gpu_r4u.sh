#!/bin/bash
# Round-4 GPU step: staggered windows (half windows on the first generation's first slot of
# every CU) — parity, then decode timing against the same build without the stagger.
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_small.py > gpurun_out/u_tests.log 2>&1; tail -3 gpurun_out/u_tests.log
bash tools/ab_decode.sh "nostag" "4 3 2 1"
: > gpurun_out/ab10m.log
for rep in 1 2; do for v in librr_serdes.so librr_serdes_nostag.so; do
  RR_LIB=$v timeout -k 10 200 python tools/time_decode.py 4 10000000 5 | grep cfg >> gpurun_out/ab10m.log
done; done
cat gpurun_out/ab10m.log

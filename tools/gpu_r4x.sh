#!/bin/bash
# Round-4 GPU step: kernel-argument preload (kp build) against the current build — decode at
# 100K config 1 and 1M configs 1-4, encode config 4, parity on the kp build.
set -e
mkdir -p gpurun_out
RR_LIB=librr_serdes_kp.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_small.py > gpurun_out/x_tests.log 2>&1; tail -2 gpurun_out/x_tests.log
: > gpurun_out/ab100k.log
for rep in 1 2 3; do for v in librr_serdes.so librr_serdes_kp.so; do
  RR_LIB=$v timeout -k 10 120 python tools/time_decode.py 1 100000 50 | grep cfg >> gpurun_out/ab100k.log
done; done
cat gpurun_out/ab100k.log
bash tools/ab_decode.sh "kp" "4 3 2 1"
bash tools/ab_encode.sh "kp" "4"

#!/bin/bash
# Round-4 GPU step: count kernel with Lists walked from an LDS stage (32-bit walk) — parity, then
# the count kernel's duration at three stage sizes.
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/s_tests.log 2>&1; tail -3 gpurun_out/s_tests.log
for v in librr_serdes.so librr_serdes_lb8k.so librr_serdes_lb2k.so; do
  echo $v; bash tools/kstats_decode.sh gpurun_out/ks_$v $v 4 | grep count_kernel
done

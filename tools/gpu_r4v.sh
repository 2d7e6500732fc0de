#!/bin/bash
# Round-4 GPU step: snappy decompress with a register window for the tag chain (snzW) — the
# snappy GPU tests on it, then timing against the current build.
set -e
mkdir -p gpurun_out
RR_LIB=librr_serdes_snzW.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_snappy.py > gpurun_out/v_tests.log 2>&1; tail -3 gpurun_out/v_tests.log
: > gpurun_out/absnz.log
for rep in 1 2; do for c in 4 3; do for v in librr_serdes.so librr_serdes_snzW.so; do
  echo "$v" >> gpurun_out/absnz.log
  RR_LIB=$v timeout -k 10 200 python tools/time_snappy.py $c 1000000 5 2>&1 | grep -v amdgpu.ids | grep decompress >> gpurun_out/absnz.log
done; done; done
cat gpurun_out/absnz.log

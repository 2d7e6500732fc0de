#!/bin/bash
# Round-4 GPU step: parity + timing of two candidate builds — count kernel with a last-wave
# table flush (cntL), snappy with long-literal head bytes in the first chunk round trip (snzH).
set -e
mkdir -p gpurun_out
RR_LIB=librr_serdes_cntL.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_small.py > gpurun_out/cntL_tests.log 2>&1; tail -3 gpurun_out/cntL_tests.log
RR_LIB=librr_serdes_snzH.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_snappy.py > gpurun_out/snzH_tests.log 2>&1; tail -3 gpurun_out/snzH_tests.log
bash tools/ab_decode.sh "cntL prev" "4 3 1"
: > gpurun_out/ab10m.log
for v in librr_serdes.so librr_serdes_cntL.so; do
  RR_LIB=$v timeout -k 10 200 python tools/time_decode.py 4 10000000 5 | grep cfg >> gpurun_out/ab10m.log
done
cat gpurun_out/ab10m.log
: > gpurun_out/absnz.log
for rep in 1 2; do for c in 4 3; do for v in librr_serdes.so librr_serdes_snzH.so; do
  echo "$v" >> gpurun_out/absnz.log
  RR_LIB=$v timeout -k 10 200 python tools/time_snappy.py $c 1000000 5 2>&1 | grep -v amdgpu.ids >> gpurun_out/absnz.log
done; done; done
cat gpurun_out/absnz.log

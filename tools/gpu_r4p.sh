#!/bin/bash
# Round-4 GPU step: decode with one-load first slots and 16-byte window heads — parity, then
# timing against the pre-round build and a kernarg-preload build (kp).
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_small.py tests/test_gpu_snappy.py > gpurun_out/p_tests.log 2>&1; tail -3 gpurun_out/p_tests.log
RR_LIB=librr_serdes_kp.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/kp_tests.log 2>&1; tail -3 gpurun_out/kp_tests.log
bash tools/ab_decode.sh "prev kp" "3 4 1"
: > gpurun_out/ab10m.log
for v in librr_serdes.so librr_serdes_prev.so librr_serdes_kp.so; do
  RR_LIB=$v timeout -k 10 200 python tools/time_decode.py 4 10000000 5 | grep cfg >> gpurun_out/ab10m.log
done
cat gpurun_out/ab10m.log
bash tools/kstats_decode.sh gpurun_out/ks_cur3 librr_serdes.so 3

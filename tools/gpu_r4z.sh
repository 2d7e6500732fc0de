#!/bin/bash
# Round-4 GPU step: E1 tasks per thread per round (U4, U8 builds) against the current build —
# encode kernel durations and the call's time.
set -e
mkdir -p gpurun_out
for v in librr_serdes.so librr_serdes_U4.so librr_serdes_U8.so; do
  echo $v
  RR_LIB=$v timeout -k 10 120 python tools/time_encode.py 4 1000000 20 | grep -v amdgpu
done
bash tools/ab_encode.sh "U4 U8" "4"

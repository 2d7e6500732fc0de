#!/bin/bash
# Round-4 GPU step: where config 1's 100K-value decode spends its time — decode_kernel alone,
# copy + stage only (ablation 1), + the class sort (ablation 2); timing-only builds.
set -e
mkdir -p gpurun_out
for v in librr_serdes.so librr_serdes_abl1.so librr_serdes_abl2.so; do
  echo $v; RR_N=100000 bash tools/kstats_decode.sh gpurun_out/kt_$v $v 1 | grep "_kernel"
done

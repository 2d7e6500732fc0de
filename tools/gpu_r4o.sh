#!/bin/bash
# Round-4 GPU step: decode timing across the round's commits (bisect of a config-3 slowdown) and
# per-kernel durations of the current and the pre-round build on config 3.
set -e
mkdir -p gpurun_out
bash tools/ab_decode.sh "prev bca7c8e1 b26c0f82 bc836fe1" "3 4"
bash tools/kstats_decode.sh gpurun_out/ks_cur3 librr_serdes.so 3
bash tools/kstats_decode.sh gpurun_out/ks_prev3 librr_serdes_prev.so 3

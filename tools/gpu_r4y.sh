#!/bin/bash
# Round-4 GPU step: values per batch of the List and HT-set classes (L32: 32 Lists per batch,
# T8: 8 HT sets per batch) against the current build.
set -e
mkdir -p gpurun_out
bash tools/ab_decode.sh "L32 T8" "4"
bash tools/ab_decode.sh "L32 T8" "4"

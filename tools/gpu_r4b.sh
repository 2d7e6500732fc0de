#!/bin/bash
# Round-4 GPU step: the parity subset (decode paths), decode A/B against librr_serdes_prev.so,
# then per-kernel times of the new decode on configs 4 and 1.
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
bash tools/ab_decode.sh "prev" "4 3 2 1" > /dev/null && cat gpurun_out/ab.log
bash tools/kstats_decode.sh gpurun_out/ks4 librr_serdes.so 4
bash tools/kstats_decode.sh gpurun_out/ks1 librr_serdes.so 1

#!/bin/bash
# GPU build-loop step: parity tests, decode kernel stats, decode A/B vs $1, encode A/B vs $2
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_encode.py -m gpu -x -q --timeout 240 \
    --timeout-method thread -k "not config5 and not 10m" > gpurun_out/t.log 2>&1 && echo "tests ok" || { tail -30 gpurun_out/t.log; exit 1; }
bash tools/kstats_decode.sh gpurun_out/ks_new librr_serdes.so 4
bash tools/ab_decode.sh "$1" "4 2" > /dev/null && cat gpurun_out/ab.log
bash tools/ab_encode.sh "$2" "4 3" > /dev/null && cat gpurun_out/ab_enc.log

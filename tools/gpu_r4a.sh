#!/bin/bash
# Round-4 GPU step: the whole GPU suite, then decode / encode A/B against librr_serdes_prev.so.
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
bash tools/ab_decode.sh "prev" "4 3 2 1" > /dev/null && cat gpurun_out/ab.log
bash tools/ab_encode.sh "prev" "4 3" > /dev/null && cat gpurun_out/ab_enc.log

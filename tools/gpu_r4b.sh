#!/bin/bash
# Round-4 GPU step: the GPU suite, decode A/B (round-3 build, stage 1, working tree), per-kernel
# times of the new decode on configs 4 and 1, the per-value latency bench.
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -60 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 300 python tests/test_compat.py latency 4 2000 > gpurun_out/latency.log 2>&1; cat gpurun_out/latency.log
bash tools/ab_decode.sh "prev s1" "4 3 2 1" > /dev/null && cat gpurun_out/ab.log
bash tools/kstats_decode.sh gpurun_out/ks4 librr_serdes.so 4
bash tools/kstats_decode.sh gpurun_out/ks1 librr_serdes.so 1
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1; tail -c 3000 gpurun_out/bench.log

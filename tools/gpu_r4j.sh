#!/bin/bash
# Round-4 GPU step: the GPU suite, the latency probe and bench (wave-per-value small encode).
set -e
mkdir -p gpurun_out
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/t.log 2>&1 || rc=$?
grep -E "^FAILED|passed|failed" gpurun_out/t.log | tail -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tests/test_compat.py latency 4 2000 > gpurun_out/latency.log 2>&1; cat gpurun_out/latency.log
timeout -k 10 300 python tests/test_compat.py latency 1 2000 > gpurun_out/latency1.log 2>&1; cat gpurun_out/latency1.log
timeout -k 10 120 python tools/time_decode.py 1 100000 50 > gpurun_out/t1.log 2>&1; grep cfg gpurun_out/t1.log
RR_N=100000 bash tools/kstats_decode.sh gpurun_out/ks1s librr_serdes.so 1

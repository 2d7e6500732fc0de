#!/bin/bash
# Round-4 GPU step: the GPU suite, decode A/B, the latency probe and the per-value latency bench.
set -e
mkdir -p gpurun_out
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/t.log 2>&1 || rc=$?
grep -E "^FAILED|passed|failed" gpurun_out/t.log | tail -30
[ $rc -le 1 ] || exit $rc
bash tools/ab_decode.sh "prev" "4 1" > /dev/null && cat gpurun_out/ab.log
timeout -k 10 120 tools/micro/lat_probe > gpurun_out/lat_probe.log 2>&1; cat gpurun_out/lat_probe.log
timeout -k 10 300 python tests/test_compat.py latency 4 2000 > gpurun_out/latency.log 2>&1; cat gpurun_out/latency.log
timeout -k 10 300 python tests/test_compat.py latency 1 2000 > gpurun_out/latency1.log 2>&1; cat gpurun_out/latency1.log

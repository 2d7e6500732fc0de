#!/bin/bash
# Round-4 GPU step: the GPU suite, snappy A/B (paired copies vs the committed two-phase build),
# decode A/B with nontemporal window loads, the latency probe and bench.
set -e
mkdir -p gpurun_out
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/t.log 2>&1 || rc=$?
grep -E "^FAILED|passed|failed" gpurun_out/t.log | tail -30
[ $rc -le 1 ] || exit $rc
for c in 4 3; do
  timeout -k 10 200 python tools/time_snappy.py $c 1000000 5 >> gpurun_out/snz.log 2>&1
  RR_LIB=librr_serdes_snzB.so timeout -k 10 200 python tools/time_snappy.py $c 1000000 5 >> gpurun_out/snz.log 2>&1
done; grep -v amdgpu.ids gpurun_out/snz.log
bash tools/ab_decode.sh "ntl" "4 2" > /dev/null && cat gpurun_out/ab.log
timeout -k 10 120 tools/micro/lat_probe > gpurun_out/lat_probe.log 2>&1; cat gpurun_out/lat_probe.log
timeout -k 10 300 python tests/test_compat.py latency 4 2000 > gpurun_out/latency.log 2>&1; cat gpurun_out/latency.log

#!/bin/bash
# Round-4 GPU step: the GPU suite, decode A/B, the latency probe, snappy A/B.
set -e
mkdir -p gpurun_out
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/t.log 2>&1 || rc=$?
grep -E "^FAILED|passed|failed" gpurun_out/t.log | tail -30
[ $rc -le 1 ] || exit $rc
bash tools/ab_decode.sh "prev" "4 1" > /dev/null && cat gpurun_out/ab.log
timeout -k 10 120 tools/micro/lat_probe > gpurun_out/lat_probe.log 2>&1; cat gpurun_out/lat_probe.log
for c in 4 3; do
  timeout -k 10 200 python tools/time_snappy.py $c 1000000 5 >> gpurun_out/snz.log 2>&1
  RR_LIB=librr_serdes_snzA.so timeout -k 10 200 python tools/time_snappy.py $c 1000000 5 >> gpurun_out/snz.log 2>&1
done; grep -v amdgpu.ids gpurun_out/snz.log
bash tools/kstats_decode.sh gpurun_out/ks4 librr_serdes.so 4
bash tools/kstats_decode.sh gpurun_out/ks1 librr_serdes.so 1

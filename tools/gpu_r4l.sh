#!/bin/bash
# Round-4 GPU step: the GPU suite; decode A/B (first_off + zero kernel) on 1M configs 4, 1, 2 and
# the 100K config 1; encode A/B; the latency bench; the 100K timeline.
set -e
mkdir -p gpurun_out
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/t.log 2>&1 || rc=$?
grep -E "^FAILED|passed|failed" gpurun_out/t.log | tail -30
[ $rc -le 1 ] || exit $rc
bash tools/ab_decode.sh "prev" "4 1 2" > /dev/null && cat gpurun_out/ab.log
bash tools/ab_decode.sh "prev" "1" 100000 > /dev/null && cat gpurun_out/ab.log
bash tools/ab_encode.sh "prev" "4" > /dev/null && cat gpurun_out/ab_enc.log
timeout -k 10 300 python tests/test_compat.py latency 4 2000 > gpurun_out/latency.log 2>&1; cat gpurun_out/latency.log
bash tools/gpu_r4k.sh
rm -f gpurun_out/snz.log
for c in 4 3; do
  timeout -k 10 200 python tools/time_snappy.py $c 1000000 5 >> gpurun_out/snz.log 2>&1
  for w in 18432 17920; do RR_LIB=librr_serdes_snz$w.so timeout -k 10 200 python tools/time_snappy.py $c 1000000 5 >> gpurun_out/snz.log 2>&1; done
done; grep -v amdgpu.ids gpurun_out/snz.log

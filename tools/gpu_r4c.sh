#!/bin/bash
# Round-4 GPU step: the GPU suite, snappy PMC passes, then the timing legs of gpu_r4b.
set -e
mkdir -p gpurun_out
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/t.log 2>&1 || rc=$?
grep -E "^FAILED|passed|failed" gpurun_out/t.log | tail -30
[ $rc -le 1 ] || exit $rc
for c in 4 3; do timeout -k 10 200 python tools/time_snappy.py $c 1000000 5 >> gpurun_out/snz.log 2>&1; done; cat gpurun_out/snz.log
bash tools/pmc_snappy.sh gpurun_out/pmc_snz 4
python3 tools/pmc_by_kernel.py -a gpurun_out/pmc_snz/sq1 gpurun_out/pmc_snz/sq2 > gpurun_out/pmc_snz.txt; cat gpurun_out/pmc_snz.txt
timeout -k 10 300 python tests/test_compat.py latency 4 2000 > gpurun_out/latency.log 2>&1; cat gpurun_out/latency.log
bash tools/ab_decode.sh "prev" "4 1" > /dev/null && cat gpurun_out/ab.log
bash tools/ab_encode.sh "prev" "4" > /dev/null && cat gpurun_out/ab_enc.log
timeout -k 10 200 python tools/time_copy.py > gpurun_out/copy.log 2>&1; cat gpurun_out/copy.log
bash tools/kstats_decode.sh gpurun_out/ks4 librr_serdes.so 4
bash tools/kstats_decode.sh gpurun_out/ks1 librr_serdes.so 1
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1; tail -c 3000 gpurun_out/bench.log

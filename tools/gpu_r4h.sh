#!/bin/bash
# Round-4 GPU step: the GPU suite, decode A/B and per-kernel times, the latency bench.
set -e
mkdir -p gpurun_out
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/t.log 2>&1 || rc=$?
grep -E "^FAILED|passed|failed" gpurun_out/t.log | tail -30
[ $rc -le 1 ] || exit $rc
bash tools/ab_decode.sh "prev" "4 1 2" > /dev/null && cat gpurun_out/ab.log
bash tools/kstats_decode.sh gpurun_out/ks4 librr_serdes.so 4
bash tools/kstats_decode.sh gpurun_out/ks1 librr_serdes.so 1
bash tools/kstats_decode.sh gpurun_out/ks1p librr_serdes_prev.so 1
timeout -k 10 200 python tools/time_copy.py > gpurun_out/copy.log 2>&1; cat gpurun_out/copy.log
bash tools/pmc_snappy.sh gpurun_out/pmc_snz 4
python3 tools/pmc_by_kernel.py -a gpurun_out/pmc_snz/sq1 gpurun_out/pmc_snz/sq2 > gpurun_out/pmc_snz.txt; grep -A9 "snz_dec_kernel" gpurun_out/pmc_snz.txt

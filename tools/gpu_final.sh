#!/bin/bash
# One GPU call: the parity subset, an encode A/B against librr_serdes_prev.so, then the round's
# evidence (profiles, PMC, bench lines) and BASELINE.md's per-config rows.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_parity.py -m gpu -x -q --timeout 240 \
    --timeout-method thread -k "not config5 and not 10m" > gpurun_out/t.log 2>&1 && tail -1 gpurun_out/t.log
[ -f redrock_old_amd/librr_serdes_prev.so ] && bash tools/ab_encode.sh "prev" "4 3" > /dev/null && cat gpurun_out/ab_enc.log
bash tools/round_evidence.sh ${1:-r3}
bash tools/baseline_table.sh

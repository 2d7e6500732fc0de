#!/bin/bash
# Round-4 evidence (GPU box): the GPU suite, then the round's profiles and bench lines
# (tools/round_evidence.sh r4) and BASELINE.md's per-config lines (tools/baseline_table.sh).
set -e
mkdir -p gpurun_out
rc=0; timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/t.log 2>&1 || rc=$?
grep -E "^FAILED|passed|failed" gpurun_out/t.log | tail -30
[ $rc -eq 0 ] || exit 1
bash tools/round_evidence.sh r4

#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_dec.py > gpurun_out/diag.log 2>&1 || { cat gpurun_out/diag.log; exit 1; }
cat gpurun_out/diag.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/t.log 2>&1 || true
grep -E "FAILED|passed|failed" gpurun_out/t.log | tail -40

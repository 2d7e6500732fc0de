#!/bin/bash
# round-3 experiment batch (GPU box): parity of the default build, decode A/B, probes
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t5.log 2>&1
echo "parity rc=$?"; tail -2 gpurun_out/t5.log
timeout -k 10 400 bash tools/ab_decode.sh "${1:-zlold}" "${2:-4 3 2}" > /dev/null 2>&1; cat gpurun_out/ab.log
for v in ${3:-probe probezlold}; do for c in ${4:-4 3}; do RR_LIB=librr_serdes_$v.so timeout -k 10 100 python tools/probe_decode.py $c 1000000; done; done

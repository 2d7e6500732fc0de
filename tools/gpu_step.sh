#!/bin/bash
# One GPU call of the round's build loop (GPU box, repo root): the decode / encode parity tests,
# then A/B timings of the default library against the variants named in $1.
# usage: tools/gpu_step.sh "variants" ["pytest -k expression"]
set -e
mkdir -p gpurun_out
K=${2:-"not full_size and not config5"}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_encode.py -m gpu -x -q --timeout 240 \
    --timeout-method thread -k "$K" > gpurun_out/gpu_step_tests.log 2>&1 && echo "tests ok" || { tail -30 gpurun_out/gpu_step_tests.log; exit 1; }
tail -2 gpurun_out/gpu_step_tests.log
bash tools/ab_decode.sh "$1" "4 3 2" > /dev/null && cat gpurun_out/ab.log
bash tools/ab_encode.sh "$1" "4 3" > /dev/null && cat gpurun_out/ab_enc.log

set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_compat.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_t.log 2>&1
echo done

set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "fuzz" --timeout 300 --timeout-method thread > gpurun_out/fuzz1.log 2>&1
echo done

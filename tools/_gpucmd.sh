set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_snappy.py tests/test_compat.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/snz_t.log 2>&1
echo done

set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_snappy.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/snz2.log 2>&1
echo done

set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_compat.py -m gpu -v --timeout 200 --timeout-method thread -s > gpurun_out/kv1.log 2>&1
echo done

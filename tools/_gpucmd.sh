set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_snappy.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/snz6.log 2>&1
timeout -k 10 120 python -u tools/time_snappy.py 4 1000000 3 16384 > gpurun_out/tsnz5.log 2>&1
timeout -k 10 120 python -u tools/time_snappy.py 3 1000000 3 16384 >> gpurun_out/tsnz5.log 2>&1
echo done

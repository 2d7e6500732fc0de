set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_snappy.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/snz7.log 2>&1
for c in 4 3; do timeout -k 10 120 python -u tools/time_snappy.py $c 1000000 3 16384 | grep -v decompress > gpurun_out/tsnz7_$c.log 2>&1; done
echo done

set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_snappy.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/snz_t.log 2>&1
rm -f gpurun_out/snz.log
for c in 4 3 2; do timeout -k 10 120 python tools/time_snappy.py $c 1000000 5 >> gpurun_out/snz.log 2>&1; done
echo done

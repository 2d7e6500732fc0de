set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_dist.py tests/test_gpu_encode.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_t.log 2>&1
rm -f gpurun_out/dprof.log
for c in 4 3 2; do timeout -k 10 100 python tools/time_decode.py $c | grep cfg >> gpurun_out/dprof.log; done
timeout -k 10 600 python bench.py --no-snappy --no-split > gpurun_out/bench.json 2> gpurun_out/bench.err
echo done

set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -rf > gpurun_out/t18.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/r2_bench2.log 2>&1
echo done

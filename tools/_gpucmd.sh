timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/t5.log 2>&1; echo rc=$? >> gpurun_out/t5.log
timeout -k 10 300 python bench.py --n 10000000 --no-cpu --no-host --steps 10 --warmup 3 > gpurun_out/b5_10m.json 2> gpurun_out/b5_10m.err
timeout -k 10 300 python bench.py --no-cpu --no-host > gpurun_out/b5.json 2> gpurun_out/b5.err

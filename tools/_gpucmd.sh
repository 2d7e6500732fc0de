set -e
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --n 10000000 --steps 10 --warmup 2 --no-cpu --no-split --no-snappy > gpurun_out/bench10m.json 2> gpurun_out/bench10m.err
echo done

set -e
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
echo done

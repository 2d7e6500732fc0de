#!/bin/bash
# Round-end check on the GPU box (repo root): the GPU suite, smoke(), and the round's two bench
# lines (tools/bench_lines.sh r4 -> gpurun_out/ev/).
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/final_tests.log 2>&1; grep -E "passed|failed" gpurun_out/final_tests.log | tail -3
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1; tail -1 gpurun_out/final_smoke.log
bash tools/bench_lines.sh r4 > /dev/null
python3 -c "import json; d=json.load(open('gpurun_out/ev/r4_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['encode']['gib_s'], d['snappy']['compress'], d['snappy']['decompress']['GBs_output'], d['snappy']['cpu_16t'])"

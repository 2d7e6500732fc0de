#!/bin/bash
# Round-end check on the GPU box (repo root): the GPU suite, smoke(), and one default bench line.
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/final_tests.log 2>&1; grep -E "passed|failed" gpurun_out/final_tests.log | tail -3
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1; tail -1 gpurun_out/final_smoke.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/final_bench.log 2>&1; grep '^{' gpurun_out/final_bench.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['encode']['gib_s'])"

#!/bin/bash
# Round-4 GPU step: one system release per one-launch kernel — small-path and compat GPU tests,
# the latency probe, and per-value latency through the shim.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_small.py tests/test_compat.py -m gpu > gpurun_out/ee_tests.log 2>&1; tail -2 gpurun_out/ee_tests.log
timeout -k 10 120 ./tools/micro/lat_probe > gpurun_out/lat3.json 2> gpurun_out/lat3.err; cat gpurun_out/lat3.json
: > gpurun_out/latee.log
for rep in 1 2; do for c in 4 1; do
  echo "cfg$c" >> gpurun_out/latee.log
  timeout -k 10 200 python tests/test_compat.py latency $c 2000 2>&1 | grep '^{' >> gpurun_out/latee.log
done; done
python3 - <<'PY'
import json
for l in open("gpurun_out/latee.log"):
    if l.startswith("{"):
        d = json.loads(l); print(tag, d["shim_desObject_us"]["median"], d["shim_serObject_us"]["median"], d["decode_host_n1_small_us"]["median"])
    else:
        tag = l.strip()
PY

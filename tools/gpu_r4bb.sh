#!/bin/bash
# Round-4 GPU step: the compat shim's serialize path with per-thread buffers kept across calls —
# the compat GPU tests, then per-value latency (current vs the committed build's shim, both
# over the same library: tests/test_compat.py builds the shim from source each run).
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_compat.py -m gpu > gpurun_out/bb_tests.log 2>&1; tail -2 gpurun_out/bb_tests.log
: > gpurun_out/latbb.log
for rep in 1 2 3; do for c in 4 1; do
  echo "cur cfg$c" >> gpurun_out/latbb.log
  timeout -k 10 200 python tests/test_compat.py latency $c 2000 2>&1 | grep '^{' >> gpurun_out/latbb.log
done; done
python3 - <<'PY'
import json
for l in open("gpurun_out/latbb.log"):
    if l.startswith("{"):
        d = json.loads(l); print(tag, d["shim_desObject_us"]["median"], d["shim_serObject_us"]["median"], d["decode_host_n1_small_us"]["median"])
    else:
        tag = l.strip()
PY

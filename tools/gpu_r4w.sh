#!/bin/bash
# Round-4 GPU step: one-launch kernels with LDS-only barriers after their host-visible stores —
# the small-path and compat GPU tests, then per-value latency through the shim against the
# committed build (LD_LIBRARY_PATH picks redrock_old_amd/headlib/librr_serdes.so).
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_small.py tests/test_compat.py -m gpu > gpurun_out/w_tests.log 2>&1; tail -3 gpurun_out/w_tests.log
: > gpurun_out/latab.log
for rep in 1 2; do for c in 4 1; do
  echo "cur cfg$c" >> gpurun_out/latab.log
  timeout -k 10 200 python tests/test_compat.py latency $c 2000 2>&1 | grep '^{' >> gpurun_out/latab.log
  echo "head cfg$c" >> gpurun_out/latab.log
  LD_LIBRARY_PATH=$PWD/redrock_old_amd/headlib timeout -k 10 200 python tests/test_compat.py latency $c 2000 2>&1 | grep '^{' >> gpurun_out/latab.log
done; done
python3 - <<'PY'
import json
for l in open("gpurun_out/latab.log"):
    if l.startswith("{"):
        d = json.loads(l); print(tag, d["shim_desObject_us"]["median"], d["shim_serObject_us"]["median"], d["decode_host_n1_small_us"]["median"])
    else:
        tag = l.strip()
PY

# The round's verification command (GPU box, repo root): every GPU test, the smoke test, the
# default bench line.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_all.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/smoke.log 2>&1
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
echo done

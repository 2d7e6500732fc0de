set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/t19.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke19.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/r2_bench3.log 2>&1
timeout -k 10 400 bash tools/profile_bench.sh gpurun_out/r2prof3
echo done

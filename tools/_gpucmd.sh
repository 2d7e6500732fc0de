set -e
mkdir -p gpurun_out
cd tests && PYTHONPATH=.. timeout -k 10 200 python -u test_compat.py bench > ../gpurun_out/rdbbench.log 2>&1
echo done

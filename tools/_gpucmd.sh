set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t17.log 2>&1
CONFIGS="4 3" timeout -k 10 300 bash tools/var_sweep.sh > gpurun_out/sweep2.log 2>&1
CONFIGS="4 3" timeout -k 10 300 bash tools/var_sweep.sh >> gpurun_out/sweep2.log 2>&1
RR_LIB=librr_serdes_probe.so timeout -k 10 100 python tools/probe_decode.py 4 > gpurun_out/probe2.log 2>&1
echo done

timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t3.log 2>&1; echo rc=$? >> gpurun_out/t3.log
CONFIGS="4 3" timeout -k 10 300 bash tools/var_sweep.sh > gpurun_out/sweep3.log 2>&1
RR_LIB=librr_serdes_probe.so timeout -k 10 120 python tools/probe_decode.py 4 > gpurun_out/probe3.log 2>&1

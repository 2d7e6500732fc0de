timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -rf > gpurun_out/t11.log 2>&1; echo rc=$? >> gpurun_out/t11.log
CONFIGS="4 3 2" timeout -k 10 300 bash tools/var_sweep.sh > gpurun_out/sweep11.log 2>&1
RR_LIB=librr_serdes_probe.so timeout -k 10 120 python tools/probe_decode.py 4 > gpurun_out/probe11.log 2>&1

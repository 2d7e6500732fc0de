set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/enc_t.log 2>&1
rm -f gpurun_out/encsweep.log gpurun_out/eprobe.log
for r in 1 2; do for c in 4 3 2; do timeout -k 10 100 python tools/time_encode.py $c 2>&1 | grep cfg >> gpurun_out/encsweep.log; done; done
RR_LIB=librr_serdes_probe.so timeout -k 10 100 python tools/probe_encode.py 4 >> gpurun_out/eprobe.log 2>&1
echo done

set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_dist.py tests/test_gpu_encode.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/pf1.log 2>&1
rm -f gpurun_out/pfsweep.log
for r in 1 2; do for L in librr_serdes.so librr_serdes_nopf.so; do for c in 4 3 2; do RR_LIB=$L timeout -k 10 100 python tools/time_decode.py $c | grep cfg >> gpurun_out/pfsweep.log; done; done; done
RR_LIB=librr_serdes_probe.so timeout -k 10 100 python tools/probe_decode.py 4 > gpurun_out/probe_pf.log 2>&1
echo done

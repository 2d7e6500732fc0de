set -e
mkdir -p gpurun_out
rm -f gpurun_out/esweep.log
RR_LIB=librr_serdes_gearly.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "golden or config_parity or full_size or fuzz" --timeout 200 --timeout-method thread > gpurun_out/early_t.log 2>&1
for r in 1 2; do for L in librr_serdes.so librr_serdes_gearly.so librr_serdes_rearly.so; do for c in 4 3 2; do RR_LIB=$L timeout -k 10 100 python tools/time_decode.py $c | grep cfg >> gpurun_out/esweep.log; done; done; done
RR_LIB=librr_serdes_pgearly.so timeout -k 10 100 python tools/probe_decode.py 4 > gpurun_out/probe_early.log 2>&1
echo done

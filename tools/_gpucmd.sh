set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_encode.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/enc_t.log 2>&1
RR_LIB=librr_serdes_e6.so timeout -k 10 300 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread >> gpurun_out/enc_t.log 2>&1
rm -f gpurun_out/encsweep.log
for r in 1 2; do for L in librr_serdes.so librr_serdes_e6.so; do for c in 4 3 2; do RR_LIB=$L timeout -k 10 100 python tools/time_encode.py $c 2>&1 | grep cfg >> gpurun_out/encsweep.log; done; done; done
echo done

set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_dist.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/ovl_t.log 2>&1
rm -f gpurun_out/ovlsweep.log
for r in 1 2; do for L in librr_serdes.so librr_serdes_k4.so librr_serdes_k6.so librr_serdes_noovl.so; do for c in 4 3 2; do RR_LIB=$L timeout -k 10 100 python tools/time_decode.py $c | grep cfg >> gpurun_out/ovlsweep.log; done; done; done
RR_LIB=librr_serdes_probe.so timeout -k 10 100 python tools/probe_decode.py 4 > gpurun_out/probe_ovl.log 2>&1
echo done

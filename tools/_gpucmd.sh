set -e
mkdir -p gpurun_out
rm -f gpurun_out/tsnz4.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_snappy.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/snz5.log 2>&1
for L in librr_serdes.so librr_serdes_a4_32.so librr_serdes_a8_64.so librr_serdes_a16_16.so librr_serdes_a4_16.so; do
  for c in 4 3; do RR_LIB=$L timeout -k 10 120 python -u tools/time_snappy.py $c 1000000 3 16384 | grep compress >> gpurun_out/tsnz4.log 2>&1; echo $L >> gpurun_out/tsnz4.log; done
done
echo done

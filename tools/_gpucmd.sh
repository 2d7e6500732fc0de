set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
timeout -k 10 300 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/enc_t.log 2>&1
cd /tmp
for c in 4 2 3; do for L in librr_serdes.so librr_serdes_s8.so librr_serdes_s2.so librr_serdes_u1.so; do
  RR_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_${c}_${L} -o run -- python3 $R/tools/time_encode.py $c > /tmp/o.log 2>&1
  f=$(find /tmp/p_${c}_${L} -name '*kernel_stats.csv' | head -1); echo "== cfg $c $L $(grep cfg= /tmp/o.log)" >> $R/gpurun_out/eprof.log; python3 $R/tools/kstats.py $f | grep -v at::native >> $R/gpurun_out/eprof.log
done; done
echo done

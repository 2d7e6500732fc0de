set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_encode.py tests/test_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_t.log 2>&1
rm -f gpurun_out/dprof.log
cd /tmp
for c in 4 2; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pd_${c} -o run -- python3 $R/tools/time_decode.py $c > /tmp/o.log 2>&1
  f=$(find /tmp/pd_${c} -name '*kernel_stats.csv' | head -1); echo "== dec cfg $c $(grep cfg /tmp/o.log)" >> $R/gpurun_out/dprof.log; python3 $R/tools/kstats.py $f | grep -v at::native >> $R/gpurun_out/dprof.log
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pe_${c} -o run -- python3 $R/tools/time_encode.py $c > /tmp/o.log 2>&1
  f=$(find /tmp/pe_${c} -name '*kernel_stats.csv' | head -1); echo "== enc cfg $c $(grep cfg= /tmp/o.log)" >> $R/gpurun_out/dprof.log; python3 $R/tools/kstats.py $f | grep -v at::native >> $R/gpurun_out/dprof.log
done
cd $R
for c in 4 3 2; do timeout -k 10 100 python tools/time_decode.py $c | grep cfg >> gpurun_out/dprof.log; timeout -k 10 100 python tools/time_encode.py $c | grep cfg >> gpurun_out/dprof.log; done
echo done

set -e
mkdir -p gpurun_out
rm -f gpurun_out/nsweep.log
for n in 250000 500000 1000000 2000000 4000000 8000000; do timeout -k 10 200 python tools/time_decode.py 4 $n | grep cfg >> gpurun_out/nsweep.log; done
echo done

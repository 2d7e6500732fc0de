#!/bin/bash
# A/B of the snappy kernels (GPU box, repo root): tools/time_snappy.py on the default library and
# the variants in $1, configs $2, two alternations; then the GPU snappy suite on each library in $3.
set -e
mkdir -p gpurun_out
out=gpurun_out/ab_snappy.log
: > $out
for rep in 1 2; do
  for cfg in ${2:-4 3 2}; do
    for v in default $1; do
      lib=librr_serdes_$v.so; [ $v = default ] && lib=librr_serdes.so
      echo "== $v cfg $cfg" >> $out
      RR_LIB=$lib timeout -k 10 200 python tools/time_snappy.py $cfg 1000000 3 | grep -E "ratio|compress" >> $out
    done
  done
done
cat $out
for v in $3; do
  lib=librr_serdes_$v.so; [ $v = default ] && lib=librr_serdes.so
  RR_LIB=$lib timeout -k 10 400 python -u -m pytest tests/test_gpu_snappy.py -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/snappy_suite_$v.log 2>&1 && echo "snappy suite $v: $(tail -1 gpurun_out/snappy_suite_$v.log)" \
    || { echo "snappy suite $v FAILED"; tail -40 gpurun_out/snappy_suite_$v.log; exit 1; }
done

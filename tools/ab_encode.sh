#!/bin/bash
# A/B timing of encode builds on the GPU box (diagnostics): default library vs variants.
# usage: tools/ab_encode.sh "variant1 variant2 ..." "cfgs"
set -e
mkdir -p gpurun_out
out=gpurun_out/ab_enc.log
: > $out
for rep in 1 2; do
  for cfg in ${2:-4}; do
    timeout -k 10 120 python tools/time_encode.py $cfg 1000000 20 | grep -v amdgpu >> $out
    for v in $1; do
      RR_LIB=librr_serdes_$v.so timeout -k 10 120 python tools/time_encode.py $cfg 1000000 20 | grep -v amdgpu >> $out
    done
  done
done
cat $out

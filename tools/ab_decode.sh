#!/bin/bash
# A/B timing of decode builds on the GPU box (diagnostics): default library vs variants.
# usage: tools/ab_decode.sh "variant1 variant2 ..." "cfgs" [n]
set -e
mkdir -p gpurun_out
out=gpurun_out/ab.log
: > $out
vars=${1:-old}; cfgs=${2:-4}; n=${3:-1000000}
for rep in 1 2; do
  for cfg in $cfgs; do
    timeout -k 10 120 python tools/time_decode.py $cfg $n 20 | grep cfg >> $out
    for v in $vars; do
      RR_LIB=librr_serdes_$v.so timeout -k 10 120 python tools/time_decode.py $cfg $n 20 | grep cfg >> $out
    done
  done
done
cat $out

#!/bin/bash
# Kernel times against the batch size (diagnostics, GPU box): does a kernel's time step with its
# count of resident-grid generations?  usage: tools/gen_sweep.sh "n1 n2 ..." [config]
CFG=${2:-4}
for N in $1; do
  echo "== n=$N"
  RR_N=$N bash tools/kstats_decode.sh gpurun_out/gs/dec_$N librr_serdes.so $CFG || exit 1
  RR_N=$N bash tools/kstats_encode.sh gpurun_out/gs/enc_$N librr_serdes.so $CFG || exit 1
done

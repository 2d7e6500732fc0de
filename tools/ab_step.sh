#!/bin/bash
# An A/B step of round 6 (GPU box, repo root): decode timings of the default library against the
# variants named in $1 (tools/ab_decode.sh), per-kernel durations of each (tools/kstats_decode.sh),
# and the parity subset on each variant listed in $2 (RR_LIB).  Each step under its own limit.
# usage: tools/ab_step.sh "variants" "parity-variants" [cfgs]
set -e
mkdir -p gpurun_out
bash tools/ab_decode.sh "$1" "${3:-4 3}" > /dev/null && cat gpurun_out/ab.log
for v in default $1; do
  lib=librr_serdes_$v.so; [ $v = default ] && lib=librr_serdes.so
  bash tools/kstats_decode.sh gpurun_out/ks_$v $lib 4 | grep -E "count_kernel|decode_kernel" | sed "s/^/$v /"
done
for v in $2; do
  RR_LIB=librr_serdes_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_small.py -m gpu -x -q \
     --timeout 240 --timeout-method thread -k "not full_size and not config5 and not uneven" > gpurun_out/parity_$v.log 2>&1 \
     && echo "parity $v: $(tail -1 gpurun_out/parity_$v.log)" || { echo "parity $v FAILED"; tail -30 gpurun_out/parity_$v.log; exit 1; }
done

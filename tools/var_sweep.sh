#!/bin/bash
# Times every in-tree decode variant library (redrock_old_amd/librr_serdes*.so) on configs 4 and 3.
set -e
for lib in $(cd redrock_old_amd && ls librr_serdes*.so); do
  for c in ${CONFIGS:-4 3}; do RR_LIB=$lib timeout -k 10 120 python tools/time_decode.py $c; done
done

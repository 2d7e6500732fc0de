#!/bin/bash
# Times every in-tree decode variant library (redrock_old_amd/librr_serdes*.so, except the
# probe build, which needs tools/probe_decode.py) on the configs in $CONFIGS (default 4 3).
set -e
for lib in $(cd redrock_old_amd && ls librr_serdes*.so | grep -v probe); do
  for c in ${CONFIGS:-4 3}; do RR_LIB=$lib timeout -k 10 120 python tools/time_decode.py $c; done
done

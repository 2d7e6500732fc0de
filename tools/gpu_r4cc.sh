#!/bin/bash
# Round-4 GPU step: ds_permute semantics probe, then the snappy compressor with its overwrite
# marks through ds_permute (perm: no mark words in LDS, 5 waves per CU) — snappy GPU tests on
# it, then timing against the current build.
set -e
mkdir -p gpurun_out
timeout -k 10 60 ./tools/micro/permute_probe
RR_LIB=librr_serdes_perm.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_snappy.py > gpurun_out/cc_tests.log 2>&1; tail -2 gpurun_out/cc_tests.log
: > gpurun_out/abcomp.log
for rep in 1 2; do for c in 4 3; do for v in librr_serdes.so librr_serdes_perm.so; do
  echo "$v" >> gpurun_out/abcomp.log
  RR_LIB=$v timeout -k 10 200 python tools/time_snappy.py $c 1000000 5 2>&1 | grep -v amdgpu.ids | grep compress >> gpurun_out/abcomp.log
done; done; done
cat gpurun_out/abcomp.log

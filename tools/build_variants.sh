#!/bin/bash
# Builds decode tuning variants as redrock_old_amd/librr_serdes_<name>.so (diagnostics only).
# usage: tools/build_variants.sh name "-DRR_DEC_WIN=8192 -DRR_DEC_SLACK=4096" [name2 "flags2" ...]
set -e
cd "$(dirname "$0")/../redrock_old_amd/csrc"
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  mkdir -p ../../build/var_$name
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 $flags -c rr_kernels.hip -o ../../build/var_$name/k.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 $flags -c rr_snappy.hip -o ../../build/var_$name/s.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../librr_serdes_$name.so ../../build/var_$name/k.o ../../build/var_$name/s.o ../../build/csrc/rr_api.o ../../build/csrc/rr_shard.o ../../build/csrc/rr_snappy_api.o ../../build/csrc/rr_rdb.o ../../build/csrc/rr_kv.o ../../build/csrc/rr_gen.o ../../build/csrc/rr_host.o -L/opt/rocm/lib -lrccl -lm
  echo built librr_serdes_$name.so
done

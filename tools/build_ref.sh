#!/bin/bash
# Builds the kernels of a git revision as redrock_old_amd/librr_serdes_<name>.so (A/B timing
# against the working tree on the same GPU box; diagnostics only).  The host objects are the
# working tree's, so the launch ABI (rr_kernels.h) must be unchanged between the two.
# usage: tools/build_ref.sh <rev> <name> ["-DEXTRA ..."]
set -e
rev=$1; name=$2; flags=$3
root=$(cd "$(dirname "$0")/.." && pwd)
src=$root/build/ref_$name/src; obj=$root/build/ref_$name
rm -rf "$src"; mkdir -p "$src/redrock_old_amd/csrc" "$src/include"
for f in $(git -C "$root" ls-tree --name-only "$rev" redrock_old_amd/csrc/ include/); do
  git -C "$root" show "$rev:$f" > "$src/$f"
done
make -C "$root/redrock_old_amd/csrc" >/dev/null
cd "$src/redrock_old_amd/csrc"
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 $flags"
$H -c rr_kernels.hip -o "$obj/k.o"
$H -c rr_snappy.hip -o "$obj/s.o"
B=$root/build/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$root/redrock_old_amd/librr_serdes_$name.so" "$obj/k.o" "$obj/s.o" \
  $B/rr_api.o $B/rr_shard.o $B/rr_snappy_api.o $B/rr_rdb.o $B/rr_kv.o $B/rr_gen.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -lm
echo "built librr_serdes_$name.so from $rev"

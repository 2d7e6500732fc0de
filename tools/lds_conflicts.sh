#!/bin/bash
# LDS bank-conflict attribution (GPU box, repo root): SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
# and LDS instruction counts of the decode for ablation builds (copy+stage only, + class sort,
# full) into gpurun_out/lds/<lib>.  usage: tools/lds_conflicts.sh "lib1 lib2 ..."
ROOT=$(pwd)
mkdir -p gpurun_out/lds
cd /tmp && export TMPDIR=/tmp
for L in $1; do
  RR_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS \
      --output-format csv -d $ROOT/gpurun_out/lds/$L -o run -- python3 $ROOT/tools/time_decode.py 4 1000000 3 \
      > $ROOT/gpurun_out/lds/$L.log 2>&1 || { echo "$L failed"; exit 1; }
  python3 - "$ROOT/gpurun_out/lds/$L" <<'PY'
import csv, glob, sys, collections
tot = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for p in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").split("::")[-1]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in tot.items():
    if "decode_kernel" in k or "count_kernel" in k:
        bc, ia = c.get("SQ_LDS_BANK_CONFLICT", 0), c.get("SQ_LDS_IDX_ACTIVE", 0)
        print(f"{sys.argv[1].split('/')[-1]:28s} {k:20s} conflict/active {bc / max(ia, 1):.3f}  LDS insts {c.get('SQ_INSTS_LDS', 0):.3e}"
              f"  wait_inst_lds/wave_cycles {c.get('SQ_WAIT_INST_LDS', 0) / max(c.get('SQ_WAVE_CYCLES', 1), 1):.3f}")
PY
done

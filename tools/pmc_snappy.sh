#!/bin/bash
# SQ counter passes over the snappy kernels (tools/time_snappy.py), one counter group per pass.
# Usage (GPU box, from the repo root): bash tools/pmc_snappy.sh OUTDIR [config]
set -e
OUT=$(realpath -m "$1"); CFG=${2:-4}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {  # name counters...
    local name=$1; shift
    timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
        python3 "$ROOT/tools/time_snappy.py" "$CFG" 1000000 2 > "$OUT/$name.log" 2>&1
}
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY
run sq2 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE

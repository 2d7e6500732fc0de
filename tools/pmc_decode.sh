#!/bin/bash
# PMC passes over the decode pipeline (tools/time_decode.py), one counter group per pass.
# Usage (GPU box, from the repo root): bash tools/pmc_decode.sh OUTDIR [config]
set -e
OUT=$(realpath -m "$1"); CFG=${2:-4}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
run() {  # name counters...
    local name=$1; shift
    timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
        python3 "$ROOT/tools/time_decode.py" "$CFG" 1000000 3 > "$OUT/$name.log" 2>&1
}
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$ROOT/tools/time_decode.py" "$CFG" 1000000 10 > "$OUT/trace.log" 2>&1
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY
run sq2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
run fetch FETCH_SIZE
run write WRITE_SIZE
run tcc TCC_HIT_sum TCC_MISS_sum

set -e
mkdir -p gpurun_out/snzpmc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/snzpmc/sq1 -o run -- python3 $GRAFT_REPO_ROOT/tools/time_snappy.py 4 200000 1 > $GRAFT_REPO_ROOT/gpurun_out/snzpmc/sq1.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/snzpmc/sq2 -o run -- python3 $GRAFT_REPO_ROOT/tools/time_snappy.py 4 200000 1 > $GRAFT_REPO_ROOT/gpurun_out/snzpmc/sq2.log 2>&1
echo done

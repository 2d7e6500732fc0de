set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/r2_bench.log 2>&1
tail -1 gpurun_out/r2_bench.log > gpurun_out/r2_bench.json
timeout -k 10 400 bash tools/profile_bench.sh gpurun_out/r2prof
RR_PROFILE=encode timeout -k 10 400 bash tools/profile_bench.sh gpurun_out/r2prof_enc
timeout -k 10 600 bash tools/pmc_decode.sh gpurun_out/r2pmc 4
echo done

set -e
mkdir -p gpurun_out
rm -rf gpurun_out/pmc_r2b
timeout -k 10 900 bash tools/pmc_decode.sh gpurun_out/pmc_r2b 4
echo done

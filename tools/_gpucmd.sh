for i in 1 2; do CONFIGS="4" timeout -k 10 300 bash tools/var_sweep.sh; done > gpurun_out/sweep9.log 2>&1

#!/bin/bash
# Round-4 GPU step: per-kernel durations of config 1 at 100K values and config 4 at 1M (no
# zeroing launch), and the per-value latency probe.
set -e
mkdir -p gpurun_out
RR_N=100000 bash tools/kstats_decode.sh gpurun_out/ks_c1_100k librr_serdes.so 1
bash tools/kstats_decode.sh gpurun_out/ks_c4 librr_serdes.so 4
timeout -k 10 120 ./tools/micro/lat_probe > gpurun_out/lat.json 2> gpurun_out/lat.err; cat gpurun_out/lat.json

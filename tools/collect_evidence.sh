#!/bin/bash
# Local (this container): the GPU call's gpurun_out/ev and gpurun_out/bl -> the committed
# profiles/ files of round ROUNDTAG.  usage: tools/collect_evidence.sh ROUNDTAG
set -e
R=${1:-r3}
E=gpurun_out/ev
python3 tools/traffic_summary.py $E/dec profiles/${R}_decode_summary.json > /dev/null
python3 tools/traffic_summary.py $E/enc profiles/${R}_encode_summary.json > /dev/null
cp $E/dec/trace/run_kernel_stats.csv profiles/${R}_decode_kernel_stats.csv
cp $E/enc/trace/run_kernel_stats.csv profiles/${R}_encode_kernel_stats.csv
python3 tools/pmc_summary.py $E/pmc > profiles/${R}_decode_pmc.txt 2>&1
cp $E/${R}_bench.json profiles/${R}_bench.json
cp $E/${R}_bench_10m.json profiles/${R}_bench_10m.json
for f in gpurun_out/bl/*.json; do cp "$f" profiles/${R}_bench_$(basename "$f"); done
ls -la profiles/${R}_*

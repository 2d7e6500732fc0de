#!/bin/bash
# The round's profile evidence + bench lines in one GPU call (GPU box, repo root):
#   gpurun_out/ev/{dec,enc}   rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes (profile_bench.sh)
#   gpurun_out/ev/pmc         SQ / TCC counter passes of the decode (pmc_decode.sh)
#   gpurun_out/ev/*.json      traffic summaries and the bench.py lines (1M default, 10M config 4)
# The decode summary is copied into profiles/ first, so bench.py's roofline.traffic comes
# from this build.  usage: tools/round_evidence.sh ROUNDTAG (e.g. r2)
set -e
R=${1:-r2}
E=gpurun_out/ev
mkdir -p $E
cp profiles/${R}_decode_summary.json $E/${R}_decode_summary.json 2>/dev/null || true
cp profiles/${R}_encode_summary.json $E/${R}_encode_summary.json 2>/dev/null || true
bash tools/profile_bench.sh $E/dec && echo "decode profile done"
RR_PROFILE=encode bash tools/profile_bench.sh $E/enc && echo "encode profile done"
python3 tools/traffic_summary.py $E/dec $E/${R}_decode_summary.json > /dev/null
python3 tools/traffic_summary.py $E/enc $E/${R}_encode_summary.json > /dev/null
cp $E/${R}_decode_summary.json profiles/${R}_decode_summary.json
bash tools/pmc_decode.sh $E/pmc 4 && echo "pmc done"
python3 tools/pmc_summary.py $E/pmc > $E/${R}_decode_pmc.txt 2>&1 || true
bash tools/bench_lines.sh $R

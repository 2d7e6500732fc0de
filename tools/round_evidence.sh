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
timeout -k 10 600 python3 -u bench.py > $E/bench.log 2>&1 && echo "bench done"
grep '^{' $E/bench.log | tail -1 > $E/${R}_bench.json
timeout -k 10 600 python3 -u bench.py --n 10000000 --steps 10 --warmup 2 --no-cpu --no-split --no-snappy > $E/bench10m.log 2>&1 && echo "bench 10m done"
grep '^{' $E/bench10m.log | tail -1 > $E/${R}_bench_10m.json
cat $E/${R}_bench.json

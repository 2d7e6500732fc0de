#!/bin/bash
# One GPU call of round 6 (GPU box, repo root): the GPU suite, the compat shim's call-pattern and
# latency benches, and the bench line.  Each step under its own time limit; the first failure ends it.
# usage: tools/gpu_round.sh TAG [steps...]   steps: suite callpattern latency bench (default: all)
set -e
tag=$1; shift
steps=${*:-"suite callpattern latency bench"}
mkdir -p gpurun_out
for s in $steps; do
  case $s in
    suite) timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
             > gpurun_out/${tag}_suite.log 2>&1 || { tail -40 gpurun_out/${tag}_suite.log; exit 1; }
           tail -3 gpurun_out/${tag}_suite.log ;;
    callpattern) timeout -k 10 600 python tests/test_compat.py callpattern 4 > gpurun_out/${tag}_callpattern.txt 2>&1
           tail -c 3000 gpurun_out/${tag}_callpattern.txt ;;
    latency) for c in 4 1 3; do timeout -k 10 300 python tests/test_compat.py latency $c 2000; done \
             > gpurun_out/${tag}_latency.txt 2>&1; cat gpurun_out/${tag}_latency.txt ;;
    bench) timeout -k 10 600 python bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
           tail -c 2500 gpurun_out/${tag}_bench.json ;;
  esac
done

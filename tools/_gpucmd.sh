timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/t15.log 2>&1; echo rc=$? >> gpurun_out/t15.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof15 -o run -- python3 $GRAFT_REPO_ROOT/tools/time_decode.py 4 1000000 10 > $GRAFT_REPO_ROOT/gpurun_out/prof15.log 2>&1
cd $GRAFT_REPO_ROOT && for i in 1 2; do timeout -k 10 100 python tools/time_decode.py 4; done > gpurun_out/time15.log 2>&1

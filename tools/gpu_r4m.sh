#!/bin/bash
# Round-4 GPU step: probe builds of the decode (config 1 at 100K, config 4 at 1M) and the encode.
set -e
mkdir -p gpurun_out
RR_LIB=librr_serdes_probe.so timeout -k 10 200 python tools/probe_decode.py 1 100000 > gpurun_out/probe1.log 2>&1; grep -v amdgpu.ids gpurun_out/probe1.log
RR_LIB=librr_serdes_probe.so timeout -k 10 200 python tools/probe_decode.py 4 1000000 > gpurun_out/probe4.log 2>&1; grep -v amdgpu.ids gpurun_out/probe4.log
RR_LIB=librr_serdes_probe.so timeout -k 10 200 python tools/probe_encode.py 4 1000000 > gpurun_out/eprobe4.log 2>&1; grep -v amdgpu.ids gpurun_out/eprobe4.log

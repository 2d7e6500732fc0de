#!/bin/bash
# Round-4 evidence, part 2 (GPU box): BASELINE.md's per-config bench lines and the probe builds.
set -e
bash tools/baseline_table.sh
bash tools/gpu_r4m.sh

#!/bin/bash
# Solo-rank timings (t_7 / t_8 flags as in the real run) and the CPU baseline
# scaling on this box's host (2^16 .. 2^20 and the full 2^22 instance).
set -o pipefail
mkdir -p gpurun_out/r03d
SOLO="0/2 0/4 0/8 7/8" TAG=r03d bash tools/gpu_solo.sh && \
timeout -k 10 1000 python -u tools/cpu_scaling.py --circuit merkle --lgs 16 17 18 19 20 22 \
    > gpurun_out/r03d/cpu_scaling_box.json 2> gpurun_out/r03d/cpu_scaling_box.err

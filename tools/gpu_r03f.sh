#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03f
SOLO="0/8 7/8 0/4 0/2" TAG=r03f bash tools/gpu_solo.sh && \
PNP_MSM_SHARD=points timeout -k 10 300 python -u bench.py --steps 5 --solo 0/8 > gpurun_out/r03f/points_0of8.json 2> gpurun_out/r03f/points_0of8.err && \
BENCH_ARGS="--solo 0/8" bash tools/prof_trace.sh r03f_trace 2

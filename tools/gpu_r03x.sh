#!/bin/bash
# After the copy-constraint wire groups: kernel trace + stats of the default bench,
# PMC passes (FETCH / WRITE / SQ) for the accumulate traffic, solo per-rank times.
set -o pipefail
mkdir -p gpurun_out/r03x
bash tools/prof_trace.sh r03x/trace 3 && echo "trace ok" && \
bash tools/pmc_run.sh r03x/pmc && echo "pmc ok" && \
TAG=r03x/solo SOLO="0/2 0/4 0/8 7/8" bash tools/gpu_solo.sh && echo "solo ok"

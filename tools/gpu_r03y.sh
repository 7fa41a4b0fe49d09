#!/bin/bash
# Radix-2^29 quotient: prove / Merkle / full-size golden tests, a same-box A/B
# (k_quotient29 vs PNP_QUOT29=0), then the kernel trace, PMC passes and solo times.
set -o pipefail
mkdir -p gpurun_out/r03y
timeout -k 10 700 python -u -m pytest tests/test_gpu_merkle.py tests/test_gpu_prove.py tests/test_gpu_full.py -m gpu -x -v \
    --timeout 300 --timeout-method thread > gpurun_out/r03y/pytest_first.log 2>&1 && echo "first tests ok" && \
bash tools/abn.sh 3 base PNP_QUOT29=0 > gpurun_out/r03y/ab.txt 2>&1 && echo "ab ok" && \
bash tools/prof_trace.sh r03y/trace 3 && echo "trace ok" && \
bash tools/pmc_run.sh r03y/pmc && echo "pmc ok" && \
TAG=r03y/solo SOLO="0/2 0/4 0/8 7/8" bash tools/gpu_solo.sh && echo "solo ok"

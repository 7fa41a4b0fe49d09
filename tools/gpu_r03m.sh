#!/bin/bash
# quotient gate terms on the side stream: A/B vs the previous library, solo 8-rank, GPU suite
set -o pipefail
mkdir -p gpurun_out/r03m
bash tools/abn.sh 3 base $PWD/ab_libs/lib_prev.so > gpurun_out/r03m/ab.txt 2>&1 && echo "ab ok" && \
SOLO="0/8" TAG=r03m bash tools/gpu_solo.sh && echo "solo ok" && \
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread \
    > gpurun_out/r03m/pytest.log 2>&1 && echo "pytest ok"

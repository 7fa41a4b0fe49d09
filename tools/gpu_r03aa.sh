#!/bin/bash
# z over its runs of sigma-fixed rows, group slots by bit reversal: Merkle / prove /
# full-size / sharded tests, A/B (z groups on / PNP_Z_GROUPS=0), solo per-rank times.
set -o pipefail
mkdir -p gpurun_out/r03aa
timeout -k 10 900 python -u -m pytest tests/test_gpu_merkle.py tests/test_gpu_prove.py tests/test_gpu_full.py \
    tests/test_gpu_lagrange.py tests/test_shard.py -m gpu -x -v --timeout 400 --timeout-method thread \
    > gpurun_out/r03aa/pytest_first.log 2>&1 && echo "first tests ok" && \
bash tools/abn.sh 3 base PNP_Z_GROUPS=0 > gpurun_out/r03aa/ab.txt 2>&1 && echo "ab ok" && \
TAG=r03aa/solo SOLO="0/2 0/4 0/8 7/8" bash tools/gpu_solo.sh && echo "solo ok"

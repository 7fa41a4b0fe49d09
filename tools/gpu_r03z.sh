#!/bin/bash
# Groups spread over n-slot segments, level-by-level table build, k_quotient29 at
# 4 waves/SIMD: prove / Merkle / full-size / sharded tests, A/B of the quotient,
# solo per-rank times.
set -o pipefail
mkdir -p gpurun_out/r03z
timeout -k 10 900 python -u -m pytest tests/test_gpu_merkle.py tests/test_gpu_prove.py tests/test_gpu_full.py \
    tests/test_gpu_lagrange.py tests/test_shard.py -m gpu -x -v --timeout 400 --timeout-method thread \
    > gpurun_out/r03z/pytest_first.log 2>&1 && echo "first tests ok" && \
bash tools/abn.sh 3 base PNP_QUOT29=0 > gpurun_out/r03z/ab.txt 2>&1 && echo "ab ok" && \
TAG=r03z/solo SOLO="0/2 0/4 0/8 7/8" bash tools/gpu_solo.sh && echo "solo ok"

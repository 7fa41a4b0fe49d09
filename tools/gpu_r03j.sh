#!/bin/bash
# Lagrange-basis wire commitments: unit tests, golden proofs, bench.
set -o pipefail
mkdir -p gpurun_out/r03j
timeout -k 10 600 python -u -m pytest tests/test_gpu_lagrange.py -x -v -s --timeout 300 --timeout-method thread \
    > gpurun_out/r03j/pytest_lag.log 2>&1 && echo "lagrange tests ok" && \
timeout -k 10 900 python -u -m pytest tests/test_gpu_full.py -x -v -s --timeout 600 --timeout-method thread -k "golden or merkle" \
    > gpurun_out/r03j/pytest_full.log 2>&1 && echo "golden ok" && \
timeout -k 10 600 python -u bench.py > gpurun_out/r03j/bench.json 2> gpurun_out/r03j/bench.err && echo "bench ok"

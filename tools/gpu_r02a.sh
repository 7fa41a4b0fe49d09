#!/bin/bash
# Round-2 first GPU pass: op microbenchmark, the -m gpu suite, smoke, bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 tools/ubbin/ubench_ops > gpurun_out/ubench_ops.txt 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 > gpurun_out/bench.json 2> gpurun_out/bench.err

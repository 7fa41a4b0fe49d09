#!/bin/bash
# Session re-entry check of the committed tree: the full -m gpu suite (incl. the
# world-1 RCCL exchange test), smoke, and the default bench line.
set -o pipefail
mkdir -p gpurun_out/r03u
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
    > gpurun_out/r03u/pytest_gpu.log 2>&1 && echo "tests ok" && \
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03u/smoke.log 2>&1 && echo "smoke ok" && \
timeout -k 10 600 python -u bench.py > gpurun_out/r03u/bench.json 2> gpurun_out/r03u/bench.err && echo "bench ok"

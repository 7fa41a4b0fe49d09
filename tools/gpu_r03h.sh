#!/bin/bash
# Whole -m gpu suite, smoke, bench line, solo-rank timings (bucket ranges).
set -o pipefail
mkdir -p gpurun_out/r03h
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread \
    > gpurun_out/r03h/pytest.log 2>&1 && \
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03h/smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/r03h/bench.json 2> gpurun_out/r03h/bench.err && \
SOLO="0/2 0/4 0/8 7/8" TAG=r03h bash tools/gpu_solo.sh

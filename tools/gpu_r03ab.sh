#!/bin/bash
# Round-3 end set on the final tree: the whole -m gpu suite, smoke, the default bench
# line, kernel trace + stats, PMC passes, solo times and kernel traces of ranks 0 / 7 of 8.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/r03ab
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
    > gpurun_out/r03ab/pytest_gpu.log 2>&1 && echo "tests ok" && \
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03ab/smoke.log 2>&1 && echo "smoke ok" && \
timeout -k 10 600 python -u bench.py > gpurun_out/r03ab/bench.json 2> gpurun_out/r03ab/bench.err && echo "bench ok" && \
bash tools/prof_trace.sh r03ab/trace 3 && echo "trace ok" && \
bash tools/pmc_run.sh r03ab/pmc && echo "pmc ok" && \
TAG=r03ab/solo SOLO="0/2 0/4 0/8 7/8" bash tools/gpu_solo.sh && echo "solo ok" && \
BENCH_ARGS="--solo 7/8" bash tools/prof_trace.sh r03ab/trace_solo7 3 && \
BENCH_ARGS="--solo 0/8" bash tools/prof_trace.sh r03ab/trace_solo0 3 && echo "solo traces ok"

#!/bin/bash
# Copy-constraint wire groups: the Merkle / prove tests first, then the whole
# -m gpu suite, smoke, the default bench line, and a PNP_WIRE_GROUPS=0 bench.
set -o pipefail
mkdir -p gpurun_out/r03v
timeout -k 10 600 python -u -m pytest tests/test_gpu_merkle.py tests/test_gpu_prove.py -m gpu -x -v --timeout 300 \
    --timeout-method thread > gpurun_out/r03v/pytest_first.log 2>&1 && echo "first tests ok" && \
timeout -k 10 480 python -u bench.py --cpu-lg 0 > gpurun_out/r03v/bench.json 2> gpurun_out/r03v/bench.err && echo "bench ok" && \
PNP_WIRE_GROUPS=0 timeout -k 10 480 python -u bench.py --cpu-lg 0 --drop-in "" > gpurun_out/r03v/bench_off.json 2> gpurun_out/r03v/bench_off.err && echo "bench off ok" && \
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
    > gpurun_out/r03v/pytest_gpu.log 2>&1 && echo "tests ok" && \
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03v/smoke.log 2>&1 && echo "smoke ok"

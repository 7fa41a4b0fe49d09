#!/bin/bash
# Copy-constraint wire groups, after the per-window-layout fix: the whole -m gpu
# suite, smoke, then a same-box interleaved A/B (groups on / PNP_WIRE_GROUPS=0).
set -o pipefail
mkdir -p gpurun_out/r03w
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
    > gpurun_out/r03w/pytest_gpu.log 2>&1 && echo "tests ok" && \
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03w/smoke.log 2>&1 && echo "smoke ok" && \
bash tools/abn.sh 3 base PNP_WIRE_GROUPS=0 > gpurun_out/r03w/ab.txt 2>&1 && echo "ab ok"

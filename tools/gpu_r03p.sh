#!/bin/bash
# GPU suite + smoke + bench line after the sort changes
set -o pipefail
mkdir -p gpurun_out/r03p
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread \
    > gpurun_out/r03p/pytest.log 2>&1 && echo "pytest ok" && \
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03p/smoke.log 2>&1 && echo "smoke ok" && \
timeout -k 10 600 python -u bench.py > gpurun_out/r03p/bench.json 2> gpurun_out/r03p/bench.err && echo "bench ok"

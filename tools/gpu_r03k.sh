#!/bin/bash
# Whole -m gpu suite and smoke with Lagrange-basis wire commitments.
set -o pipefail
mkdir -p gpurun_out/r03k
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread \
    > gpurun_out/r03k/pytest.log 2>&1 && echo "pytest ok" && \
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03k/smoke.log 2>&1 && echo "smoke ok"

#!/bin/bash
# Final tree: the whole -m gpu suite, smoke, the default bench line.
set -o pipefail
mkdir -p gpurun_out/r03af
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
    > gpurun_out/r03af/pytest_gpu.log 2>&1 && echo "tests ok" && \
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03af/smoke.log 2>&1 && echo "smoke ok" && \
timeout -k 10 600 python -u bench.py > gpurun_out/r03af/bench.json 2> gpurun_out/r03af/bench.err && echo "bench ok" && \
bash tools/abn.sh 3 base gpurun_variants/tilef16k/libpnp_plonk.so > gpurun_out/r03af/ab_tilef.txt 2>&1 && echo "ab tilef ok"

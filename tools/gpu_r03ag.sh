#!/bin/bash
# Final tree: the 8-rank full-size shared-GPU tests first, then the whole -m gpu
# suite, smoke and the default bench line.
set -o pipefail
mkdir -p gpurun_out/r03ag
timeout -k 10 900 python -u -m pytest tests/test_shard.py -m gpu -x -v -k "full_size" --timeout 400 --timeout-method thread \
    > gpurun_out/r03ag/pytest_shard.log 2>&1 && echo "shard ok" && \
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread --deselect \
    "tests/test_shard.py::test_sharded_full_size_matches_golden" > gpurun_out/r03ag/pytest_gpu.log 2>&1 && echo "tests ok" && \
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03ag/smoke.log 2>&1 && echo "smoke ok" && \
timeout -k 10 600 python -u bench.py > gpurun_out/r03ag/bench.json 2> gpurun_out/r03ag/bench.err && echo "bench ok"

#!/bin/bash
# Golden HEIGHT=15 Merkle proof on the GPU (single GPU, 2 and 8 gloo ranks),
# the small-range MSM tests (leaf fix), the bench line, solo 0/8.
set -o pipefail
mkdir -p gpurun_out/r03c
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
    "tests/test_shard.py::test_sharded_full_size_matches_golden" \
    > gpurun_out/r03c/pytest.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/r03c/bench.json 2> gpurun_out/r03c/bench.err && \
SOLO="0/8 7/8" TAG=r03c bash tools/gpu_solo.sh

#!/bin/bash
# Bucket-range MSM sharding: small multi-rank parity (both modes), then solo timings.
set -o pipefail
mkdir -p gpurun_out/r03e
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
    "tests/test_shard.py::test_sharded_gen_proof_parity" "tests/test_shard.py::test_sharded_merkle_circuit" \
    > gpurun_out/r03e/pytest.log 2>&1 && \
SOLO="0/2 0/4 0/8 7/8" TAG=r03e bash tools/gpu_solo.sh

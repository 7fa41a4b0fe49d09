#!/bin/bash
# Round-3 check: the new GPU tests (v1 key semantics, Merkle instance CPU/GPU
# generation, sharded Merkle vs the CPU restatement), then the bench line with
# its proof check, v1 drop-in both ways and the Merkle CPU baseline.
set -o pipefail
mkdir -p gpurun_out/r03a
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_prove.py tests/test_gpu_full.py::test_synthetic_merkle_gpu_equals_cpu_small \
    "tests/test_shard.py::test_sharded_merkle_circuit" tests/test_gpu_ops.py::test_commit_key_strided_ark_layout \
    tests/test_gpu_ops.py::test_proof_infinity_mask_of_gpu_proof > gpurun_out/r03a/pytest.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/r03a/bench.json 2> gpurun_out/r03a/bench.err

#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03g
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
    "tests/test_shard.py::test_sharded_gen_proof_parity" "tests/test_shard.py::test_sharded_merkle_circuit" \
    > gpurun_out/r03g/pytest.log 2>&1 && \
SOLO="0/8 7/8 0/4 0/2" TAG=r03g bash tools/gpu_solo.sh && \
for rw in 0/8 0/4 0/2; do PNP_MSM_SHARD=points timeout -k 10 300 python -u bench.py --steps 5 --solo $rw > gpurun_out/r03g/points_${rw/\//of}.json 2> gpurun_out/r03g/points.err || exit 1; done

#!/bin/bash
# The -m gpu suite on the box (one process), log under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread ${1:+-k "$1"} > gpurun_out/pytest_gpu.log 2>&1

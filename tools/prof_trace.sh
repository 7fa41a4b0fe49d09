#!/bin/bash
# Kernel trace + stats of a short bench run (one warmup + K timed proofs):
#   bash tools/prof_trace.sh <tag> [steps]
set -o pipefail
R=$(pwd)
TAG=${1:-trace}
STEPS=${2:-2}
mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/$TAG -o run -- \
    python3 $R/bench.py --steps $STEPS --warmup 1 --cpu-lg 0 --drop-in "" --no-verify $BENCH_ARGS > $R/gpurun_out/$TAG/bench.log 2>&1

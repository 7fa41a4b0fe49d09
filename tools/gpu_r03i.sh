#!/bin/bash
# Round-3 end profiles: kernel trace + stats of the default bench (3 proofs),
# then FETCH_SIZE / WRITE_SIZE / SQ passes (separate --pmc runs).
set -o pipefail
mkdir -p gpurun_out/r03i
bash tools/prof_trace.sh r03i/trace 3 && echo "trace ok" && \
bash tools/pmc_run.sh r03i/pmc && echo "pmc ok"

#!/bin/bash
# Round-3 end profiles (after the Lagrange-basis commitments): kernel trace + stats of the default bench (3 proofs),
# then FETCH_SIZE / WRITE_SIZE / SQ passes (separate --pmc runs).
set -o pipefail
mkdir -p gpurun_out/r03s
bash tools/prof_trace.sh r03s/trace 3 && echo "trace ok" && \
bash tools/pmc_run.sh r03s/pmc && echo "pmc ok"

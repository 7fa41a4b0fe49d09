#!/bin/bash
# Round-end measurement set: smoke, the default bench line, a rocprofv3 kernel
# trace of a short bench (timeline / stats for profiles/).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err && \
bash tools/prof_trace.sh ${TAG:-r02_final} 3

#!/bin/bash
# PMC passes over one bench proof (one counter group per run, no tracing
# domains): FETCH_SIZE, WRITE_SIZE, SQ issue/wait breakdown.  Run on the GPU
# box from the repo root:  bash tools/pmc_run.sh <tag>
set -e -o pipefail
R=$(pwd)
TAG=${1:-pmc}
RX='k_accumulate29|k_ntt_pass|k_quotient|k_coarse_scatter|k_fine_sort|k_tree_level|k_t_combine'
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/$TAG
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-include-regex "$RX" -f csv \
      -d $R/gpurun_out/$TAG/p$i -o run -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-lg 0 --drop-in "" \
      > $R/gpurun_out/$TAG/p$i.log 2>&1
done

#!/bin/bash
# One PMC pass (no tracing domains) over one bench proof: GRBM_GUI_ACTIVE
# (summed over the 8 XCDs) and SQ_BUSY_CYCLES per kernel, for the clock the
# chip holds in each kernel (tools/pmc_clock.py):  bash tools/pmc_clock.sh <tag>
set -o pipefail
R=$(pwd)
TAG=${1:-pmc_clock}
RX='k_accumulate29|k_ntt_pass|k_quotient|k_tree_leafw29|k_merge_tails29|k_fine_sort|k_coarse_scatter'
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/$TAG
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU --kernel-include-regex "$RX" -f csv \
    -d $R/gpurun_out/$TAG/p1 -o run -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-lg 0 --drop-in "" \
    > $R/gpurun_out/$TAG/p1.log 2>&1 || { echo "pmc pass failed rc=$?"; exit 1; }
echo "pmc pass ok"

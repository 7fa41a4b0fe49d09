#!/bin/bash
# PMC passes (one counter group per run, no tracing domains) over one bench
# proof, for the accumulate / NTT / quotient kernels:  bash tools/pmc_r02.sh <tag>
set -o pipefail
R=$(pwd)
TAG=${1:-pmc}
RX='k_accumulate29|k_ntt_pass|k_quotient|k_tree_leafw29|k_merge_tails29'
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/$TAG
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
         "SQ_IFETCH SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM" \
         "SQC_ICACHE_MISSES SQC_ICACHE_HITS"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P --kernel-include-regex "$RX" -f csv \
      -d $R/gpurun_out/$TAG/p$i -o run -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-lg 0 --drop-in "" \
      > $R/gpurun_out/$TAG/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
  echo "pass $i ok"
done

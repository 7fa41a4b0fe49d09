#!/bin/bash
# tools/msm_c_sweep.py with one fresh process per (lg, c)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/msm_c_sweep.jsonl
for LG in ${LGS:-19 20 21}; do
  for C in ${CS:-16 17 18 19 20}; do
    SWEEP_C=$C timeout -k 10 120 python -u tools/msm_c_sweep.py $LG >> gpurun_out/msm_c_sweep.jsonl 2>> gpurun_out/msm_c_sweep.err || exit 1
  done
done

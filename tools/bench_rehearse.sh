#!/bin/bash
# Multi-rank bench rehearsal on a 1-GPU box: N ranks share the GPU, gloo
# exchanges (PNP_BENCH_BACKEND=gloo); exercises bench.py's distributed path
# (shard setup, barriers, max-over-ranks timing, rank-0 JSON) except RCCL.
#   bash tools/bench_rehearse.sh <ranks> <lg>      (REHEARSE_ARGS: more bench.py
#   arguments, e.g. "--op msm" for BASELINE config 3's sharded MSM line)
set -o pipefail
mkdir -p gpurun_out
N=${1:-2}; LG=${2:-18}
PNP_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus $N --lg $LG --steps 2 --warmup 1 ${REHEARSE_ARGS:-} \
  > gpurun_out/rehearse_n$N.json 2> gpurun_out/rehearse_n$N.err

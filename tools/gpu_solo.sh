#!/bin/bash
# Per-rank critical path of the multi-GPU proof, measured alone on one GPU
# (bench.py --solo R/W: rank R's MSM point ranges, round-4 blocks and
# coefficient range; loopback exchanges).  Writes gpurun_out/${TAG}/solo_*.json.
set -o pipefail
TAG=${TAG:-r03_solo}
mkdir -p gpurun_out/$TAG
for rw in ${SOLO:-0/1 0/2 0/4 0/8 7/8}; do
  f=gpurun_out/$TAG/solo_${rw/\//of}.json
  if [ "$rw" = "0/1" ]; then
    timeout -k 10 300 python -u bench.py --steps 5 --no-verify --drop-in "" --cpu-lg 0 > $f 2> $f.err || exit $?
  else
    timeout -k 10 300 python -u bench.py --steps 5 --solo $rw > $f 2> $f.err || exit $?
  fi
done

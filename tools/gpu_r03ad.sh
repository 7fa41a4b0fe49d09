#!/bin/bash
# Solo probes: which ranks of 8 have the slow round-1 accumulation, and with point ranges.
set -o pipefail
mkdir -p gpurun_out/r03ad
for rw in 1/8 3/8 5/8 6/8; do
  timeout -k 10 300 python -u bench.py --steps 4 --solo $rw > gpurun_out/r03ad/solo_${rw/\//of}.json 2>/dev/null || exit 1
  echo "solo $rw: $(python3 -c "import json;d=json.loads(open('gpurun_out/r03ad/solo_${rw/\//of}.json').read().strip().splitlines()[-1]);print(d['value'],d['stages_ms']['r1_commit'])")"
done
for rw in 0/8 7/8; do
  PNP_MSM_SHARD=points timeout -k 10 300 python -u bench.py --steps 4 --solo $rw > gpurun_out/r03ad/pts_${rw/\//of}.json 2>/dev/null || exit 1
  echo "points solo $rw: $(python3 -c "import json;d=json.loads(open('gpurun_out/r03ad/pts_${rw/\//of}.json').read().strip().splitlines()[-1]);print(d['value'],d['stages_ms']['r1_commit'])")"
done

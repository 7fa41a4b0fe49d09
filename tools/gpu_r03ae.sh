#!/bin/bash
# Solo probes at 2 and 4 ranks (rank 1 of 2 takes point ranges) with and without wire groups.
set -o pipefail
mkdir -p gpurun_out/r03ae
for V in "PNP_AB=0" "PNP_WIRE_GROUPS=0"; do
  for rw in 1/2 1/4 3/4; do
    f=gpurun_out/r03ae/${V%%=*}_${rw/\//of}.json
    env $V timeout -k 10 300 python -u bench.py --steps 4 --solo $rw > $f 2>/dev/null || exit 1
    echo "$V solo $rw: $(python3 -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print(d['value'],d['stages_ms']['r1_commit'],d['stages_ms']['r3_z2_pi'])")"
  done
done

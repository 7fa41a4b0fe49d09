#!/bin/bash
# stage-boundary syncs on/off: 1-GPU A/B and solo 8-rank A/B
set -o pipefail
mkdir -p gpurun_out/r03r
bash tools/abn.sh 4 base PNP_STAGE_SYNC=0 > gpurun_out/r03r/ab1.txt 2>&1 && echo "ab1 ok" && \
for r in 1 2 3; do
  for V in 1 0; do
    PNP_STAGE_SYNC=$V timeout -k 10 300 python -u bench.py --steps 5 --solo 0/8 > gpurun_out/r03r/solo8_s${V}_r$r.json 2>/dev/null || exit 1
    echo "solo8 sync=$V round $r: $(python3 -c "import json;print(json.loads(open('gpurun_out/r03r/solo8_s${V}_r$r.json').read().strip().splitlines()[-1])['value'])")"
  done
done

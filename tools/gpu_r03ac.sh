#!/bin/bash
# Key-load buffer reuse (v1 drop-in cost) + probes of the solo rank-7 round-1 accumulation.
set -o pipefail
mkdir -p gpurun_out/r03ac
timeout -k 10 600 python -u -m pytest tests/test_gpu_prove.py tests/test_gpu_merkle.py tests/test_gpu_general.py -m gpu -x -v \
    --timeout 300 --timeout-method thread > gpurun_out/r03ac/pytest.log 2>&1 && echo "tests ok" && \
timeout -k 10 600 python -u bench.py --cpu-lg 0 > gpurun_out/r03ac/bench.json 2> gpurun_out/r03ac/bench.err && echo "bench ok" && \
for V in "PNP_AB=0" "PNP_NO_OVERLAP=1" "PNP_WIRE_GROUPS=0"; do
  env $V timeout -k 10 300 python -u bench.py --steps 5 --solo 7/8 > gpurun_out/r03ac/solo7_${V%%=*}.json 2> gpurun_out/r03ac/solo7_${V%%=*}.err || exit 1
  echo "solo7 $V: $(python3 -c "import json;d=json.loads(open('gpurun_out/r03ac/solo7_${V%%=*}.json').read().strip().splitlines()[-1]);print(d['value'],d['stages_ms']['r1_commit'])")"
done

#!/bin/bash
# fused digits + histogram, sort tile-size variants: MSM parity tests, kernel
# traces (2 proofs each) and an interleaved A/B
set -o pipefail
R=$PWD
mkdir -p gpurun_out/r03n
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_lagrange.py tests/test_gpu_full.py -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r03n/pytest.log 2>&1 && echo "pytest ok" || exit 1
for V in tk8 tk16 tf16; do
  PNP_PLONK_LIB=$R/ab_libs/lib_$V.so bash tools/prof_trace.sh r03n/$V 2 || exit 1
  echo "trace $V ok"
done
PNP_MSM_FUSE_DIGITS=0 bash tools/prof_trace.sh r03n/nofuse 2 && echo "trace nofuse ok" && \
bash tools/prof_trace.sh r03n/base 2 && echo "trace base ok" && \
bash tools/abn.sh 2 base PNP_MSM_FUSE_DIGITS=0 $R/ab_libs/lib_tk8.so $R/ab_libs/lib_tk16.so $R/ab_libs/lib_tf16.so > gpurun_out/r03n/ab.txt 2>&1 && echo "ab ok"

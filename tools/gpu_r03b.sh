#!/bin/bash
# Karatsuba A/B (ubench + whole proof, interleaved) and the solo-rank runs.
set -o pipefail
mkdir -p gpurun_out/r03b
timeout -k 10 120 tools/ubbin/ubench_kara 48 > gpurun_out/r03b/ubench_kara.txt 2>&1 && \
timeout -k 10 600 bash tools/abn.sh 3 base lib_var/kara/libpnp_plonk.so > gpurun_out/r03b/ab_kara.txt 2>&1 && \
TAG=r03b bash tools/gpu_solo.sh

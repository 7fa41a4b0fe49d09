set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
for C in 16 18 19 20; do
  PNP_FOLD_C=$C timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-lg 0 > gpurun_out/bench_c$C.json 2> gpurun_out/bench_c$C.err || exit 1
done

# A/B of two library builds on one box: bash tools/ab.sh <libA> <libB> [rounds]
set -o pipefail
mkdir -p gpurun_out/ab
for r in $(seq 1 ${3:-2}); do
  for v in A B; do
    L=$1; [ $v = B ] && L=$2
    PNP_PLONK_LIB=$L timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-lg 0 > gpurun_out/ab/$v$r.json 2> gpurun_out/ab/$v$r.err || exit 1
  done
done

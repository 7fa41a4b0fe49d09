# A/B of one build under two environments on one box:
#   bash tools/ab_env.sh "<envA>" "<envB>" [rounds]     e.g. "" "PNP_MSM_NOPIPE=1"
set -o pipefail
mkdir -p gpurun_out/ab
for r in $(seq 1 ${3:-2}); do
  for v in A B; do
    E=$1; [ $v = B ] && E=$2
    env $E timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-lg 0 > gpurun_out/ab/$v$r.json 2> gpurun_out/ab/$v$r.err || exit 1
  done
done

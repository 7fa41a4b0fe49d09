set -o pipefail
for C in 18 20; do
  PNP_FOLD_C=$C bash tools/prof_trace.sh trace_c$C 1 || exit 1
done

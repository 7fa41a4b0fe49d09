# A/B/n on one box, interleaved rounds:
#   bash tools/abn.sh <rounds> <variant> ...
# variant: "base" (the in-tree build), a library path (PNP_PLONK_LIB), or
# VAR=value (an environment setting for the in-tree build), several of them
# joined by '@' (e.g. PNP_MSM_PIPE=1@PNP_PLONK_LIB=lib_var/x/libpnp_plonk.so); ABN_ARGS: extra
# bench.py arguments for every run (e.g. "--solo 0/8")
set -o pipefail
mkdir -p gpurun_out/ab
R=$1; shift
for r in $(seq 1 $R); do
  i=0
  for V in "$@"; do
    i=$((i+1))
    case "$V" in
      base) E="PNP_AB=0" ;;
      *=*) E="${V//@/ }" ;;
      *) E="PNP_PLONK_LIB=$V" ;;
    esac
    env $E timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --cpu-lg 0 --drop-in "" $ABN_ARGS > gpurun_out/ab/v$i.r$r.json 2> gpurun_out/ab/v$i.r$r.err || exit 1
    echo "round $r $V: $(python3 -c "import json;print(json.load(open('gpurun_out/ab/v$i.r$r.json'))['value'])")"
  done
done

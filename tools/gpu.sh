#!/bin/bash
# The one GPU-box runner (replaces the per-call gpu_r0*.sh scripts).
#
#   bash tools/gpu.sh <tag> <step> [<step> ...]
#
# Every step runs under its own time limit, writes under gpurun_out/<tag>/,
# and the steps are chained: the first failing step ends the call (no step
# runs on the GPU after a fault, an abort or a time limit).  Steps:
#
#   tests[=K]        pytest -m gpu (optionally -k K, '+' for spaces), one process
#   smoke            __graft_entry__.smoke()
#   bench[=ARGS]     bench.py (default arguments unless ARGS, '+'-separated),
#                    JSON line in bench.json, log in bench.err
#   stats[=STEPS]    rocprofv3 --kernel-trace --stats over a short bench
#   trace=ARGS       the same over bench.py ARGS ('+'-separated, e.g. --solo+7/8+--steps+2)
#   pmc[=COUNTERS]   one rocprofv3 --pmc pass over one bench proof (counters
#                    '+'-separated; default the SQ issue / VALU group);
#                    PMC_BENCH_ARGS: other bench.py arguments (e.g. --op ntt --lg 20)
#   traffic          FETCH_SIZE and WRITE_SIZE passes (two runs)
#   solo[=R/W,...]   bench.py --solo for each R/W (default 0/2,0/4,0/8,7/8)
#   ab=N:V1,V2,...   tools/abn.sh N rounds over the variants
#   rehearse=N:LG    bench.py --gpus N at 2^LG, N gloo ranks sharing the GPU
#   py=SCRIPT[+ARGS] python SCRIPT ARGS (a tool or test driver), 300 s limit
set -o pipefail
R=$(pwd)
TAG=${1:?tag}; shift
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
RX='k_accumulate29|k_ntt_pass|k_bitrev|k_quotient|k_coarse_scatter|k_fine_sort|k_tree_level|k_t_combine|k_merge_tails29|k_tree_leafw29|k_digits_hist|k_count_pieces'
BENCH1="--steps 1 --warmup 0 --cpu-lg 0 --drop-in '' --no-verify"

run_step() {
  local step=$1 arg=${1#*=}
  [ "$arg" = "$step" ] && arg=""
  case "$step" in
    tests*)
      timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v -rs --timeout ${TEST_TIMEOUT:-400} --timeout-method thread \
          ${arg:+-k "${arg//+/ }"} > "$OUT/pytest_gpu.log" 2>&1 ;;
    smoke)
      timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ;;
    bench*)
      # bench.json for the default arguments, bench_<args>.json otherwise
      local bn=bench${arg:+_$(echo "$arg" | tr -c 'A-Za-z0-9' '_' | cut -c1-40)}
      timeout -k 10 900 python -u bench.py ${arg//+/ } > "$OUT/$bn.json" 2> "$OUT/$bn.err" ;;
    stats*)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/stats" -o run -- \
          python3 "$R/bench.py" --steps ${arg:-3} --warmup 1 --cpu-lg 0 --drop-in "" --no-verify > "$OUT/stats.log" 2>&1) ;;
    trace=*)
      # kernel trace of a bench run with these arguments ('+'-separated)
      local d=$OUT/trace_$(echo "$arg" | tr -c 'A-Za-z0-9' '_' | cut -c1-40)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$d" -o run -- \
          python3 "$R/bench.py" --cpu-lg 0 --drop-in "" --no-verify ${arg//+/ } > "$d.log" 2>&1) ;;
    pmc*)
      local c=${arg:-SQ_WAVES+SQ_INSTS_VALU+SQ_WAVE_CYCLES+SQ_WAIT_ANY+SQ_WAIT_INST_ANY+SQ_ACTIVE_INST_ANY+SQ_ACTIVE_INST_VALU+SQ_INSTS_SALU}
      local d=$OUT/pmc_$(echo "$c" | tr '+' '_' | cut -c1-40)
      # the one profiled proof is the process's first: without PNP_DEFER_TABLES=0
      # it defers the Lagrange / copy-group tables and commits the wires and z
      # densely — not the steady-state proof the bench times
      (cd /tmp && export TMPDIR=/tmp && export PNP_DEFER_TABLES=${PNP_DEFER_TABLES:-0} && timeout -s KILL 200 rocprofv3 --pmc ${c//+/ } --kernel-include-regex "$RX" -f csv \
          -d "$d" -o run -- python3 "$R/bench.py" --steps 1 --warmup 0 --cpu-lg 0 --drop-in "" --no-verify \
          ${PMC_BENCH_ARGS:-} > "$d.log" 2>&1) ;;
    traffic)
      run_step pmc=FETCH_SIZE && run_step pmc=WRITE_SIZE ;;
    solo*)
      for rw in $(echo "${arg:-0/2,0/4,0/8,7/8}" | tr ',' ' '); do
        timeout -k 10 300 python -u bench.py --steps 5 --solo "$rw" > "$OUT/solo_${rw/\//of}.json" \
            2> "$OUT/solo_${rw/\//of}.err" || return $?
      done ;;
    ab=*)
      local n=${arg%%:*} v=${arg#*:}
      bash tools/abn.sh "$n" $(echo "$v" | tr ',' ' ') > "$OUT/ab.txt" 2>&1 ;;
    rehearse=*)
      # bench.py's multi-rank path with N gloo ranks sharing the GPU (N:LG)
      local rn=${arg%%:*} rl=${arg#*:}
      bash tools/bench_rehearse.sh "$rn" "$rl" && cp gpurun_out/rehearse_n$rn.json gpurun_out/rehearse_n$rn.err "$OUT/" ;;
    py=*)
      timeout -k 10 300 python -u ${arg//+/ } > "$OUT/py_$(basename "${arg%%+*}").log" 2>&1 ;;
    *)
      echo "gpu.sh: unknown step $step"; return 2 ;;
  esac
}

for s in "$@"; do
  t0=$(date +%s)
  if run_step "$s"; then
    echo "[$TAG] $s ok ($(( $(date +%s) - t0 )) s)"
  else
    rc=$?
    echo "[$TAG] $s FAILED rc=$rc ($(( $(date +%s) - t0 )) s)"
    exit $rc
  fi
done

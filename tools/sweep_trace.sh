set -o pipefail
R=$(pwd)
mkdir -p $R/gpurun_out/sweep_trace
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/sweep_trace -o run -- python3 $R/tools/msm_c_sweep.py ${SWEEP_LG:-22} > $R/gpurun_out/sweep_trace/log.txt 2>&1

# usage (GPU box): bash tools/driver_trace.sh <tag> <config> [<config> ...]
# The driver's bench command (--gpus 1 --steps 20 --warmup 5) under a rocprofv3 kernel trace, per
# config, then tools/step_account.py: where the step's time goes above the dominant kernel, and
# tools/launch_series.py: the dominant kernel's per-launch durations (the clock transient).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; shift
O=$ROOT/gpurun_out/prof_$tag; mkdir -p $O
export TMPDIR=/tmp
for cfg in "$@"; do
  case $cfg in c2) dom=k_linear_fused ;; c3) dom=k_mnl_duo ;; c4) dom=k_linear_cluster ;; c5) dom=k_spec_slice ;; *) dom=k_linear_fused ;; esac
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/drv_$cfg -o drv -- \
      python $ROOT/bench.py --gpus 1 --config $cfg --steps 20 --warmup 5 --no-cpu-baseline \
      > $O/drv_${cfg}.json 2> $O/drv_${cfg}.err) || exit 1
  python $ROOT/tools/step_account.py --trace "$O/drv_$cfg/**/*kernel_trace.csv" --bench $O/drv_${cfg}.json \
      --dominant $dom > $O/drv_${cfg}_account.json || exit 1
  python $ROOT/tools/launch_series.py $(ls $O/drv_$cfg/*kernel_trace.csv $O/drv_$cfg/*/*kernel_trace.csv 2>/dev/null | head -1) $dom
done
echo done

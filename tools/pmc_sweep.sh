# usage (GPU box): bash tools/pmc_sweep.sh <tag> <config> "<counters pass 1>" "<counters pass 2>" ...
# One rocprofv3 --pmc pass per counter set (each within the per-block limits), bench.py as the
# program, csv under gpurun_out/pmc_<tag>/p<k>/.  Stops at the first failure.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; cfg=$2; shift 2
OUT=$ROOT/gpurun_out/pmc_$tag
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp || exit 1
k=0
for set in "$@"; do
  k=$((k + 1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/p$k -o run -- \
      python $ROOT/bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --allow-other-path \
      > /dev/null 2> $OUT/p$k.err || exit 1
done
echo done

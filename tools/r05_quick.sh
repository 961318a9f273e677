# usage (GPU box): bash tools/r05_quick.sh <tag> <pytest -k expression> [config ...]
# A selection of GPU tests, then per config a bench line and a kernel-trace --stats run.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; sel=$2; shift 2
OUT=$ROOT/gpurun_out/$tag
mkdir -p $OUT
cd $ROOT || exit 1
if [ -n "$sel" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "$sel" \
      > $OUT/gputests.log 2>&1 || exit 1
fi
export TMPDIR=/tmp
for c in "$@"; do
  timeout -k 10 300 python bench.py --config $c --steps 30 --warmup 200 --no-cpu-baseline \
      > $OUT/${c}_bench.json 2> $OUT/${c}_bench.err || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o $c -- \
      python $ROOT/bench.py --config $c --steps 30 --warmup 200 --no-cpu-baseline \
      > $OUT/${c}_bench_under_rocprof.json 2> $OUT/${c}_trace.err || exit 1
done
echo done

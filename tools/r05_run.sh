# usage (GPU box): bash tools/r05_run.sh <tag> [pytest selection...]
# The round-5 check: MFMA rounding probe, the GPU suite (or a selection), and bench lines.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; shift
OUT=$ROOT/gpurun_out/$tag
mkdir -p $OUT
cd $ROOT || exit 1
if [ -x tools/_mfma_bf16_round ]; then
  timeout -k 10 60 ./tools/_mfma_bf16_round > $OUT/mfma_bf16_round.txt 2>&1 || exit 1
fi
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -x -v -s --timeout 300 --timeout-method thread \
    > $OUT/gputests.log 2>&1 || exit 1
for c in c2 c3 c5; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 > $OUT/${c}_w5.json 2> $OUT/${c}_w5.err || exit 1
done
timeout -k 10 600 python bench.py --config c4 --scaling strong --steps 20 --warmup 5 \
    > $OUT/c4strong_w5.json 2> $OUT/c4strong_w5.err || exit 1
echo done

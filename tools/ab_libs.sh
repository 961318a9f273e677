# usage (GPU box): bash tools/ab_libs.sh <tag> <config> <warmup> <lib|default> ...
# bench lines of one config with each library (TR_HIP_LIB), two rounds interleaved
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; cfg=$2; wu=$3; shift 3
OUT=$ROOT/gpurun_out/$tag
mkdir -p $OUT
cd $ROOT || exit 1
for rnd in ${AB_ROUNDS:-1 2}; do
  for lib in "$@"; do
    nm=$(basename $lib .so)
    if [ "$lib" = default ]; then
      timeout -k 10 300 python bench.py --config $cfg --steps 30 --warmup $wu --no-cpu-baseline --allow-other-path \
          > $OUT/${cfg}_${nm}_$rnd.json 2> $OUT/${cfg}_${nm}_$rnd.err || exit 1
    else
      TR_HIP_LIB=$ROOT/$lib timeout -k 10 300 python bench.py --config $cfg --steps 30 --warmup $wu --no-cpu-baseline \
          --allow-other-path > $OUT/${cfg}_${nm}_$rnd.json 2> $OUT/${cfg}_${nm}_$rnd.err || exit 1
    fi
    python -c "import json;d=json.load(open('$OUT/${cfg}_${nm}_$rnd.json'));print('$nm',$rnd,round(d['roofline']['kernel_avg_ms'],4),round(d['ms_per_step'],4))"
  done
done

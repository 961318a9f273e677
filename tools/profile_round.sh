# usage (GPU box): bash tools/profile_round.sh <tag> <config> [<config> ...]
# Per config: one plain bench line, one rocprofv3 --kernel-trace --stats run, and two PMC passes
# (FETCH_SIZE, WRITE_SIZE separately, MI355X_MICROARCH.md HBM section), then tools/pmc_traffic.py
# folds the counters into profiles/traffic.json. Every GPU step has its own time limit and the
# script stops at the first failure.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; shift
OUT=$ROOT/gpurun_out/prof_$tag
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp || exit 1
for cfg in "$@"; do
  case $cfg in
    c2) alg=8590196736; dom=k_linear_fused ;;
    c3) alg=2148007936; dom=k_mnl_duo ;;
    c4) alg=8590000128; dom=k_linear_cluster ;;
    c5) alg=4328783872; dom=k_spec_slice ;;
    c6) alg=8590196736; dom=k_linear_fused ;;  # windowed: window bytes (overlapping rows hit L2 / MALL)
    c7) alg=1073774592; dom=k_linear_fused ;;  # HostStream: one launch per 8192-sample chunk
    *) alg=""; dom=k_linear_fused ;;
  esac
  echo "[$cfg] bench" >&2
  timeout -k 10 300 python $ROOT/bench.py --config $cfg --steps 30 --warmup 200 \
      > $OUT/${cfg}_bench.json 2> $OUT/${cfg}_bench.err || exit 1
  echo "[$cfg] kernel trace" >&2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o $cfg -- \
      python $ROOT/bench.py --config $cfg --steps 30 --warmup 200 --no-cpu-baseline \
      > $OUT/${cfg}_bench_under_rocprof.json 2> $OUT/${cfg}_trace.err || exit 1
  echo "[$cfg] pmc FETCH_SIZE" >&2
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o $cfg -- \
      python $ROOT/bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline \
      > /dev/null 2> $OUT/${cfg}_fetch.err || exit 1
  echo "[$cfg] pmc WRITE_SIZE" >&2
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o $cfg -- \
      python $ROOT/bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline \
      > /dev/null 2> $OUT/${cfg}_write.err || exit 1
  if [ "$cfg" = c3 ] || [ "$cfg" = c5 ]; then
    echo "[$cfg] pmc MFMA busy" >&2
    timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
        -d $OUT/mfma -o $cfg -- python $ROOT/bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline \
        > /dev/null 2> $OUT/${cfg}_mfma.err || exit 1
    # algorithmic flops per launch: c3 factored pass 4*P*R per sample; c5 4*W*D*(n_out + Rs*Cc) per sample
    case $cfg in c3) fl=17179869184; kre="k_mnl_duo" ;; c5) fl=77913391104; kre="k_spec_slice" ;; esac
    python $ROOT/tools/pmc_mfma.py --config $cfg --csv $(ls $OUT/mfma/${cfg}*counter_collection.csv | tail -1) \
        --kernel "$kre" --flops $fl --out $OUT/${cfg}_mfma.json || exit 1
  fi
  python $ROOT/tools/pmc_traffic.py --config $cfg --fetch $(ls $OUT/fetch/${cfg}*counter_collection.csv | tail -1) \
      --write $(ls $OUT/write/${cfg}*counter_collection.csv | tail -1) ${alg:+--algorithmic $alg} --dominant $dom \
      --out $OUT/traffic.json > /dev/null || exit 1
done
echo done >&2

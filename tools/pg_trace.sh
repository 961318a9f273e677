# Kernel trace of bench.py through the sharded code path at world size 1 (RCCL all-reduce of the
# gradient arena every step, TR_BENCH_FORCE_PG=1), to see what the collective adds per step.
#   gpurun -- 'bash tools/pg_trace.sh c2 c3'  ->  gpurun_out/pgtrace/{<cfg>.json, kt_<cfg>/}
set -o pipefail
mkdir -p gpurun_out/pgtrace
export TR_BENCH_FORCE_PG=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29531 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in "$@"; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 50 --warmup 100 > gpurun_out/pgtrace/$c.json 2> gpurun_out/pgtrace/$c.err || exit 1
  timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/pgtrace/kt_$c -o k -- python3 bench.py --config $c --no-cpu-baseline --steps 30 --warmup 20 > /dev/null 2>&1 || exit 1
done
echo done

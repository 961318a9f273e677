# A/B of the per-iteration tail on one GPU, bench.py with the live kernel timing sampled (every
# 10th launch, the default), on every launch, and off; plus a kernel trace of the default run.
# OLD_LIB=<path to a build of other sources> adds a run of that library (its ABI must match).
#   gpurun -- 'bash tools/ab_run.sh'   ->  gpurun_out/ab/{new,every1,newnt[,old]}_<config>.json, kt_new_<config>/
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/gpu_tests.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in ${CONFIGS:-c2 c3 c5}; do
  B="timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 50 --warmup 100"
  $B > gpurun_out/ab/new_$c.json 2>/dev/null || exit 1
  $B --timing-every 1 > gpurun_out/ab/every1_$c.json 2>/dev/null || exit 1
  $B --no-kernel-timing > gpurun_out/ab/newnt_$c.json 2>/dev/null || exit 1
  if [ -n "$OLD_LIB" ]; then TR_HIP_LIB=$OLD_LIB $B > gpurun_out/ab/old_$c.json 2>/dev/null || exit 1; fi
  timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/ab/kt_new_$c -o k -- python3 bench.py --config $c --no-cpu-baseline --steps 30 --warmup 20 > /dev/null 2>&1 || exit 1
done
echo done

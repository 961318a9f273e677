set -o pipefail
mkdir -p gpurun_out/gaps
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in c3 c2 c5; do
  timeout -k 10 120 python bench.py --config $c --no-cpu-baseline > gpurun_out/gaps/$c.ev.json 2> gpurun_out/gaps/$c.ev.err || exit 1
  timeout -k 10 120 python bench.py --config $c --no-cpu-baseline --no-kernel-timing > gpurun_out/gaps/$c.noev.json 2> gpurun_out/gaps/$c.noev.err || exit 1
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gaps/kt_$c -- python3 bench.py --config $c --no-cpu-baseline --no-kernel-timing --steps 30 > gpurun_out/gaps/$c.kt.json 2> gpurun_out/gaps/$c.kt.err || exit 1
  python tools/kernel_gaps.py "gpurun_out/gaps/kt_$c/**/*kernel_trace.csv" > gpurun_out/gaps/$c.gaps.txt 2>&1
done
echo ok

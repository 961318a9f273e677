# bench ms/step vs untimed warm-up length (same box, back to back)
set -o pipefail
mkdir -p gpurun_out/wu
for c in c3 c2; do
  for w in 5 50 200 5; do
    timeout -k 10 120 python bench.py --config $c --no-cpu-baseline --warmup $w > gpurun_out/wu/$c.w$w.json 2> gpurun_out/wu/$c.w$w.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/wu/$c.w$w.json')); print('$c', $w, round(d['ms_per_step'],4), round(d['roofline']['kernel_avg_ms'],4))"
  done
done
timeout -k 10 150 python tools/fit_overhead.py --config c3 || exit 1

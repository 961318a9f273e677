# usage: bash tools/variants.sh <config> <name>=<ENV assignments;...> ...   (GPU box)
set -o pipefail
mkdir -p gpurun_out
cfg=$1; shift
for spec in "$@"; do
  name=${spec%%=*}; envs=${spec#*=}
  env ${envs//;/ } timeout -k 10 300 python bench.py --config $cfg --steps 30 --warmup 5 --no-cpu-baseline $EXTRA > gpurun_out/v_${cfg}_$name.json 2> gpurun_out/v_${cfg}_$name.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/v_${cfg}_$name.json')); r=d['roofline']; print('$cfg', '$name', round(d['value']/1e6,2), 'Msps', round(d['ms_per_step'],4), 'ms', r['kernel'], round(r['kernel_avg_ms'],4), round(r['achieved']), 'GB/s', {k:(round(v,4) if v else None) for k,v in d['kernel_avg_ms'].items()})"
done

# usage (here, after gpurun merged gpurun_out/prof_<tag>/): bash tools/collect_profiles.sh <tag> <round> <config>...
# Copies one profile_round.sh run into profiles/<round>_<cfg>_*: the bench lines, the rocprofv3
# kernel stats, the PMC csvs trimmed to this library's tr:: kernels, and merges traffic.json.
set -e
tag=$1; round=$2; shift 2
src=gpurun_out/prof_$tag
for c in "$@"; do
  cp $src/${c}_bench.json profiles/${round}_${c}_bench.json
  cp $src/${c}_bench_under_rocprof.json profiles/${round}_${c}_bench_under_rocprof.json
  cp $src/trace/${c}_kernel_stats.csv profiles/${round}_${c}_kernel_stats.csv
  if [ -f $src/${c}_mfma.json ]; then
    cp $src/${c}_mfma.json profiles/${round}_${c}_mfma.json
    f=$(ls $src/mfma/${c}*counter_collection.csv | tail -1)
    { head -1 $f; grep 'tr::' $f || true; } > profiles/${round}_${c}_pmc_mfma.csv
  fi
  for p in fetch write; do
    f=$(ls $src/$p/${c}*counter_collection.csv | tail -1)
    { head -1 $f; grep 'tr::' $f || true; } > profiles/${round}_${c}_pmc_${p}.csv
  done
done
python - "$src/traffic.json" "$round" <<'PY'
import json, sys
new = json.load(open(sys.argv[1]))
old = json.load(open("profiles/traffic.json"))
old.update(new)
old["round"] = f"profile set {sys.argv[2]}"
json.dump(old, open("profiles/traffic.json", "w"), indent=1)
PY

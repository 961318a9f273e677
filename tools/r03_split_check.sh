# GPU box: spectral tests on the split kernel, c5 bench split vs f32, then the whole GPU suite
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_spectral.py -x -q --timeout 120 --timeout-method thread > gpurun_out/spec_split.log 2>&1 || { echo "spectral tests failed"; tail -30 gpurun_out/spec_split.log; exit 1; }
timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline > gpurun_out/bench_c5_split.json 2> gpurun_out/bench_c5_split.err || exit 1
TR_SLICE_SPLIT=0 timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline > gpurun_out/bench_c5_f32.json 2> gpurun_out/bench_c5_f32.err || exit 1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { tail -30 gpurun_out/gputest.log; exit 1; }
tail -3 gpurun_out/gputest.log
timeout -k 10 200 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || exit 1
timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit 1
echo done

set -o pipefail
mkdir -p gpurun_out/r3base
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3base/tests.log 2>&1 && \
timeout -k 10 200 python bench.py > gpurun_out/r3base/bench.json 2> gpurun_out/r3base/bench.err && \
timeout -k 10 200 python bench.py --prewarm_ms 0 > gpurun_out/r3base/bench_noprewarm.json 2>> gpurun_out/r3base/bench.err && \
bash bench/gpu_prof.sh r3base/prof_lenet -- --steps 5
